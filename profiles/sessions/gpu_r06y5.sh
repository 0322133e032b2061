# round 6, session y5: the stage-twiddle prefetch extended to the fused tree
# passes (MODE 3 / 11) of 256-VGPR tiles (PIFFT_TW_PREFETCH_TREE=1; exact
# anchors, so bitwise equal) against HEAD: hashes, then A/B round robin
set -o pipefail
out=gpurun_out/r06y5
mkdir -p $out
for v in base twtree; do
  PIFFT_LIB=abvar/$v.so timeout -k 10 120 python tools/bitwise_libs.py > $out/bitwise_$v.txt 2>&1 || exit 1
done
export AB_ROUNDS=3
tools/ab.sh "--log-n 20 --prec 64 --workers 8 --steps 300 --warmup 20" abvar/base.so abvar/twtree.so > $out/c2.txt 2>&1 &&
tools/ab.sh "--log-n 20 --prec 64 --workers 8 --count 1 --steps 300 --warmup 20" abvar/base.so abvar/twtree.so > $out/c2_slice.txt 2>&1 &&
tools/ab.sh "--log-n 20 --prec 64 --workers 4 --steps 300 --warmup 20" abvar/base.so abvar/twtree.so > $out/f64_2e20_p4.txt 2>&1 &&
tools/ab.sh "--log-n 22 --prec 64 --workers 8 --steps 200 --warmup 20" abvar/base.so abvar/twtree.so > $out/f64_2e22_p8.txt 2>&1 &&
tools/ab.sh "--log-n 20 --prec 32 --workers 8 --steps 300 --warmup 20" abvar/base.so abvar/twtree.so > $out/f32_2e20_p8.txt 2>&1
