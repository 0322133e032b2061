# round 6, session t: the stage-twiddle prefetch for single / first passes of
# 256-VGPR tiles (PIFFT_TW_PREFETCH=3: every anchor, bitwise equal by
# construction) -- output hashes of both builds, then A/B timing round robin
set -o pipefail
out=gpurun_out/r06t
mkdir -p $out
for v in base twpre3g; do
  PIFFT_LIB=abvar/$v.so timeout -k 10 120 python tools/bitwise_libs.py --set single > $out/bitwise_$v.txt 2>&1 || exit 1
done
export AB_ROUNDS=3
tools/ab.sh "--log-n 20 --prec 64 --steps 300 --warmup 20" abvar/base.so abvar/twpre3g.so > $out/c1.txt 2>&1 &&
tools/ab.sh "--log-n 12 --prec 32 --batch 4096 --steps 300 --warmup 20" abvar/base.so abvar/twpre3g.so > $out/c3.txt 2>&1 &&
tools/ab.sh "--log-n 12 --prec 32 --batch 512 --steps 300 --warmup 20" abvar/base.so abvar/twpre3g.so > $out/f32_4096x512.txt 2>&1 &&
tools/ab.sh "--log-n 12 --prec 64 --batch 1024 --steps 300 --warmup 20" abvar/base.so abvar/twpre3g.so > $out/f64_4096x1024.txt 2>&1 &&
tools/ab.sh "--log-n 22 --prec 64 --steps 200 --warmup 20" abvar/base.so abvar/twpre3g.so > $out/f64_2e22.txt 2>&1 &&
tools/ab.sh "--log-n 20 --prec 64 --workers 8 --count 1 --steps 300 --warmup 20" abvar/base.so abvar/twpre3g.so > $out/c2_slice.txt 2>&1 &&
AB_ROUNDS=2 tools/ab.sh "--log-n 28 --prec 64 --steps 10 --warmup 3" abvar/base.so abvar/twpre3g.so > $out/c4.txt 2>&1
