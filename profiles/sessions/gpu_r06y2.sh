# round 6, session y2: config 2's second pass (k_pass<double,1024,8,10,...>, 128
# workgroups on 256 CUs) built for 2 waves per SIMD (wil1), and with its later
# stages' twiddles fetched with the loads (wil2), against HEAD; bitwise hashes
set -o pipefail
out=gpurun_out/r06y2
mkdir -p $out
for v in base wil2; do
  PIFFT_LIB=abvar/$v.so timeout -k 10 120 python tools/bitwise_libs.py > $out/bitwise_$v.txt 2>&1 || exit 1
done
export AB_ROUNDS=3
tools/ab.sh "--log-n 20 --prec 64 --workers 8 --steps 300 --warmup 20" abvar/base.so abvar/wil1.so abvar/wil2.so > $out/c2.txt 2>&1 &&
tools/ab.sh "--log-n 21 --prec 64 --workers 8 --steps 300 --warmup 20" abvar/base.so abvar/wil1.so abvar/wil2.so > $out/f64_2e21_p8.txt 2>&1 &&
tools/ab.sh "--log-n 24 --prec 64 --workers 8 --steps 100 --warmup 10" abvar/base.so abvar/wil1.so abvar/wil2.so > $out/f64_2e24_p8.txt 2>&1
