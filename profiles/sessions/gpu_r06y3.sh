# round 6, session y3: config 1's streaming form per pass (PIFFT_FIRST_NT /
# PIFFT_LAST_NT: 0 plain, 1 non-temporal loads and stores); round 6 measured
# only both passes plain (r06e_c1_nt.txt)
set -o pipefail
out=gpurun_out/r06y3
mkdir -p $out
V='[{}, {"PIFFT_FIRST_NT":"0"}, {"PIFFT_LAST_NT":"0"}, {"PIFFT_FIRST_NT":"0","PIFFT_LAST_NT":"0"}]'
for r in 1 2 3; do
  PIFFT_TUNING=1 timeout -k 10 120 python tools/tune.py --log-n 20 --prec 64 --steps 300 --warmup 20 --variants "$V" --check >> $out/c1_nt.txt 2>&1 || exit 1
done
for r in 1 2; do
  PIFFT_TUNING=1 timeout -k 10 120 python tools/tune.py --log-n 19 --prec 64 --steps 300 --warmup 20 --variants "$V" >> $out/f64_2e19_nt.txt 2>&1 || exit 1
  PIFFT_TUNING=1 timeout -k 10 120 python tools/tune.py --log-n 21 --prec 64 --steps 300 --warmup 20 --variants "$V" >> $out/f64_2e21_nt.txt 2>&1 || exit 1
done
