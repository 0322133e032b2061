set -o pipefail
mkdir -p gpurun_out
V='[{}, {"PIFFT_RADIX_LOGS":"6,6"}, {"PIFFT_RADIX_LOGS":"5,7"}, {"PIFFT_RADIX_LOGS":"7,5"}, {"PIFFT_RADIX_LOGS":"4,8"}, {"PIFFT_RADIX_LOGS":"8,4"}]'
for b in 512 1024 4096; do
  echo "== batch $b"
  timeout -k 10 120 python -u tools/tune.py --log-n 12 --prec 32 --batch $b --steps 50 --warmup 5 --variants "$V" 2>&1 || exit 1
done
