set -o pipefail
V='[{}, {"PIFFT_COL_C64":"16"}, {"PIFFT_RADIX_LOGS":"9,8,8","PIFFT_COL_C64":"16"}, {"PIFFT_RADIX_LOGS":"8,9,8"}, {"PIFFT_RADIX_LOGS":"9,9,7"}, {"PIFFT_RADIX_LOGS":"9,7,9"}, {}]'
for w in 8 4 2; do
echo "== 2^28 worker 0 of $w"
timeout -k 10 120 python -u tools/tune.py --log-n 28 --prec 64 --workers $w --count 1 --steps 10 --warmup 3 --variants "$V" || exit 1
done
