set -o pipefail
for spec in "--log-n 12 --prec 32 --batch 512 --steps 50 --warmup 10" "--log-n 12 --prec 32 --batch 1024 --steps 50 --warmup 10" "--log-n 12 --prec 32 --batch 4096 --steps 30 --warmup 5" "--log-n 20 --prec 64 --steps 50 --warmup 10" "--log-n 20 --prec 64 --workers 8 --steps 50 --warmup 10" "--log-n 13 --prec 64 --batch 64 --steps 50 --warmup 10" "--log-n 28 --prec 64 --steps 10 --warmup 3" "--log-n 28 --prec 64 --workers 8 --count 1 --steps 10 --warmup 3"; do
  echo "#### $spec"
  AB_ROUNDS=2 bash tools/ab.sh "$spec" abvar/twp0.so abvar/twp1.so abvar/twp2.so | grep -E "==|wall" | sed 's/(sum of launches.*//' || exit 1
done
