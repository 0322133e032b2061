set -o pipefail
for spec in "--log-n 24 --workers 8" "--log-n 28 --workers 8" "--log-n 28 --workers 16" "--log-n 28 --workers 64" "--log-n 20 --workers 8" "--log-n 12 --prec 32 --batch 4096 --workers 4"; do
  echo "== $spec"
  timeout -k 10 120 python -u tools/tune.py $spec --steps 20 --warmup 5 --variants '[{},{}]' | grep wall | sed 's/(sum of launches.*:://' || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tree2_tests.log 2>&1 || { tail -30 gpurun_out/tree2_tests.log; exit 1; }
tail -1 gpurun_out/tree2_tests.log
