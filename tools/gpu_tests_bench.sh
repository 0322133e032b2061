set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { tail -20 gpurun_out/full_tests.log; exit 1; }
tail -3 gpurun_out/full_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_head.log 2>&1 || exit 1
tail -1 gpurun_out/bench_head.log
