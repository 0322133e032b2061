set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02b/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r02b/gpu_tests.log; exit 1; }
tail -2 gpurun_out/r02b/gpu_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r02b/bench.log 2>&1 || { tail -20 gpurun_out/r02b/bench.log; exit 1; }
grep '^{' gpurun_out/r02b/bench.log > gpurun_out/r02b/bench.json
bash tools/gpu_lds_pmc.sh
