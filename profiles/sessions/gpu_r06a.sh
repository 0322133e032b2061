set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_bench.py -k "rccl or one_rank" > gpurun_out/r06a/rccl_tests.txt 2>&1 && \
timeout -k 10 120 ./tools/probe_last_pass_bin 3 > gpurun_out/r06a/last_pass_ceiling.log 2>&1
