# round 6, session b: the whole GPU suite recording the instances its plans
# use (tests/golden/instances_tests.txt), then the per-stage workgroup clocks
# of the latency-bound configs (C1, C2, C2's one-GPU slice)
set -o pipefail
mkdir -p gpurun_out/r06b
export PIFFTTEST_RECORD_INSTANCES=gpurun_out/r06b/instances_tests.txt
timeout -k 10 840 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/r06b/gpu_tests.txt 2>&1 && \
unset PIFFTTEST_RECORD_INSTANCES && \
timeout -k 10 120 python -u tools/wg_clock.py --log-n 20 > gpurun_out/r06b/wgc_c1.txt 2>&1 && \
timeout -k 10 120 python -u tools/wg_clock.py --log-n 20 --workers 8 > gpurun_out/r06b/wgc_c2.txt 2>&1 && \
timeout -k 10 120 python -u tools/wg_clock.py --log-n 20 --workers 8 --count 1 > gpurun_out/r06b/wgc_c2_slice.txt 2>&1
