# round 6, session i: a longer seeded fuzz on the pruned library at HEAD
# (random N, P, worker ranges, batches, output orders, both precisions vs the
# oracle; worker-interleaved all-worker plans; large shapes)
set -o pipefail
out=gpurun_out/r06i
mkdir -p $out
FUZZ_COUNT=1200 FUZZ_SEED=606 FUZZ_WIL_COUNT=240 FUZZ_WIL_SEED=6060 FUZZ_LARGE_COUNT=32 FUZZ_LARGE_SEED=60606 \
  timeout -k 10 1000 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fuzz.py > $out/fuzz.txt 2>&1
