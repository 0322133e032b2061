# round 6, session x3: the longer seeded fuzz again after the fused-pass prefetch (new seeds)
# (random N, P, worker ranges, batches, output orders, both precisions vs the
# oracle; worker-interleaved all-worker plans; large shapes)
set -o pipefail
out=gpurun_out/r06x3
mkdir -p $out
FUZZ_COUNT=3000 FUZZ_SEED=909 FUZZ_WIL_COUNT=600 FUZZ_WIL_SEED=9090 FUZZ_LARGE_COUNT=64 FUZZ_LARGE_SEED=90909 \
  timeout -k 10 1000 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fuzz.py > $out/fuzz.txt 2>&1
