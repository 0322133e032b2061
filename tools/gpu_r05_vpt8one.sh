#!/bin/bash
# tools/gpu_r05_vpt8one.sh [tag] -- round 5: fp64 P = 2 at 8192 values as one
# fused launch at 8 values per thread (1024 threads; 16 spills) -- the small-plan
# GPU tests, then the A/B against the three launches, single and batched.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05v8}
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "fused_all_worker or single_pass_all_worker or tiny" > "$out/tests.txt" 2>&1 || { tail -40 "$out/tests.txt"; exit 1; }
tail -2 "$out/tests.txt"
V='[{}, {"PIFFT_WIL_ONE_LAUNCH":"0"}, {}, {"PIFFT_WIL_ONE_LAUNCH":"0"}]'
for b in 1 64; do
  echo "=== fp64 2^13 P = 2 batch $b" >> "$out/v8.log"
  timeout -k 10 120 python3 -u tools/tune.py --log-n 13 --prec 64 --workers 2 --batch $b --steps 1000 --warmup 300 --check \
    --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/v8.log" || exit 1
done
echo done
