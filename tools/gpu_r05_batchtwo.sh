#!/bin/bash
# tools/gpu_r05_batchtwo.sh [tag] -- round 5: batched all-worker transforms
# whose local FFT is one pass but too long for one launch: the two-pass
# worker-interleaved plan with the fused tree (PIFFT_WIL_SINGLE_BATCH=1)
# against tree + pass (+ interleave), outputs checked against each other.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05bt}
mkdir -p "$out"
V='[{}, {"PIFFT_WIL_SINGLE_BATCH":"1"}, {}, {"PIFFT_WIL_SINGLE_BATCH":"1"}]'
for s in "64 14 2 16" "64 15 4 8" "64 16 8 4" "32 15 4 64" "32 14 8 32" "32 17 16 2" "64 14 2 256" "64 17 8 16" "32 16 4 256" "64 13 2 64"; do
  set -- $s
  echo "=== fp$1 2^$2 P = $3 batch $4" >> "$out/batchtwo.log"
  timeout -k 10 120 python3 -u tools/tune.py --log-n $2 --prec $1 --workers $3 --batch $4 --steps 500 --warmup 100 --check \
    --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/batchtwo.log" || exit 1
done
echo done
