#!/bin/bash
# tools/gpu_r05_batchone.sh [tag] -- round 5: batched all-worker transforms of
# P M <= 8192 values as one fused launch (one workgroup per transform) against
# the previous plans (tree + pass + natural store / interleave:
# PIFFT_WIL_ONE_LAUNCH=0), outputs checked against each other.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05bo}
mkdir -p "$out"
V='[{}, {"PIFFT_WIL_ONE_LAUNCH":"0"}, {}, {"PIFFT_WIL_ONE_LAUNCH":"0"}]'
for s in "32 12 4 4096" "64 12 4 1024" "32 13 8 64" "64 10 16 16" "64 12 32 256" "64 12 8 2" "32 10 2 4096" "64 13 4 512" "32 12 16 8" "64 11 8 4096"; do
  set -- $s
  echo "=== fp$1 2^$2 P = $3 batch $4" >> "$out/batchone.log"
  timeout -k 10 120 python3 -u tools/tune.py --log-n $2 --prec $1 --workers $3 --batch $4 --steps 500 --warmup 100 --check \
    --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/batchone.log" || exit 1
done
echo done
