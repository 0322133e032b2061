#!/bin/bash
# tools/gpu_r05_tiny2.sh [tag] -- round 5: the edges of the small all-worker
# rules: one launch up to 16384 values (PIFFT_WIL_ONE_MAX; 1024-thread tiles
# where spill-free) and the two-pass plan from M = 2^11 (PIFFT_WIL_SINGLE_MIN_LOG)
# against the defaults, outputs checked against each other.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05za}
mkdir -p "$out"
V='[{}, {"PIFFT_WIL_ONE_MAX":"16384"}, {"PIFFT_WIL_SINGLE_MIN_LOG":"11"}, {"PIFFT_WIL_ONE_LAUNCH":"0"}, {}, {"PIFFT_WIL_ONE_MAX":"16384"}, {"PIFFT_WIL_SINGLE_MIN_LOG":"11"}]'
for s in "32 13 2" "64 13 2" "64 14 4" "32 14 4" "64 14 8" "32 14 8" "64 14 16" "32 14 16" "64 15 8" "64 15 16" "32 15 16" "64 16 16"; do
  set -- $s
  echo "=== fp$1 2^$2 P = $3" >> "$out/tiny2.log"
  timeout -k 10 120 python3 -u tools/tune.py --log-n $2 --prec $1 --workers $3 --steps 2000 --warmup 500 --check \
    --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/tiny2.log" || exit 1
done
echo done
