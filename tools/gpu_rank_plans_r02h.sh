#!/bin/bash
# tools/gpu_rank_plans_r02h.sh -- one rank's plan of the G-GPU split at HEAD
# (padded workspace rows): fp64 2^28 for G = 1, 2, 4, 8 (worker 0 of G) and
# config 5's fp64 2^32 worker 0 of 8; per-launch times by tools/tune.py.
set -o pipefail
mkdir -p gpurun_out/rank
for spec in "28 1" "28 2" "28 4" "28 8" "32 8"; do
  set -- $spec
  echo "== fp64 2^$1, worker 0 of $2"
  timeout -k 10 180 python3 -u tools/tune.py --log-n $1 --workers $2 --first 0 --count 1 --steps 10 --warmup 3 \
      --variants '[{}, {}]' 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/rank/rank_plans.log
