#!/bin/bash
# tools/gpu_r04za_rank_plans.sh -- round-4 session za: one rank's plan of the
# G-GPU split of fp64 2^28 (workers 0 and G-1 of G) and config 5's fp64 2^32
# worker 0 of 8 on one MI355X at HEAD (tools/tune.py with bench.py's
# workspace tuning, 2 runs each): the per-GPU time of the driver's 1/2/4/8
# curve before its 8-GPU node measures it.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r04za}
mkdir -p "$out"
for g in 1 2 4 8; do
  for q in 0 $((g - 1)); do
    [ $g -eq 1 ] && [ $q -gt 0 ] && continue
    echo "== fp64 2^28, worker $q of $g" >> "$out/rank_plans.log"
    timeout -k 10 200 python3 -u tools/tune.py --log-n 28 --prec 64 --workers $g --first $q --count 1 --steps 20 --warmup 5 --tune-ws 8 --variants '[{}, {}]' 2>&1 | grep -v "amdgpu.ids" >> "$out/rank_plans.log" || exit 1
  done
done
echo "== fp64 2^32, worker 0 of 8" >> "$out/rank_plans.log"
timeout -k 10 300 python3 -u tools/tune.py --log-n 32 --prec 64 --workers 8 --first 0 --count 1 --steps 10 --warmup 3 --tune-ws 4 --variants '[{}, {}]' 2>&1 | grep -v "amdgpu.ids" >> "$out/rank_plans.log" || exit 1
cat "$out/rank_plans.log"
