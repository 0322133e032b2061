#!/bin/bash
# tools/gpu_r05_rank2.sh [tag] -- round 5, second rank-plan session: r05c
# (profiles/r05c_rank_orders.log) found WIDER leaf segments slower for the
# fused tree + first pass (R = 256 / C = 32: 0.90 ms, R = 128 / C = 64: 0.94
# vs R = 512 / C = 16: 0.82 at G = 8).  This tries the other direction:
# narrower segments / more rows in flight -- R = 1024 first (C = 8, 128 B) and
# R = 512 at the 4096-value tile (C = 8, twice the workgroups) -- per G, and
# the 4096 first-pass tile on the one-GPU plan.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05d}
mkdir -p "$out"
run() {  # g variants
  echo "== fp64 2^28, worker 0 of $1" >> "$out/rank_orders2.log"
  timeout -k 10 240 python3 -u tools/tune.py --log-n 28 --prec 64 --workers $1 --first 0 --count 1 --steps 20 --warmup 5 --tune-ws 4 --variants "$2" 2>&1 | grep -v "amdgpu.ids" >> "$out/rank_orders2.log"
}
run 8 '[{}, {"PIFFT_FIRST_TILE64":"4096"}, {"PIFFT_RADIX_LOGS":"10,8,7"}, {"PIFFT_RADIX_LOGS":"10,7,8"}, {}, {"PIFFT_FIRST_TILE64":"4096"}, {"PIFFT_RADIX_LOGS":"10,8,7"}]' || exit 1
run 4 '[{}, {"PIFFT_FIRST_TILE64":"4096"}, {"PIFFT_RADIX_LOGS":"10,8,8"}, {}, {"PIFFT_FIRST_TILE64":"4096"}, {"PIFFT_RADIX_LOGS":"10,8,8"}]' || exit 1
run 2 '[{}, {"PIFFT_FIRST_TILE64":"4096"}, {"PIFFT_RADIX_LOGS":"10,9,8"}, {}, {"PIFFT_FIRST_TILE64":"4096"}, {"PIFFT_RADIX_LOGS":"10,9,8"}]' || exit 1
run 1 '[{}, {"PIFFT_FIRST_TILE64":"4096"}, {}, {"PIFFT_FIRST_TILE64":"4096"}]' || exit 1
cat "$out/rank_orders2.log"
