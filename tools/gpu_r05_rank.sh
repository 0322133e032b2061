#!/bin/bash
# tools/gpu_r05_rank.sh [tag] -- round 5: radix orders of one rank's plan of
# the G-GPU split of fp64 2^28 (worker 0 of G; the fused tree + first pass
# reads all P leaves per input, so its first radix sets the leaf-read segment
# width: R = 512 C = 16 -> 256 B, R = 256 C = 32 -> 512 B, R = 128 C = 64 ->
# 1 KiB), tools/tune.py with bench.py's workspace tuning, two runs each.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05_rank}
mkdir -p "$out"
run() {  # g variants
  echo "== fp64 2^28, worker 0 of $1" >> "$out/rank_orders.log"
  timeout -k 10 240 python3 -u tools/tune.py --log-n 28 --prec 64 --workers $1 --first 0 --count 1 --steps 20 --warmup 5 --tune-ws 4 --variants "$2" 2>&1 | grep -v "amdgpu.ids" >> "$out/rank_orders.log"
}
run 8 '[{}, {"PIFFT_RADIX_LOGS":"8,8,9"}, {"PIFFT_RADIX_LOGS":"8,9,8"}, {"PIFFT_RADIX_LOGS":"7,9,9"}, {"PIFFT_XCD_GROUP":"0"}, {"PIFFT_XCD_GROUP":"3"}, {"PIFFT_XCD_GROUP":"4"}, {}, {"PIFFT_RADIX_LOGS":"8,8,9"}, {"PIFFT_RADIX_LOGS":"7,9,9"}]' || exit 1
run 4 '[{}, {"PIFFT_RADIX_LOGS":"8,9,9"}, {"PIFFT_RADIX_LOGS":"7,9,10"}, {}, {"PIFFT_RADIX_LOGS":"8,9,9"}]' || exit 1
run 2 '[{}, {"PIFFT_RADIX_LOGS":"8,9,10"}, {"PIFFT_RADIX_LOGS":"8,10,9"}, {}, {"PIFFT_RADIX_LOGS":"8,9,10"}]' || exit 1
cat "$out/rank_orders.log"
