#!/bin/bash
# tools/gpu_r03t.sh -- round-3 session t: the new 512-512-1024 plan's workspace
# row pad (PIFFT_W_PAD elements; default 16 KiB + 256 B) now that the padded
# hand-off is pass 2 -> pass 3 with 1024 rows 4 MiB apart; tuned workspaces
# (4 placements, losers held so every try is new); and 8 placements
set -o pipefail
out=gpurun_out/r03t
mkdir -p "$out"
V='[{}, {"PIFFT_W_PAD":"0"}, {"PIFFT_W_PAD":"16"}, {"PIFFT_W_PAD":"528"}, {"PIFFT_W_PAD":"1048"}, {"PIFFT_W_PAD":"2064"}, {"PIFFT_W_PAD":"4112"}, {}]'
V32='[{}, {"PIFFT_W_PAD":"0"}, {"PIFFT_W_PAD":"32"}, {"PIFFT_W_PAD":"1056"}, {"PIFFT_W_PAD":"2096"}, {"PIFFT_W_PAD":"4128"}, {}]'
{ echo "=== fp64 2^28, tuned workspace (4)"; timeout -k 10 400 python -u tools/tune.py --log-n 28 --prec 64 --steps 20 --warmup 3 --tune-ws 4 --variants "$V";
  echo "=== fp32 2^28, tuned workspace (4)"; timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 32 --steps 20 --warmup 3 --tune-ws 4 --variants "$V32";
  echo "=== fp64 2^28, tuned workspace (8)"; timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 64 --steps 20 --warmup 3 --tune-ws 8 --variants '[{}, {}, {}]'; } > "$out/wpad.log" 2>&1 || { tail "$out/wpad.log"; exit 1; }
grep -E "===|wall" "$out/wpad.log"
