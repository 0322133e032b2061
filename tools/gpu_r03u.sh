#!/bin/bash
# tools/gpu_r03u.sh -- round-3 session u: fp32 2^28 workspace row pad
# (PIFFT_W_PAD elements: 2080 = 16 KiB + 256 B default, 1056 = 8 KiB + 256 B,
# 4128 = 32 KiB + 256 B), tuned workspaces, three rounds alternating; then the
# evidence session (bench + rocprofv3 check) at HEAD
set -o pipefail
out=gpurun_out/r03u
mkdir -p "$out"
V='[{}, {"PIFFT_W_PAD":"1056"}, {"PIFFT_W_PAD":"4128"}, {}, {"PIFFT_W_PAD":"1056"}, {"PIFFT_W_PAD":"4128"}, {}, {"PIFFT_W_PAD":"1056"}, {"PIFFT_W_PAD":"4128"}]'
{ echo "=== fp32 2^28, tuned workspace (4)"; timeout -k 10 400 python -u tools/tune.py --log-n 28 --prec 32 --steps 20 --warmup 3 --tune-ws 4 --variants "$V"; } > "$out/wpad32.log" 2>&1 || { tail "$out/wpad32.log"; exit 1; }
grep -E "===|wall" "$out/wpad32.log"
bash tools/gpu_r03.sh r03u none
