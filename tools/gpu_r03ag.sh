#!/bin/bash
# tools/gpu_r03ag.sh -- round-3 session ag: the new plan's first pass (R = 512,
# reading the input at 256-B row segments) at C = 32 (512-B segments, a
# 16384-value tile, one workgroup of 1024 threads per CU: PIFFT_FIRST_TILE64),
# tuned workspaces, alternating
set -o pipefail
out=gpurun_out/r03ag
mkdir -p "$out"
V='[{}, {"PIFFT_FIRST_TILE64":"16384","PIFFT_RADIX_LOGS":"9,9,10"}, {}, {"PIFFT_FIRST_TILE64":"16384","PIFFT_RADIX_LOGS":"9,9,10"}, {"PIFFT_FIRST_TILE64":"16384"}]'
{ echo "=== fp64 2^28"; timeout -k 10 400 python -u tools/tune.py --log-n 28 --prec 64 --steps 20 --warmup 3 --tune-ws 4 --variants "$V"; } > "$out/first_c32.log" 2>&1 || { tail "$out/first_c32.log"; exit 1; }
grep -E "===|wall" "$out/first_c32.log"
