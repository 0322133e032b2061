#!/bin/bash
# tools/gpu_r03l.sh -- round-3 session l: fp32 2^28 / 2^30 packed three-pass
# plans in the three radix orders (which pass carries the 1024-point rows and
# their 128-B segments)
set -o pipefail
out=gpurun_out/r03l
mkdir -p "$out"
V28='[{}, {"PIFFT_RADIX_LOGS":"9,10,9"}, {"PIFFT_RADIX_LOGS":"9,9,10"}, {}, {"PIFFT_RADIX_LOGS":"9,10,9"}, {"PIFFT_RADIX_LOGS":"9,9,10"}]'
V29='[{}, {"PIFFT_RADIX_LOGS":"10,9,10"}, {"PIFFT_RADIX_LOGS":"9,10,10"}, {}]'
{ echo "=== fp32 2^28"; timeout -k 10 200 python -u tools/tune.py --log-n 28 --prec 32 --steps 10 --warmup 3 --variants "$V28";
  echo "=== fp32 2^29"; timeout -k 10 200 python -u tools/tune.py --log-n 29 --prec 32 --steps 10 --warmup 3 --variants "$V29"; } > "$out/order32.log" 2>&1 || { tail "$out/order32.log"; exit 1; }
grep -E "===|wall" "$out/order32.log"
