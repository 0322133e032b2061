#!/bin/bash
# tools/gpu_r03p.sh -- round-3 session p: radix order of the fp64 three-pass
# plans (fp32 packed plans measured best with the 1024-point pass last,
# profiles/r03_fp32_radix_order.log): 2^28 / 2^29 / 2^30, each order twice
set -o pipefail
out=gpurun_out/r03p
mkdir -p "$out"
V28='[{}, {"PIFFT_RADIX_LOGS":"9,10,9"}, {"PIFFT_RADIX_LOGS":"9,9,10"}, {}, {"PIFFT_RADIX_LOGS":"9,10,9"}, {"PIFFT_RADIX_LOGS":"9,9,10"}]'
V29='[{}, {"PIFFT_RADIX_LOGS":"10,9,10"}, {"PIFFT_RADIX_LOGS":"9,10,10"}, {"PIFFT_RADIX_LOGS":"10,10,9"}, {}, {"PIFFT_RADIX_LOGS":"10,9,10"}, {"PIFFT_RADIX_LOGS":"9,10,10"}, {"PIFFT_RADIX_LOGS":"10,10,9"}]'
V30='[{}, {"PIFFT_RADIX_LOGS":"10,10,10"}, {}]'
{ echo "=== fp64 2^28"; timeout -k 10 200 python -u tools/tune.py --log-n 28 --prec 64 --steps 10 --warmup 3 --variants "$V28";
  echo "=== fp64 2^29"; timeout -k 10 200 python -u tools/tune.py --log-n 29 --prec 64 --steps 10 --warmup 3 --variants "$V29";
  echo "=== fp64 2^30"; timeout -k 10 200 python -u tools/tune.py --log-n 30 --prec 64 --steps 6 --warmup 2 --variants "$V30";
  echo "=== fp32 2^27"; timeout -k 10 200 python -u tools/tune.py --log-n 27 --prec 32 --steps 10 --warmup 3 --variants '[{}, {"PIFFT_VPT32":"0"}, {}]'; } > "$out/order64.log" 2>&1 || { tail "$out/order64.log"; exit 1; }
grep -E "===|wall" "$out/order64.log"
