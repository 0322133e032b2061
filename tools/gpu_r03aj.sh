#!/bin/bash
# tools/gpu_r03aj.sh -- round-3 session aj: config 2 (fp64 2^20, all 8 workers
# on one GPU, worker-interleaved) in other radix orders of its 2^17-point local
# FFT
set -o pipefail
out=gpurun_out/r03aj
mkdir -p "$out"
V='[{}, {"PIFFT_RADIX_LOGS":"8,9"}, {"PIFFT_RADIX_LOGS":"10,7"}, {"PIFFT_RADIX_LOGS":"7,10"}, {}, {"PIFFT_RADIX_LOGS":"8,9"}]'
{ echo "=== C2 fp64 2^20 P=8"; timeout -k 10 200 python -u tools/tune.py --log-n 20 --prec 64 --workers 8 --steps 300 --warmup 30 --variants "$V";
  echo "=== fp32 2^20 P=8"; timeout -k 10 200 python -u tools/tune.py --log-n 20 --prec 32 --workers 8 --steps 300 --warmup 30 --variants "$V"; } > "$out/c2_orders.log" 2>&1 || { tail "$out/c2_orders.log"; exit 1; }
grep -E "===|wall" "$out/c2_orders.log"
