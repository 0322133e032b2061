#!/bin/bash
# tools/gpu_c3_twopass.sh -- config-3 shares (fp32 N=4096): the single-pass
# plan vs forced two-pass plans (PIFFT_SINGLE_MAX_LOG=11 + PIFFT_RADIX_LOGS)
# at several lines per workgroup; 16-128 MiB stays Infinity-Cache resident.
set -o pipefail
mkdir -p gpurun_out
S='"PIFFT_SINGLE_MAX_LOG":"11"'
V="[{}, {$S,\"PIFFT_RADIX_LOGS\":\"6,6\"}, {$S,\"PIFFT_RADIX_LOGS\":\"6,6\",\"PIFFT_COL_C32\":\"8\"}, {$S,\"PIFFT_RADIX_LOGS\":\"6,6\",\"PIFFT_COL_C32\":\"16\"}, {$S,\"PIFFT_RADIX_LOGS\":\"6,6\",\"PIFFT_COL_C32\":\"32\"}, {$S,\"PIFFT_RADIX_LOGS\":\"4,8\"}, {$S,\"PIFFT_RADIX_LOGS\":\"8,4\"}, {}]"
for b in 512 1024 2048 4096; do
  echo "== batch $b"
  timeout -k 10 120 python -u tools/tune.py --log-n 12 --prec 32 --batch $b --steps 50 --warmup 5 --variants "$V" 2>&1 | grep -v amdgpu.ids || exit 1
done
