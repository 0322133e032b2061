#!/bin/bash
# tools/gpu_radix.sh -- explicit radix orders for C4 (PIFFT_RADIX_LOGS)
set -o pipefail
mkdir -p gpurun_out
V='[{},{"PIFFT_RADIX_LOGS":"10,10,8"},{"PIFFT_RADIX_LOGS":"8,10,10"},{"PIFFT_RADIX_LOGS":"9,10,9"},{"PIFFT_RADIX_LOGS":"9,9,10"},{"PIFFT_RADIX_LOGS":"7,7,7,7"},{}]'
timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 64 --variants "$V" > gpurun_out/radix_c4.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/radix_c4.log | cut -c1-230
