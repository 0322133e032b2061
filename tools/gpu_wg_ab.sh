#!/bin/bash
# tools/gpu_wg_ab.sh -- A/B of PIFFT_MIN_WG_PER_CU builds (launch-bounds
# occupancy target) on C4 and on a small config-3 share.
#   gpurun -- bash tools/gpu_wg_ab.sh variants/base.so variants/wg1.so variants/wg4.so
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 bash tools/ab.sh "--log-n 28 --prec 64" "$@" > gpurun_out/wg_c4.log 2>&1 || exit 1
timeout -k 10 200 bash tools/ab.sh "--log-n 12 --prec 32 --batch 512 --steps 50 --warmup 5" "$@" > gpurun_out/wg_c3.log 2>&1 || exit 1
timeout -k 10 200 bash tools/ab.sh "--log-n 12 --prec 32 --batch 4096 --steps 50 --warmup 5" "$@" >> gpurun_out/wg_c3.log 2>&1 || exit 1
