#!/bin/bash
# tools/gpu_lastc.sh -- last-pass tile width (PIFFT_LAST_C) and streaming form (C4)
set -o pipefail
mkdir -p gpurun_out
V='[{},{"PIFFT_LAST_C":32},{"PIFFT_LAST_C":32,"PIFFT_LAST_NT":0},{"PIFFT_LAST_C":32,"PIFFT_LAST_XCD_GROUP":0},{"PIFFT_LAST_C":8},{},{"PIFFT_LAST_C":32}]'
timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 64 --variants "$V" > gpurun_out/lastc_c4.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/lastc_c4.log | cut -c1-230
