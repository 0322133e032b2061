#!/bin/bash
# tools/gpu_last.sh -- last-pass streaming form and XCD grouping sweep (C4)
set -o pipefail
mkdir -p gpurun_out
V='[{},{"PIFFT_LAST_NT":2},{"PIFFT_LAST_NT":0},{"PIFFT_LAST_NT":3},{"PIFFT_LAST_XCD_GROUP":0},{"PIFFT_LAST_XCD_GROUP":4},{"PIFFT_LAST_XCD_GROUP":6},{"PIFFT_LAST_NT":2,"PIFFT_LAST_XCD_GROUP":4},{}]'
timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 64 --variants "$V" > gpurun_out/last_c4.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/last_c4.log | cut -c1-230
