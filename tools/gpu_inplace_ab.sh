#!/bin/bash
# (PIFFT_INPLACE_LAST was an A/B knob, removed after this measurement -- profiles/r02_wpad.log; the
# script is kept as the record of how the numbers were taken.)
# tools/gpu_inplace_ab.sh -- A/B of the last pass in place (PIFFT_INPLACE_LAST):
# C4 over fresh (W, y) pairs, then the small plans (C1 2^20, 2^22, C2 slice).
set -o pipefail
mkdir -p gpurun_out/ip
PROBE_TRIALS=7 PROBE_PADS=1040,1040ip,0ip timeout -k 10 300 python3 -u tools/probe_wpad.py 2>&1 | grep -v amdgpu.ids > gpurun_out/ip/c4.log || exit 1
cat gpurun_out/ip/c4.log
V='[{}, {"PIFFT_INPLACE_LAST": "1"}, {}, {"PIFFT_INPLACE_LAST": "1"}]'
for spec in "20 1 0 1" "22 1 0 1" "20 8 0 1" "24 1 0 1"; do
  set -- $spec
  echo "== fp64 2^$1 P=$2 first $3 count $4"
  timeout -k 10 120 python3 -u tools/tune.py --log-n $1 --workers $2 --first $3 --count $4 --steps 200 --warmup 20 --variants "$V" 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/ip/small.log
