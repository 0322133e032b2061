#!/bin/bash
# tools/gpu_wpad_shapes.sh -- padded workspace rows (PIFFT_W_PAD) vs none on
# other plan shapes than C4: the worker plans of the 2- and 8-GPU jobs at
# 2^28, an 8-way worker at 2^30, and one-worker plans at 2^25 / 2^26 fp64.
set -o pipefail
mkdir -p gpurun_out/place
o=gpurun_out/place/probe_wpad_shapes.log
: > $o
for spec in "28 2" "28 8" "30 8" "25 1" "26 1"; do
  set -- $spec
  echo "== fp64 2^$1, worker 0 of P=$2" >> $o
  PROBE_LOG_N=$1 PROBE_P=$2 PROBE_TRIALS=5 PROBE_PADS=0,1040 timeout -k 10 200 python3 -u tools/probe_wpad.py 2>&1 | grep -v amdgpu.ids >> $o || exit 1
done
cat $o
