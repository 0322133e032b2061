#!/bin/bash
# tools/gpu_planner_sweep.sh -- the planner's pick against the other pass counts
# and radix orders (tools/tune.py variants), fp32, one-worker plans and one
# worker of an 8-GPU job, over sizes around the configs.
set -o pipefail
mkdir -p gpurun_out
V='[{}, {"PIFFT_ORDER":"0"}, {"PIFFT_ORDER":"1"}, {"PIFFT_PASSES":"3"}, {"PIFFT_PASSES":"4"}]'
for logn in 24 26 28 30; do
  echo "== fp32 2^$logn P=1"
  timeout -k 10 120 python -u tools/tune.py --log-n $logn --prec 32 --steps 5 --warmup 2 --variants "$V" 2>&1 \
      | grep -v amdgpu | grep -v "torch copy" | cut -c1-220 || exit 1
done
for logn in 26 28 30; do
  echo "== fp32 2^$logn worker 7 of P=8"
  timeout -k 10 120 python -u tools/tune.py --log-n $logn --prec 32 --workers 8 --first 7 --count 1 --steps 5 --warmup 2 \
      --variants "$V" 2>&1 | grep -v amdgpu | grep -v "torch copy" | cut -c1-220 || exit 1
done
