#!/bin/bash
# tools/gpu_small_sweep.sh -- latency-bound small transforms: config 1 (fp64
# 2^20, one worker) under forced pass decompositions / lines per workgroup,
# and config-3 shares (fp32 4096-point, 512 / 1024 transforms) by lines.
set -o pipefail
mkdir -p gpurun_out/small
V1='[{}, {"PIFFT_RADIX_LOGS":"7,7,6"}, {"PIFFT_RADIX_LOGS":"7,7,6","PIFFT_COL_C64":"8"}, {"PIFFT_RADIX_LOGS":"7,7,6","PIFFT_COL_C64":"4"}, {"PIFFT_RADIX_LOGS":"5,5,5,5"}, {"PIFFT_RADIX_LOGS":"8,6,6"}, {"PIFFT_RADIX_LOGS":"10,10","PIFFT_MIN_WORKGROUPS":"128"}, {"PIFFT_RADIX_LOGS":"9,11"}, {"PIFFT_RADIX_LOGS":"11,9"}, {}]'
V3='[{}, {"PIFFT_SINGLE_C32":"2"}, {"PIFFT_SINGLE_C32":"4"}, {"PIFFT_NT":"1"}, {}]'
{
for ln in 18 19 20 21 22; do
  echo "== fp64 2^$ln P=1"
  timeout -k 10 120 python -u tools/tune.py --log-n $ln --prec 64 --steps 50 --warmup 10 --variants "$V1" || exit 1
done
for b in 512 1024; do
  echo "== fp32 4096 x $b"
  timeout -k 10 120 python -u tools/tune.py --log-n 12 --prec 32 --batch $b --steps 50 --warmup 10 --variants "$V3" || exit 1
done
} > gpurun_out/small/sweep.log 2>&1 || { tail -20 gpurun_out/small/sweep.log; exit 1; }
grep -E "==|wall" gpurun_out/small/sweep.log | sed 's/(sum of launches/(launches/'
