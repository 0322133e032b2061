#!/bin/bash
# tools/gpu_r03o.sh -- round-3 session o: config 2's one-GPU slice (fp64 2^20,
# worker 0 of 8; the per-GPU work of C2 split over 8 GPUs): the fused tree +
# first pass runs 64 workgroups at R = 512, C = 4.  Radix orders / pass counts
# that give the fused pass more workgroups.
set -o pipefail
out=gpurun_out/r03o
mkdir -p "$out"
V='[{}, {"PIFFT_RADIX_LOGS":"8,9"}, {"PIFFT_RADIX_LOGS":"6,6,5"}, {"PIFFT_RADIX_LOGS":"5,6,6"}, {"PIFFT_RADIX_LOGS":"7,5,5"}, {"PIFFT_STRIDED_CMIN":"2"}, {"PIFFT_RADIX_LOGS":"8,9","PIFFT_STRIDED_CMIN":"2"}, {}]'
{ echo "=== fp64 2^20 worker 0 of 8"; timeout -k 10 200 python -u tools/tune.py --log-n 20 --prec 64 --workers 8 --count 1 --steps 50 --warmup 10 --variants "$V";
  echo "=== fp64 2^20 worker 5 of 8"; timeout -k 10 200 python -u tools/tune.py --log-n 20 --prec 64 --workers 8 --first 5 --count 1 --steps 50 --warmup 10 --variants "$V";
  echo "=== fp64 2^24 worker 0 of 8"; timeout -k 10 200 python -u tools/tune.py --log-n 24 --prec 64 --workers 8 --count 1 --steps 20 --warmup 5 --variants '[{}, {"PIFFT_RADIX_LOGS":"10,11"}, {"PIFFT_RADIX_LOGS":"7,7,7"}, {}]'; } > "$out/c2_slice.log" 2>&1 || { tail "$out/c2_slice.log"; exit 1; }
grep -E "===|wall" "$out/c2_slice.log"
