#!/bin/bash
# tools/gpu_r03w.sh -- round-3 session w: the small configs' tile widths
# (Infinity-Cache resident, launch/latency-bound): C1 fp64 2^20 at fewer,
# wider workgroups (PIFFT_MIN_WORKGROUPS 256 -> C = 4, 128 -> 8, 64 -> 16);
# C2 (8 interleaved workers) at C = 16 (PIFFT_WIL_CMIN); C3 at 2 lines per
# workgroup (PIFFT_SINGLE_C32)
set -o pipefail
out=gpurun_out/r03w
mkdir -p "$out"
{ echo "=== C1 fp64 2^20"; timeout -k 10 200 python -u tools/tune.py --log-n 20 --prec 64 --steps 100 --warmup 20 --variants '[{}, {"PIFFT_MIN_WORKGROUPS":"128"}, {"PIFFT_MIN_WORKGROUPS":"64"}, {"PIFFT_MIN_WORKGROUPS":"128","PIFFT_NT":"0"}, {}]';
  echo "=== C2 fp64 2^20 P=8"; timeout -k 10 200 python -u tools/tune.py --log-n 20 --prec 64 --workers 8 --steps 100 --warmup 20 --variants '[{}, {"PIFFT_WIL_CMIN":"16"}, {"PIFFT_WIL_CMIN":"4"}, {}]';
  echo "=== C3 fp32 4096 x 4096"; timeout -k 10 200 python -u tools/tune.py --log-n 12 --prec 32 --batch 4096 --steps 50 --warmup 10 --variants '[{}, {"PIFFT_SINGLE_C32":"2"}, {"PIFFT_SINGLE_C32":"4"}, {}]'; } > "$out/small.log" 2>&1 || { tail "$out/small.log"; exit 1; }
grep -E "===|wall" "$out/small.log"
