#!/bin/bash
# tools/gpu_r03y.sh -- round-3 session y: leaf loads in flight in the fused
# tree + first pass for small tiles (<= 256 threads; PIFFT_TREE_LOADS_SMALL
# 8 = round 2, 16, 32): config 2's one-GPU slice and other one-worker plans
set -o pipefail
out=gpurun_out/r03y
mkdir -p "$out"
libs="abvar/tl8.so abvar/tl16.so abvar/tl32.so"
{ AB_ROUNDS=2 bash tools/ab.sh "--log-n 20 --prec 64 --workers 8 --count 1 --steps 100 --warmup 20" $libs &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 20 --prec 64 --workers 8 --first 5 --count 1 --steps 100 --warmup 20" $libs &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 20 --prec 32 --workers 8 --count 1 --steps 100 --warmup 20" $libs &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 22 --prec 64 --workers 8 --count 1 --steps 50 --warmup 10" $libs &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 24 --prec 64 --workers 8 --count 1 --steps 30 --warmup 5" $libs &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 20 --prec 64 --workers 16 --count 1 --steps 100 --warmup 20" $libs &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 28 --prec 64 --workers 8 --count 1 --steps 10 --warmup 3" $libs; } > "$out/tree_loads.log" 2>&1 || { tail "$out/tree_loads.log"; exit 1; }
grep -E "==|wall" "$out/tree_loads.log"
