#!/bin/bash
# tools/gpu_r03aa.sh -- round-3 session aa: packed VPT-32 fp32 passes with the
# second component's LDS addresses recomputed (PIFFT_PK_REMAT=1: no spill, was
# 52 B / 20 B per lane in the 1024-point MODE 2 / MODE 1 instances) vs kept
# live (0); library variants, tuned workspaces
set -o pipefail
out=gpurun_out/r03aa
mkdir -p "$out"
libs="abvar/remat0.so abvar/remat1.so"
{ AB_ROUNDS=3 bash tools/ab.sh "--log-n 28 --prec 32 --steps 20 --warmup 3 --tune-ws 4" $libs &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 29 --prec 32 --steps 10 --warmup 3 --tune-ws 4" $libs &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 30 --prec 32 --steps 6 --warmup 2 --tune-ws 4" $libs &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 27 --prec 32 --steps 20 --warmup 3 --tune-ws 4" $libs; } > "$out/remat.log" 2>&1 || { tail "$out/remat.log"; exit 1; }
grep -E "==|wall" "$out/remat.log"
