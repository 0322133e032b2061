#!/bin/bash
# tools/gpu_r03m.sh -- round-3 session m: the evidence session at HEAD
# (tools/gpu_r03.sh: GPU tests, bench, rocprofv3 check), then the A/B of the
# tree's twiddle table: packed by level vs one N/2 table (C2: fp64 2^20 P=8
# all workers; fp32 the same; fp64 2^22 P=16)
set -o pipefail
bash tools/gpu_r03.sh r03m || exit 1
out=gpurun_out/r03m
{ AB_ROUNDS=2 bash tools/ab.sh "--log-n 20 --prec 64 --workers 8 --steps 50 --warmup 10" abvar/tree_old.so abvar/tree_packed.so &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 20 --prec 32 --workers 8 --steps 50 --warmup 10" abvar/tree_old.so abvar/tree_packed.so &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 22 --prec 64 --workers 16 --steps 30 --warmup 5" abvar/tree_old.so abvar/tree_packed.so; } > "$out/tree_table_ab.log" 2>&1 || { tail "$out/tree_table_ab.log"; exit 1; }
grep -E "==|wall" "$out/tree_table_ab.log"
