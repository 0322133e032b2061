#!/bin/bash
# tools/gpu_r03ad.sh -- round-3 session ad: the radix-4 cross-lane last stage
# (v_permlane32_swap + v_permlane16_swap instead of an LDS exchange) in the
# 1024-point FIRST pass (PIFFT_PERMLANE=3): off since round 1 because it
# spilled; the instance now compiles spill-free (123 VGPRs, LDS ops 128 -> 64).
# Config 1 (fp64 2^20: 1024 x 1024, first pass C = 4) and fp32 2^20
set -o pipefail
out=gpurun_out/r03ad
mkdir -p "$out"
libs="abvar/perm1.so abvar/perm3.so"
{ AB_ROUNDS=3 bash tools/ab.sh "--log-n 20 --prec 64 --steps 200 --warmup 20" $libs &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 20 --prec 32 --steps 200 --warmup 20" $libs &&
  AB_ROUNDS=1 bash tools/ab.sh "--log-n 24 --prec 64 --steps 50 --warmup 10 --variants [{\"PIFFT_RADIX_LOGS\":\"10,7,7\"}]" $libs; } > "$out/perm.log" 2>&1 || { tail "$out/perm.log"; exit 1; }
grep -E "==|wall" "$out/perm.log"
