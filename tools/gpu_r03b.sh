#!/bin/bash
# tools/gpu_r03b.sh -- round-3 session b: A/B of the kernel changes (vector nt
# accesses, branch-free tile loads; abvar/r02kern.so = the round-2 kernels
# with this round's ABI) on the configs, then the r03 evidence session.
set -o pipefail
out=gpurun_out/r03b
mkdir -p "$out"
for cfg in "--log-n 28 --prec 64" "--log-n 28 --prec 32" "--log-n 20 --prec 64 --steps 50" \
           "--log-n 20 --prec 64 --workers 8 --steps 50" "--log-n 12 --prec 32 --batch 4096 --steps 50"; do
  echo "=== $cfg"
  AB_ROUNDS=2 bash tools/ab.sh "$cfg" abvar/r02kern.so cs87project-msolano2_amd/libpifft.so || exit 1
done > "$out/ab_kernels.log" 2>&1 || { tail -20 "$out/ab_kernels.log"; exit 1; }
grep -E "===|==|wall" "$out/ab_kernels.log"
bash tools/gpu_r03.sh r03b tests
