#!/bin/bash
# tools/gpu_r03b.sh -- round-3 session b: A/B of the kernel changes (vector nt
# accesses, branch-free tile loads; abvar/r02kern.so = the round-2 kernels
# with this round's ABI) on the configs; fp32 2^28 three-pass variants
# (16384-value tile at 16 values x 1024 threads, or 32 values x 512 threads);
# then the r03 evidence session.
set -o pipefail
out=gpurun_out/r03b
mkdir -p "$out"
for cfg in "--log-n 28 --prec 64" "--log-n 28 --prec 32" "--log-n 20 --prec 64 --steps 50" \
           "--log-n 20 --prec 64 --workers 8 --steps 50" "--log-n 12 --prec 32 --batch 4096 --steps 50"; do
  echo "=== $cfg"
  AB_ROUNDS=2 bash tools/ab.sh "$cfg" abvar/r02kern.so cs87project-msolano2_amd/libpifft.so || exit 1
done > "$out/ab_kernels.log" 2>&1 || { tail -20 "$out/ab_kernels.log"; exit 1; }
grep -E "===|==|wall" "$out/ab_kernels.log"
V='[{}, {"PIFFT_TILE32":"16384","PIFFT_PASSES":"3"}, {"PIFFT_TILE32":"16384","PIFFT_PASSES":"3","PIFFT_VPT32":"1"}, {}]'
timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 32 --steps 10 --warmup 3 --variants "$V" > "$out/fp32_3pass.log" 2>&1 || { tail "$out/fp32_3pass.log"; exit 1; }
grep wall "$out/fp32_3pass.log"
bash tools/gpu_r03.sh r03b tests
