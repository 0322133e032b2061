#!/bin/bash
# tools/gpu_r03c.sh -- round-3 session c:
#   1. which kernel change moved fp64 C4 (+1.5 %) and fp32 (-5 %): round-2
#      kernels vs vector nt accesses / clamped loads per precision
#   2. C1 at C = 2 (two workgroups per CU); C2 variants (all-worker fused tree,
#      interleave launch instead of the natural-order store)
#   3. tools/probe_p1: read-only / write-only / direct-to-LDS forms of the C4
#      first pass (verdict item 7)
#   4. the bench contract tests, bench.py and the rocprofv3 roofline check
set -o pipefail
out=gpurun_out/r03c
mkdir -p "$out"
for cfg in "--log-n 28 --prec 64" "--log-n 28 --prec 32"; do
  echo "=== $cfg"
  AB_ROUNDS=2 bash tools/ab.sh "$cfg" abvar/r02kern.so abvar/vecnt2.so abvar/clamp2.so cs87project-msolano2_amd/libpifft.so || exit 1
done > "$out/ab_kernels.log" 2>&1 || { tail -20 "$out/ab_kernels.log"; exit 1; }
grep -E "===|==|wall" "$out/ab_kernels.log" | sed 's/ :: .*//'
V1='[{}, {"PIFFT_STRIDED_CMIN":"2"}, {}, {"PIFFT_STRIDED_CMIN":"2"}]'
V2='[{}, {"PIFFT_FUSE_ALL_MAX_MIB":"64"}, {"PIFFT_ILV":"0"}, {"PIFFT_ILV":"0","PIFFT_INTERLEAVE_TILE_MIN64":"1"}, {"PIFFT_STRIDED_CMIN":"2"}, {"PIFFT_FUSE_ALL_MAX_MIB":"64","PIFFT_ILV":"0"}, {}]'
{ echo "=== C1"; timeout -k 10 120 python -u tools/tune.py --log-n 20 --prec 64 --steps 50 --warmup 5 --variants "$V1";
  echo "=== C2"; timeout -k 10 120 python -u tools/tune.py --log-n 20 --prec 64 --workers 8 --steps 50 --warmup 5 --variants "$V2"; } > "$out/small.log" 2>&1 || { tail "$out/small.log"; exit 1; }
grep -E "===|wall" "$out/small.log"
timeout -k 10 120 ./tools/probe_p1 > "$out/probe_p1.log" 2>&1 || { cat "$out/probe_p1.log"; exit 1; }
cat "$out/probe_p1.log"
bash tools/gpu_r03.sh r03c tests/test_bench.py
