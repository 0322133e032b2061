#!/bin/bash
# tools/gpu_r03d.sh -- round-3 session d:
#   1. C2 with the all-worker fused tree pass (now instantiated at C = 8/16)
#   2. the 2^28 plans with two sub-tiles per workgroup (k_pass H = 2)
#   3. the whole GPU suite, bench.py and the rocprofv3 roofline check
set -o pipefail
out=gpurun_out/r03d
mkdir -p "$out"
V2='[{}, {"PIFFT_FUSE_ALL_MAX_MIB":"64"}, {"PIFFT_FUSE_ALL_MAX_MIB":"64","PIFFT_ILV":"0"}, {}, {"PIFFT_FUSE_ALL_MAX_MIB":"64"}]'
{ echo "=== C2 fp64 2^20 P=8"; timeout -k 10 120 python -u tools/tune.py --log-n 20 --prec 64 --workers 8 --steps 50 --warmup 5 --variants "$V2";
  echo "=== fp64 2^21 P=8"; timeout -k 10 120 python -u tools/tune.py --log-n 21 --prec 64 --workers 8 --steps 50 --warmup 5 --variants "$V2";
  echo "=== fp32 2^20 P=8"; timeout -k 10 120 python -u tools/tune.py --log-n 20 --prec 32 --workers 8 --steps 50 --warmup 5 --variants "$V2"; } > "$out/c2_fuse_all.log" 2>&1 || { tail "$out/c2_fuse_all.log"; exit 1; }
grep -E "===|wall" "$out/c2_fuse_all.log" | sed 's/ :: .*//'
V4='[{}, {"PIFFT_SUBTILES_FIRST":"2"}, {"PIFFT_SUBTILES":"2"}, {}, {"PIFFT_SUBTILES_FIRST":"2"}, {"PIFFT_SUBTILES":"2"}]'
V5='[{}, {"PIFFT_PASSES":"3"}, {"PIFFT_PASSES":"3","PIFFT_SUBTILES_FIRST":"2"}, {"PIFFT_PASSES":"3","PIFFT_SUBTILES":"2"}, {}, {"PIFFT_PASSES":"3","PIFFT_SUBTILES":"2"}]'
{ echo "=== C4 fp64 2^28"; timeout -k 10 200 python -u tools/tune.py --log-n 28 --prec 64 --steps 10 --warmup 3 --variants "$V4";
  echo "=== fp32 2^28"; timeout -k 10 200 python -u tools/tune.py --log-n 28 --prec 32 --steps 10 --warmup 3 --variants "$V5"; } > "$out/subtiles.log" 2>&1 || { tail "$out/subtiles.log"; exit 1; }
grep -E "===|wall" "$out/subtiles.log"
bash tools/gpu_r03.sh r03d "tests/test_gpu_fullsize.py::test_subtiled_passes_bitwise_equal tests"
