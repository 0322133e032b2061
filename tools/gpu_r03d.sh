#!/bin/bash
# tools/gpu_r03d.sh -- round-3 session d: C2 with the all-worker fused tree pass
# (now instantiated at C = 8/16), then the whole GPU suite, bench.py and the
# rocprofv3 roofline check (tools/gpu_r03.sh)
set -o pipefail
out=gpurun_out/r03d
mkdir -p "$out"
V2='[{}, {"PIFFT_FUSE_ALL_MAX_MIB":"64"}, {"PIFFT_FUSE_ALL_MAX_MIB":"64","PIFFT_ILV":"0"}, {}, {"PIFFT_FUSE_ALL_MAX_MIB":"64"}]'
{ echo "=== C2 fp64 2^20 P=8"; timeout -k 10 120 python -u tools/tune.py --log-n 20 --prec 64 --workers 8 --steps 50 --warmup 5 --variants "$V2";
  echo "=== fp64 2^21 P=8"; timeout -k 10 120 python -u tools/tune.py --log-n 21 --prec 64 --workers 8 --steps 50 --warmup 5 --variants "$V2";
  echo "=== fp32 2^20 P=8"; timeout -k 10 120 python -u tools/tune.py --log-n 20 --prec 32 --workers 8 --steps 50 --warmup 5 --variants "$V2"; } > "$out/c2_fuse_all.log" 2>&1 || { tail "$out/c2_fuse_all.log"; exit 1; }
grep -E "===|wall" "$out/c2_fuse_all.log" | sed 's/ :: .*//'
bash tools/gpu_r03.sh r03d tests
