#!/bin/bash
# tools/gpu_r05_wiltile2.sh [tag] -- round 5: the fused all-worker tree pass
# (MODE 11) tile by size: fp64 4096 (J = 2, 4, 8) and 2048 (J = 2, 4) against
# the default 8192, fp32 8192 (J = 4, 8) and 4096 (J = 4) against the default
# 16384, over 2^18-2^22 and P = 2..16, every output checked against the
# default plan's (tools/tune.py --check).  Variant library:
# tools/mk_wil_tile_variant.sh.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05t}
mkdir -p "$out"
t() { echo "{\"PIFFT_WIL_FUSE_TILE\":\"$1\",\"PIFFT_WIL_FUSE_J\":\"$2\"}"; }
V64="[{}, $(t 4096 4), $(t 4096 2), $(t 4096 8), $(t 2048 2), $(t 2048 4), {\"PIFFT_WIL_FUSE\":\"0\"}, {}, $(t 4096 4)]"
V32="[{}, $(t 8192 8), $(t 8192 4), $(t 4096 4), {\"PIFFT_WIL_FUSE\":\"0\"}, {}, $(t 8192 8), $(t 8192 4)]"
run() {  # prec log_n P
  local V="$V64"; [ $1 = 32 ] && V="$V32"
  echo "=== fp$1 2^$2 P = $3" >> "$out/wiltile2.log"
  PIFFT_LIB=abvar2/wiltile.so timeout -k 10 200 python3 -u tools/tune.py --log-n $2 --prec $1 --workers $3 --steps 1000 --warmup 300 --check --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/wiltile2.log"
}
for s in "64 18 8" "64 19 8" "64 19 4" "64 20 16" "64 21 8" "64 21 4" "64 21 2" "64 22 8" "64 22 16" \
         "32 19 8" "32 20 8" "32 20 4" "32 20 2" "32 21 8" "32 22 8" "32 20 16"; do
  run $s || exit 1
done
cat "$out/wiltile2.log"
