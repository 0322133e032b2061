#!/bin/bash
# tools/gpu_r05_wiltile3.sh [tag] -- round 5: the fused all-worker tree pass
# (MODE 11) at the sizes where the default J leaves a remainder of more than
# 2048 points (split into two passes): fp64 2^21-2^23 and fp32 2^21-2^24,
# P = 2..16, J = 4 / 2 at the 8192-value tile and J = 4 / 2 at 4096 against
# the default, each output checked against the default plan's.  Variant
# library: tools/mk_wil_tile_variant.sh.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05u}
mkdir -p "$out"
t() { echo "{\"PIFFT_WIL_FUSE_TILE\":\"$1\",\"PIFFT_WIL_FUSE_J\":\"$2\"}"; }
V="[{}, $(t 8192 4), $(t 8192 2), $(t 4096 4), $(t 4096 2), {\"PIFFT_WIL_FUSE\":\"0\"}, {}, $(t 8192 4), $(t 8192 2)]"
run() {  # prec log_n P
  echo "=== fp$1 2^$2 P = $3" >> "$out/wiltile3.log"
  PIFFT_LIB=abvar2/wiltile.so timeout -k 10 200 python3 -u tools/tune.py --log-n $2 --prec $1 --workers $3 --steps 600 --warmup 200 --check --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/wiltile3.log"
}
for s in "64 21" "64 22" "64 23" "32 21" "32 22" "32 23" "32 24"; do
  for P in 2 4 8 16; do
    run $s $P || exit 1
  done
done
cat "$out/wiltile3.log"
