#!/bin/bash
# tools/gpu_r05_wiltile.sh [tag] -- round 5: the fused all-worker tree pass
# (MODE 11) at a 4096-value tile (256 workgroups for 2^20 values instead of
# 128 on 256 CUs), J = 4 / 8, 16 or 8 values per thread, and the remaining
# 1024-point pass at 4 lines (PIFFT_WIL_CMIN=4), against the default plan, for
# fp64 2^20 P = 8 (config 2), 4, 2 -- each variant's output checked against
# the default plan's (tools/tune.py --check).  Variant library:
# tools/mk_wil_tile_variant.sh.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05s}
mkdir -p "$out"
V='[{}, {"PIFFT_WIL_CMIN":"4"},
 {"PIFFT_WIL_FUSE_TILE":"4096","PIFFT_WIL_FUSE_J":"4"},
 {"PIFFT_WIL_FUSE_TILE":"4096","PIFFT_WIL_FUSE_J":"4","PIFFT_WIL_CMIN":"4"},
 {"PIFFT_WIL_FUSE_TILE":"4096","PIFFT_WIL_FUSE_J":"4","PIFFT_WIL_FUSE_VPT":"8"},
 {"PIFFT_WIL_FUSE_TILE":"4096","PIFFT_WIL_FUSE_J":"4","PIFFT_WIL_FUSE_VPT":"8","PIFFT_WIL_CMIN":"4"},
 {"PIFFT_WIL_FUSE_TILE":"4096","PIFFT_WIL_FUSE_J":"8"},
 {"PIFFT_WIL_FUSE":"0"}, {},
 {"PIFFT_WIL_FUSE_TILE":"4096","PIFFT_WIL_FUSE_J":"4"},
 {"PIFFT_WIL_FUSE_TILE":"4096","PIFFT_WIL_FUSE_J":"4","PIFFT_WIL_CMIN":"4"},
 {"PIFFT_WIL_FUSE_TILE":"4096","PIFFT_WIL_FUSE_J":"4","PIFFT_WIL_FUSE_VPT":"8","PIFFT_WIL_CMIN":"4"}]'
for P in 8 4 2; do
  echo "=== fp64 2^20 P = $P" >> "$out/wiltile.log"
  PIFFT_LIB=abvar2/wiltile.so timeout -k 10 240 python3 -u tools/tune.py --log-n 20 --prec 64 --workers $P --steps 2000 --warmup 500 --check --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/wiltile.log" || exit 1
done
cat "$out/wiltile.log"
