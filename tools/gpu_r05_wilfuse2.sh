#!/bin/bash
# tools/gpu_r05_wilfuse2.sh [tag] -- round 5, second MODE 11 session: the
# fused all-worker tree pass by J (adjacent line indices per tile: J P lines,
# first radix 8192 / (J P); PIFFT_WIL_FUSE_J) against the separate tree
# launch (PIFFT_WIL_FUSE=0), per shape, two rounds.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05m}
mkdir -p "$out"
V64='[{"PIFFT_WIL_FUSE_J":"4"}, {"PIFFT_WIL_FUSE_J":"8"}, {"PIFFT_WIL_FUSE_J":"16"}, {"PIFFT_WIL_FUSE":"0"}, {"PIFFT_WIL_FUSE_J":"4"}, {"PIFFT_WIL_FUSE_J":"8"}, {"PIFFT_WIL_FUSE_J":"16"}, {"PIFFT_WIL_FUSE":"0"}]'
V32='[{"PIFFT_WIL_FUSE_J":"8"}, {"PIFFT_WIL_FUSE_J":"16"}, {"PIFFT_WIL_FUSE_J":"32"}, {"PIFFT_WIL_FUSE":"0"}, {"PIFFT_WIL_FUSE_J":"8"}, {"PIFFT_WIL_FUSE_J":"16"}, {"PIFFT_WIL_FUSE_J":"32"}, {"PIFFT_WIL_FUSE":"0"}]'
run() {  # variants shape...
  local v="$1"; shift
  echo "=== $*" >> "$out/wilfuse2.log"
  timeout -k 10 300 python3 -u tools/tune.py "$@" --variants "$v" 2>&1 | grep -v amdgpu.ids >> "$out/wilfuse2.log" || { tail -20 "$out/wilfuse2.log"; exit 1; }
}
run "$V64" --log-n 20 --prec 64 --workers 8 --steps 2000 --warmup 500
run "$V64" --log-n 20 --prec 64 --workers 4 --steps 2000 --warmup 500
run "$V64" --log-n 20 --prec 64 --workers 2 --steps 2000 --warmup 500
run "$V64" --log-n 20 --prec 64 --workers 16 --steps 2000 --warmup 500
run "$V64" --log-n 22 --prec 64 --workers 16 --steps 1000 --warmup 200
run "$V64" --log-n 24 --prec 64 --workers 8 --steps 200 --warmup 50
run "$V64" --log-n 26 --prec 64 --workers 4 --steps 50 --warmup 10
run "$V64" --log-n 28 --prec 64 --workers 8 --steps 20 --warmup 5
run "$V64" --log-n 28 --prec 64 --workers 16 --steps 20 --warmup 5
run "$V32" --log-n 20 --prec 32 --workers 8 --steps 2000 --warmup 500
run "$V32" --log-n 24 --prec 32 --workers 8 --steps 200 --warmup 50
run "$V32" --log-n 28 --prec 32 --workers 8 --steps 20 --warmup 5
cat "$out/wilfuse2.log"
