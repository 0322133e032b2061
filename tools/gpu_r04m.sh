#!/bin/bash
# tools/gpu_r04m.sh -- round-4 session m: config 1 (fp64 2^20, one worker)
# plan forms -- lines per workgroup 8 / 16 (128-B / 256-B segments, 128 / 64
# workgroups), radix splits 512 x 2048 / 2048 x 512, streaming forms, XCD
# grouping -- A/B in one process, twice.  (PIFFT_COL_C64 alone is undone
# by the >= 512-workgroup rule: `gpu_r04m.sh 2` pairs it with
# PIFFT_MIN_WORKGROUPS, and splits the XCD grouping by pass.)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04m
mkdir -p "$out"
V2='[{}, {"PIFFT_XCD_GROUP":"0","PIFFT_LAST_XCD_GROUP":"2"}, {"PIFFT_XCD_GROUP":"1","PIFFT_LAST_XCD_GROUP":"2"}, {"PIFFT_XCD_GROUP":"3","PIFFT_LAST_XCD_GROUP":"2"}, {"PIFFT_LAST_XCD_GROUP":"1"}, {"PIFFT_LAST_XCD_GROUP":"3"}, {"PIFFT_COL_C64":"8","PIFFT_MIN_WORKGROUPS":"64"}, {"PIFFT_COL_C64":"16","PIFFT_MIN_WORKGROUPS":"32"}, {}, {"PIFFT_XCD_GROUP":"0","PIFFT_LAST_XCD_GROUP":"2"}, {"PIFFT_XCD_GROUP":"1","PIFFT_LAST_XCD_GROUP":"2"}, {"PIFFT_LAST_XCD_GROUP":"1"}, {"PIFFT_LAST_XCD_GROUP":"3"}, {"PIFFT_COL_C64":"8","PIFFT_MIN_WORKGROUPS":"64"}]'
if [ "${1:-}" = "2" ]; then
  timeout -k 10 300 python3 -u tools/tune.py --log-n 20 --prec 64 --steps 400 --warmup 50 --variants "$V2" > "$out/c1_xcd.log" 2>&1 || { tail -20 "$out/c1_xcd.log"; exit 1; }
  grep -v "amdgpu.ids" "$out/c1_xcd.log"
  exit 0
fi
V='[{}, {"PIFFT_COL_C64":"8"}, {"PIFFT_COL_C64":"16"}, {"PIFFT_RADIX_LOGS":"9,11"}, {"PIFFT_RADIX_LOGS":"11,9"}, {"PIFFT_NT":"0"}, {"PIFFT_XCD_GROUP":"0","PIFFT_LAST_XCD_GROUP":"0"}, {"PIFFT_LAST_C":"8"}, {}, {"PIFFT_COL_C64":"8"}, {"PIFFT_COL_C64":"16"}, {"PIFFT_RADIX_LOGS":"9,11"}, {"PIFFT_RADIX_LOGS":"11,9"}, {"PIFFT_NT":"0"}, {"PIFFT_LAST_C":"8"}]'
timeout -k 10 300 python3 -u tools/tune.py --log-n 20 --prec 64 --steps 400 --warmup 50 --variants "$V" > "$out/c1.log" 2>&1 || { tail -20 "$out/c1.log"; exit 1; }
grep -v "amdgpu.ids" "$out/c1.log"
