#!/bin/bash
# Historical in part: PIFFT_W_BLOCK / PIFFT_Y_BLOCK were removed after this session; at HEAD those legs run the default.
# tools/gpu_r04d.sh -- round-4 session d: the fused tree pass at 8 values per
# thread (PIFFT_FUSED_VPT=8) over the small one-worker slices whose fused
# launch has few workgroups, and config 2's worker-interleaved passes at 8
# (PIFFT_WIL_VPT=8); alternating variants per shape, one process per shape.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04d
mkdir -p "$out"
V='[{}, {"PIFFT_FUSED_VPT": 8}, {}, {"PIFFT_FUSED_VPT": 8}]'
for shape in "18 64 8 0" "19 64 8 0" "20 64 8 0" "20 64 8 7" "21 64 8 0" "22 64 8 0" "23 64 8 0" "20 64 2 0" "20 64 4 0" "20 64 16 0" "22 64 16 0" "24 64 8 0" "20 32 8 0" "21 32 8 0" "22 32 8 0"; do
  set -- $shape
  echo "=== log2 N $1, fp$2, worker $4 of $3"
  timeout -k 10 120 python3 -u tools/tune.py --log-n $1 --prec $2 --workers $3 --first $4 --count 1 --steps 400 --warmup 20 --variants "$V" 2>&1 | grep -v "amdgpu.ids\|^torch" || exit 1
done > "$out/fused_vpt8.log"
cat "$out/fused_vpt8.log"
timeout -k 10 120 python3 -u tools/tune.py --log-n 20 --prec 64 --workers 8 --steps 400 --warmup 20 --variants \
  '[{}, {"PIFFT_WIL_VPT": 8}, {}, {"PIFFT_WIL_VPT": 8}]' 2>&1 | grep -v "amdgpu.ids\|^torch" > "$out/wil_vpt8_c2.log" || exit 1
cat "$out/wil_vpt8_c2.log"
# the blocked workspace between the last two passes (PIFFT_W_BLOCK): bitwise tests, then timing
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -k blocked -x -v --timeout 200 --timeout-method thread > "$out/blocked_tests.log" 2>&1 || { tail -30 "$out/blocked_tests.log"; exit 1; }
tail -2 "$out/blocked_tests.log"
for prec in 64 32; do
  timeout -k 10 300 python3 -u tools/tune.py --log-n 28 --prec $prec --tune-ws 8 --steps 20 --variants \
    '[{}, {"PIFFT_W_BLOCK": 4}, {"PIFFT_W_BLOCK": 3}, {"PIFFT_Y_BLOCK": 4}, {"PIFFT_W_BLOCK": 4, "PIFFT_Y_BLOCK": 4}, {}, {"PIFFT_W_BLOCK": 4}, {"PIFFT_W_BLOCK": 3}, {"PIFFT_Y_BLOCK": 4}, {"PIFFT_W_BLOCK": 4, "PIFFT_Y_BLOCK": 4}, {"PIFFT_RADIX_LOGS": "9,10,9", "PIFFT_W_BLOCK": 4, "PIFFT_Y_BLOCK": 4}, {"PIFFT_RADIX_LOGS": "9,10,9"}]' 2>&1 | grep -v "amdgpu.ids" > "$out/blocked_f$prec.log" || exit 1
  cat "$out/blocked_f$prec.log"
done
