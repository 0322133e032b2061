#!/bin/bash
# Historical: PIFFT_FUSED_C was removed after this session; at HEAD that leg runs the default.
# tools/gpu_r04n.sh -- round-4 session n: config 2's slice with its fused tree
# pass at C = 2 (128 workgroups gathering leaves; PIFFT_FUSED_C), parity
# first, then A/B on the slice and its neighbours.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04n
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "slice_last_pass_forms" -m gpu -x -q --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
W='[{}, {"PIFFT_FUSED_C":"2"}, {}, {"PIFFT_FUSED_C":"2"}, {}, {"PIFFT_FUSED_C":"2"}]'
for a in "--log-n 20 --workers 8" "--log-n 19 --workers 8" "--log-n 21 --workers 8" "--log-n 21 --workers 16" "--log-n 18 --workers 4"; do
  echo "== $a" >> "$out/fused_c2.log"
  timeout -k 10 300 python3 -u tools/tune.py $a --prec 64 --first 0 --count 1 --steps 400 --warmup 50 --variants "$W" >> "$out/fused_c2.log" 2>&1 || { tail -20 "$out/fused_c2.log"; exit 1; }
done
grep -v "amdgpu.ids\|torch copy" "$out/fused_c2.log"
