#!/bin/bash
# tools/gpu_r04k.sh -- round-4 session k: config 2's one-GPU slice at other
# values per thread -- the fused tree pass at 4 (PIFFT_FUSED_VPT), the last
# pass at 8 / 4 (PIFFT_LAST_VPT) -- parity first, then A/B timings on the
# slice and on neighbouring slice / small one-worker shapes.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04k
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "slice_pass_forms" -m gpu -x -q --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"
V='[{}, {"PIFFT_FUSED_VPT":"4"}, {"PIFFT_LAST_VPT":"8"}, {"PIFFT_LAST_VPT":"4"}, {"PIFFT_FUSED_VPT":"4","PIFFT_LAST_VPT":"8"}, {"PIFFT_ORDER":"1"}, {"PIFFT_ORDER":"1","PIFFT_LAST_VPT":"8"}, {}, {"PIFFT_FUSED_VPT":"4"}, {"PIFFT_LAST_VPT":"8"}, {"PIFFT_FUSED_VPT":"4","PIFFT_LAST_VPT":"8"}]'
timeout -k 10 300 python3 -u tools/tune.py --log-n 20 --prec 64 --workers 8 --first 0 --count 1 --steps 400 --warmup 50 --variants "$V" > "$out/slice.log" 2>&1 || { tail -20 "$out/slice.log"; exit 1; }
cat "$out/slice.log"
W='[{}, {"PIFFT_LAST_VPT":"8"}, {"PIFFT_FUSED_VPT":"4"}, {}, {"PIFFT_LAST_VPT":"8"}, {"PIFFT_FUSED_VPT":"4"}]'
for a in "--log-n 18 --workers 4" "--log-n 19 --workers 8" "--log-n 21 --workers 8" "--log-n 22 --workers 8" "--log-n 21 --workers 16" "--log-n 18 --workers 8"; do
  echo "== $a" >> "$out/shapes.log"
  timeout -k 10 300 python3 -u tools/tune.py $a --prec 64 --first 0 --count 1 --steps 300 --warmup 50 --variants "$W" >> "$out/shapes.log" 2>&1 || { tail -20 "$out/shapes.log"; exit 1; }
done
for a in "--log-n 16" "--log-n 17" "--log-n 18"; do
  echo "== P=1 $a" >> "$out/shapes.log"
  timeout -k 10 300 python3 -u tools/tune.py $a --prec 64 --steps 300 --warmup 50 --variants '[{}, {"PIFFT_LAST_VPT":"8"}, {}, {"PIFFT_LAST_VPT":"8"}]' >> "$out/shapes.log" 2>&1 || { tail -20 "$out/shapes.log"; exit 1; }
done
grep -v "torch copy\|amdgpu.ids" "$out/shapes.log"
