#!/bin/bash
# tools/gpu_r04e.sh -- round-4 session e: the default 8-values-per-thread rules
# on more worker-interleaved shapes (PIFFT_WIL_VPT 8 vs 16), then a HEAD
# evidence set (tools/gpu_r04.sh r04e tbs: GPU tests, bench line, rocprofv3
# stats, roofline check).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04e
mkdir -p "$out"
for shape in "18 2" "19 4" "19 8" "21 8" "21 4" "20 4"; do
  set -- $shape
  echo "=== fp64 2^$1, all $2 workers (worker-interleaved)"
  timeout -k 10 120 python3 -u tools/tune.py --log-n $1 --prec 64 --workers $2 --steps 400 --warmup 20 --variants \
    '[{"PIFFT_WIL_VPT": 16}, {}, {"PIFFT_WIL_VPT": 16}, {}]' 2>&1 | grep -v "amdgpu.ids\|^torch" || exit 1
done > "$out/wil_vpt8_shapes.log"
cat "$out/wil_vpt8_shapes.log"
bash tools/gpu_r04.sh r04e tbs
