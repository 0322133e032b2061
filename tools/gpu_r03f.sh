#!/bin/bash
# tools/gpu_r03f.sh -- round-3 session f: the worker-interleaved layout of
# all-worker plans (C2 and larger; the tree's interleaved output staged
# through LDS) against the slice-major layout, then the whole GPU suite (the
# new layout's tests first), bench.py and the rocprofv3 roofline check
set -o pipefail
out=gpurun_out/r03f
mkdir -p "$out"
V='[{}, {"PIFFT_WORKER_IL":"0"}, {"PIFFT_WIL_CMIN":"8"}, {}, {"PIFFT_WORKER_IL":"0"}, {"PIFFT_WIL_CMIN":"8"}]'
{ for cfg in "--log-n 20 --prec 64 --workers 8 --steps 50" "--log-n 21 --prec 64 --workers 8 --steps 50" \
             "--log-n 20 --prec 32 --workers 8 --steps 50" "--log-n 24 --prec 64 --workers 8 --steps 20" \
             "--log-n 28 --prec 64 --workers 8 --steps 10" "--log-n 20 --prec 64 --workers 2 --steps 50"; do
    echo "=== $cfg"; timeout -k 10 200 python -u tools/tune.py $cfg --warmup 5 --variants "$V" || exit 1; done; } > "$out/wil.log" 2>&1 || { tail "$out/wil.log"; exit 1; }
grep -E "===|wall" "$out/wil.log"
bash tools/gpu_r03.sh r03f "tests/test_gpu_parity.py -k worker_interleaved tests"
