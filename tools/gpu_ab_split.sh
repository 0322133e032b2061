#!/bin/bash
# tools/gpu_ab_split.sh -- A/B of library variants on C4 and on one rank's
# plan of the 2/4/8-GPU jobs (the fused tree+first pass), then the fused-tree
# and size-sweep parity tests on the in-tree build.
#   gpurun --timeout 900 -- bash tools/gpu_ab_split.sh <tag> variants/a.so variants/b.so ...
set -o pipefail
tag="$1"; shift
mkdir -p gpurun_out
out="gpurun_out/$tag"
timeout -k 10 200 bash tools/ab.sh "--log-n 28 --prec 64" "$@" > "${out}_c4.log" 2>&1 || exit 1
for g in 2 4 8; do
    timeout -k 10 150 bash tools/ab.sh "--log-n 28 --prec 64 --workers $g --first $((g - 1)) --count 1" "$@" \
        > "${out}_p$g.log" 2>&1 || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "fused or size_sweep or config2 or large_split or config5" > "${out}_tests.log" 2>&1 || exit 1
tail -2 "${out}_tests.log"
