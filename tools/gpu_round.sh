#!/bin/bash
# tools/gpu_round.sh -- one gpurun job: A/B of library variants on the C4
# shapes, then the GPU parity suite on the in-tree build.  Every GPU step has
# its own time limit; the first failure ends the job.
#   gpurun --timeout 1100 -- bash tools/gpu_round.sh <tag> variants/a.so variants/b.so ...
set -o pipefail
tag="$1"; shift
mkdir -p gpurun_out
out="gpurun_out/$tag"
timeout -k 10 240 bash tools/ab.sh "--log-n 28 --prec 64" "$@" > "${out}_c4.log" 2>&1 || exit 1
timeout -k 10 240 bash tools/ab.sh "--log-n 28 --prec 64 --workers 8 --count 1" "$@" > "${out}_p8.log" 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "${out}_tests.log" 2>&1 || exit 1
tail -3 "${out}_tests.log"
