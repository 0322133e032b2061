#!/bin/bash
# tools/gpu_wpad_check.sh -- padded workspace rows: GPU parity (forced on small
# plans, and the full-size C4/C5/fp32/2^30 tests that now run padded by
# default), then the A/B over other plan shapes (tools/gpu_wpad_shapes.sh).
set -o pipefail
mkdir -p gpurun_out/place
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -m gpu -x -v -k "padded_workspace or fullsize" \
    --timeout 200 --timeout-method thread > gpurun_out/place/wpad_tests.log 2>&1 || { tail -30 gpurun_out/place/wpad_tests.log; exit 1; }
tail -2 gpurun_out/place/wpad_tests.log
bash tools/gpu_wpad_shapes.sh
