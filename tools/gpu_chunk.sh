#!/bin/bash
# tools/gpu_chunk.sh -- chunked pass pairs: parity tests, then chunk-size sweep on C4 and P=8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "chunked" > gpurun_out/chunk_tests.log 2>&1 || { tail -30 gpurun_out/chunk_tests.log; exit 1; }
tail -3 gpurun_out/chunk_tests.log
V='[{"PIFFT_CHUNK_MIB":0},{"PIFFT_CHUNK_MIB":32},{"PIFFT_CHUNK_MIB":64},{"PIFFT_CHUNK_MIB":128},{"PIFFT_CHUNK_MIB":256},{"PIFFT_CHUNK_MIB":0}]'
timeout -k 10 240 python -u tools/tune.py --log-n 28 --prec 64 --variants "$V" > gpurun_out/chunk_c4.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/tune.py --log-n 28 --prec 64 --workers 8 --first 7 --count 1 --variants "$V" > gpurun_out/chunk_p8.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/chunk_c4.log | cut -c1-200
grep -v amdgpu.ids gpurun_out/chunk_p8.log | cut -c1-200
