#!/bin/bash
# tools/gpu_vpt_sweep.sh -- single-pass launches at 8 vs 16 values per thread
# (PIFFT_SINGLE_VPT), by batch size: config-3 shares (fp32 4096-point) and
# fp64 single passes; then the GPU parity tests of single-pass plans.
set -o pipefail
mkdir -p gpurun_out/vpt
V='[{"PIFFT_SINGLE_VPT":"16"},{"PIFFT_SINGLE_VPT":"8"},{"PIFFT_SINGLE_VPT":"16"},{"PIFFT_SINGLE_VPT":"8"}]'
{
for b in 128 256 512 1024 2048 4096; do
  echo "== fp32 4096 x $b"
  timeout -k 10 120 python -u tools/tune.py --log-n 12 --prec 32 --batch $b --steps 50 --warmup 10 --variants "$V" || exit 1
done
for ln in 12 13; do for b in 1 16 128 1024; do
  echo "== fp64 2^$ln x $b"
  timeout -k 10 120 python -u tools/tune.py --log-n $ln --prec 64 --batch $b --steps 50 --warmup 10 --variants "$V" || exit 1
done; done
} > gpurun_out/vpt/sweep.log 2>&1 || { tail -20 gpurun_out/vpt/sweep.log; exit 1; }
grep -E "==|wall" gpurun_out/vpt/sweep.log | sed 's/ :: .*//'
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "golden or size_sweep or batched or config3 or bitrev or known_answer" > gpurun_out/vpt/tests.log 2>&1 || { tail -30 gpurun_out/vpt/tests.log; exit 1; }
tail -2 gpurun_out/vpt/tests.log
