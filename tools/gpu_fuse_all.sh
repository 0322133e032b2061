#!/bin/bash
# tools/gpu_fuse_all.sh -- the tree fused into the first pass for plans that
# hold ALL P workers (each worker's pass re-reads the P leaves: P x the input)
# vs the separate k_tree launch, by input size; then the GPU suite with the
# fused form forced on everywhere it applies.
set -o pipefail
V='[{}, {"PIFFT_FUSE_ALL_MAX_MIB":"100000"}, {}, {"PIFFT_FUSE_ALL_MAX_MIB":"100000"}]'
{
for spec in "--log-n 16 --workers 8" "--log-n 18 --workers 8" "--log-n 20 --workers 8" "--log-n 20 --workers 4" "--log-n 20 --workers 16" "--log-n 21 --workers 8" "--log-n 22 --workers 8" "--log-n 23 --workers 8" "--log-n 24 --workers 8" "--log-n 24 --workers 2" "--log-n 20 --prec 32 --workers 8" "--log-n 22 --prec 32 --workers 8" "--log-n 12 --prec 32 --batch 4096 --workers 4"; do
  echo "== $spec"
  timeout -k 10 120 python -u tools/tune.py $spec --steps 20 --warmup 5 --variants "$V" | grep wall | sed 's/(sum of launches.*:://' || exit 1
done
} > gpurun_out/fuse_all.log 2>&1 || { tail -5 gpurun_out/fuse_all.log; exit 1; }
cat gpurun_out/fuse_all.log
PIFFT_FUSE_ALL_MAX_MIB=100000 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fuse_all_tests.log 2>&1 || { tail -30 gpurun_out/fuse_all_tests.log; exit 1; }
tail -1 gpurun_out/fuse_all_tests.log
