#!/bin/bash
# tools/gpu_coop.sh -- k_pass2 (two passes in one cooperative launch): GPU
# parity first, then the A/B against the two-launch plans.
set -o pipefail
mkdir -p gpurun_out/coop
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "two_passes_one_launch" \
    --timeout 120 --timeout-method thread > gpurun_out/coop/tests.log 2>&1 || { tail -30 gpurun_out/coop/tests.log; exit 1; }
tail -2 gpurun_out/coop/tests.log
V='[{}, {"PIFFT_COOP": "1"}, {"PIFFT_COOP": "2"}, {}, {"PIFFT_COOP": "1"}, {"PIFFT_COOP": "2"}]'
for spec in "20 64 1" "18 64 1" "16 64 1" "20 32 1" "16 64 4"; do
  set -- $spec
  echo "== f$2 2^$1 batch $3"
  timeout -k 10 120 python3 -u tools/tune.py --log-n $1 --prec $2 --batch $3 --steps 300 --warmup 30 --variants "$V" 2>&1 | grep -v amdgpu.ids || exit 1
done | tee gpurun_out/coop/ab.log
