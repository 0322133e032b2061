#!/bin/bash
# tools/gpu_r05_p32.sh [tag] -- round 5: one fused launch at P = 32 (two
# threads per position, each with half the workers' tree): the small-plan GPU
# tests, then the one-launch plan against the four-launch one
# (PIFFT_WIL_ONE_LAUNCH=0) at n = 2^10-2^13, both precisions.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05p32}
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "tiny or single_pass_all_worker or fused_all_worker" > "$out/tests.txt" 2>&1 || { tail -40 "$out/tests.txt"; exit 1; }
tail -2 "$out/tests.txt"
V='[{}, {"PIFFT_WIL_ONE_LAUNCH":"0"}, {}, {"PIFFT_WIL_ONE_LAUNCH":"0"}]'
for prec in 64 32; do
  for n in 10 11 12 13; do
    echo "=== fp$prec 2^$n P = 32" >> "$out/p32.log"
    timeout -k 10 120 python3 -u tools/tune.py --log-n $n --prec $prec --workers 32 --steps 2000 --warmup 500 --check \
      --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/p32.log" || exit 1
  done
done
echo done
