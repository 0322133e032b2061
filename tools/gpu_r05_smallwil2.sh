#!/bin/bash
# tools/gpu_r05_smallwil2.sh [tag] -- round 5: the whole GPU suite at HEAD,
# then the single-pass all-worker rule (two-pass worker-interleaved plans
# from M = 2^12) against PIFFT_WIL_SINGLE=0 over 2^12-2^19, P = 2..16, both
# precisions, outputs checked against each other.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05x}
mkdir -p "$out"
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$out/gpu_tests.txt" 2>&1 || { tail -40 "$out/gpu_tests.txt"; exit 1; }
tail -2 "$out/gpu_tests.txt"
V='[{}, {"PIFFT_WIL_SINGLE":"0"}, {}, {"PIFFT_WIL_SINGLE":"0"}]'
for prec in 64 32; do
  for n in 12 13 14 15 16 17 18 19; do
    for P in 2 4 8 16; do
      echo "=== fp$prec 2^$n P = $P" >> "$out/ab.log"
      timeout -k 10 120 python3 -u tools/tune.py --log-n $n --prec $prec --workers $P --steps 1000 --warmup 300 --check \
        --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/ab.log" || exit 1
    done
  done
done
echo done
