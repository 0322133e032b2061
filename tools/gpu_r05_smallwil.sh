#!/bin/bash
# tools/gpu_r05_smallwil.sh [tag] -- round 5: all-worker plans whose local FFT
# is one pass (N / P <= 2^14) run tree + pass + interleave (three launches);
# the worker-interleaved two-pass plan with the fused tree (MODE 11, two
# launches) against them -- PIFFT_SINGLE_MAX_LOG = 13 / 12 / 11 forces the
# two-pass local FFT -- over 2^13-2^18, P = 2..16, both precisions, outputs
# checked against the default plan's.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05w}
mkdir -p "$out"
V='[{}, {"PIFFT_SINGLE_MAX_LOG":"13"}, {"PIFFT_SINGLE_MAX_LOG":"12"}, {"PIFFT_SINGLE_MAX_LOG":"11"}, {}, {"PIFFT_SINGLE_MAX_LOG":"13"}, {"PIFFT_SINGLE_MAX_LOG":"12"}]'
for prec in 64 32; do
  for n in 13 14 15 16 17 18; do
    for P in 2 4 8 16; do
      echo "=== fp$prec 2^$n P = $P" >> "$out/smallwil.log"
      timeout -k 10 200 python3 -u tools/tune.py --log-n $n --prec $prec --workers $P --steps 1000 --warmup 300 --check \
        --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/smallwil.log" || exit 1
    done
  done
done
echo done
