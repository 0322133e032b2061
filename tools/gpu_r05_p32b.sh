#!/bin/bash
# tools/gpu_r05_p32b.sh [tag] -- round 5: P = 32 one launch with the factored
# tree twiddles (PIFFT_WIL_TREE_MIN_LOG=0: one table lookup per level and
# thread) against the reference-formula table and the four-launch plan.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05p32b}
mkdir -p "$out"
V='[{}, {"PIFFT_WIL_TREE_MIN_LOG":"0"}, {"PIFFT_WIL_ONE_LAUNCH":"0"}, {}, {"PIFFT_WIL_TREE_MIN_LOG":"0"}, {"PIFFT_WIL_ONE_LAUNCH":"0"}]'
for prec in 64 32; do
  for n in 10 11 12 13; do
    for P in 16 32; do
      echo "=== fp$prec 2^$n P = $P" >> "$out/p32b.log"
      timeout -k 10 120 python3 -u tools/tune.py --log-n $n --prec $prec --workers $P --steps 2000 --warmup 500 --check \
        --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/p32b.log" || exit 1
    done
  done
done
echo done
