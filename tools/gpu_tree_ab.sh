#!/bin/bash
# tools/gpu_tree_ab.sh -- A/B of library variants on the fused tree+first pass:
# one worker's plan of the 8-, 4- and 2-GPU jobs at 2^28 fp64 (tools/ab.sh).
#   gpurun -- bash tools/gpu_tree_ab.sh variants/a.so variants/b.so ...
set -o pipefail
mkdir -p gpurun_out
for P in 8 4 2; do
  AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh "--log-n 28 --prec 64 --workers $P --first $((P-1)) --count 1" "$@" \
      > gpurun_out/tree_ab_p$P.log 2>&1 || exit 1
  echo "== P=$P"; grep -v amdgpu gpurun_out/tree_ab_p$P.log | grep -v "torch copy" | cut -c1-230
done
