#!/bin/bash
# tools/gpu_r05_wiltree.sh [tag] -- round 5: the worker-interleaved all-worker
# plans' tree launch (k_tree_wil) with the factored two-level twiddles
# (abvar2/wilfac.so, HEAD) against the reference-formula table (abvar2/base.so,
# the previous commit), on config 2 and neighbouring shapes (tools/ab.sh: two
# rounds, per-launch times in context).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05g}
mkdir -p "$out"
for shape in "--log-n 20 --prec 64 --workers 8" "--log-n 20 --prec 32 --workers 8" "--log-n 21 --prec 64 --workers 8" "--log-n 22 --prec 64 --workers 16" "--log-n 18 --prec 64 --workers 4"; do
  echo "=== $shape" >> "$out/wiltree.log"
  AB_ROUNDS=3 timeout -k 10 300 bash tools/ab.sh "$shape --steps 2000 --warmup 500" abvar2/base.so abvar2/wilfac.so >> "$out/wiltree.log" 2>&1 || { tail -20 "$out/wiltree.log"; exit 1; }
done
cat "$out/wiltree.log"
