#!/bin/bash
# tools/gpu_r05_wiltile4.sh [tag] -- round 5: the planner's MODE 11 refinements
# (the 4096-value tile at J = 4 below 256 workgroups; J = 4 where J = 8 splits
# the remainder) at HEAD: the all-worker GPU parity tests, then the new
# default plan against the previous one (J = 8 at the 8192-value tile) over
# 2^17-2^22, P = 2 / 4 / 8, both precisions, outputs checked against each
# other (tools/tune.py --check).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05v}
mkdir -p "$out"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "fused_all_worker or worker_interleaved or config2 or fuzz" > "$out/tests.txt" 2>&1 || { tail -30 "$out/tests.txt"; exit 1; }
tail -3 "$out/tests.txt"
OLD='{"PIFFT_WIL_FUSE_J":"8","PIFFT_WIL_FUSE_TILE":"8192"}'
for prec in 64 32; do
  for n in 17 18 19 20 21 22; do
    for P in 2 4 8; do
      echo "=== fp$prec 2^$n P = $P" >> "$out/ab.log"
      timeout -k 10 200 python3 -u tools/tune.py --log-n $n --prec $prec --workers $P --steps 1000 --warmup 300 --check \
        --variants "[{}, $OLD, {}, $OLD]" 2>&1 | grep -v amdgpu.ids >> "$out/ab.log" || exit 1
    done
  done
done
cat "$out/ab.log" | cut -c1-220
