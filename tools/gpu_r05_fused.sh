#!/bin/bash
# tools/gpu_r05_fused.sh [tag] -- round 5: the copy ceiling of one rank's fused
# tree + first pass by leaf-read segment width (tools/probe_fused2.hip, built
# in the container), then the rank plans of the 8-, 4- and 2-GPU split on the
# SAME box (tools/tune.py, default plans), so the kernel sits beside its
# ceiling.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05e}
mkdir -p "$out"
timeout -k 10 120 ./tools/probe_fused2_bin > "$out/fused_ceiling.log" 2>&1 || { cat "$out/fused_ceiling.log"; exit 1; }
for g in 8 4 2; do
  echo "== fp64 2^28, worker 0 of $g (default plan)" >> "$out/fused_ceiling.log"
  timeout -k 10 200 python3 -u tools/tune.py --log-n 28 --prec 64 --workers $g --first 0 --count 1 --steps 20 --warmup 5 --tune-ws 4 --variants '[{}, {}]' 2>&1 | grep -v "amdgpu.ids" >> "$out/fused_ceiling.log" || exit 1
done
cat "$out/fused_ceiling.log"
