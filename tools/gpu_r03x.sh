#!/bin/bash
# tools/gpu_r03x.sh -- round-3 session x: the other plan shapes the position
# model changes (profiles/r03_pos_model_shapes.log): position model vs the
# round-2 model (PIFFT_POS_MODEL=0), tuned workspaces, alternating
set -o pipefail
out=gpurun_out/r03x
mkdir -p "$out"
V='[{}, {"PIFFT_POS_MODEL":"0"}, {}, {"PIFFT_POS_MODEL":"0"}]'
run() { echo "=== $*"; timeout -k 10 300 python -u tools/tune.py "$@" --tune-ws 4 --variants "$V"; }
{ run --log-n 25 --prec 64 --workers 64 --steps 20 --warmup 5 &&
  run --log-n 25 --prec 32 --steps 20 --warmup 5 &&
  run --log-n 26 --prec 32 --steps 20 --warmup 5 &&
  run --log-n 27 --prec 32 --workers 2 --steps 20 --warmup 5 &&
  run --log-n 29 --prec 64 --workers 2 --steps 10 --warmup 3 &&
  run --log-n 29 --prec 32 --workers 16 --steps 10 --warmup 3 &&
  run --log-n 30 --prec 32 --workers 16 --steps 10 --warmup 3 &&
  run --log-n 28 --prec 64 --batch 4 --steps 5 --warmup 2; } > "$out/shapes.log" 2>&1 || { tail "$out/shapes.log"; exit 1; }
grep -E "===|wall" "$out/shapes.log"
