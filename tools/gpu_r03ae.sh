#!/bin/bash
# tools/gpu_r03ae.sh -- round-3 session ae: the tree fused into the first
# worker-interleaved pass (MODE 11, PIFFT_WIL_FUSE=1) -- parity first, then
# the A/B against the separate tree launch (config 2 and other all-worker
# plans on one GPU), and lines per workgroup
set -o pipefail
out=gpurun_out/r03ae
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "fused_tree_vs_oracle or worker_interleaved_layout" > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
grep -E "PASSED|FAILED|passed|failed" "$out/tests.log" | tail -20
V='[{}, {"PIFFT_WIL_FUSE":"1"}, {"PIFFT_WIL_FUSE":"1","PIFFT_WIL_FUSE_C":"16"}, {"PIFFT_WIL_FUSE":"1","PIFFT_WIL_FUSE_C":"32"}, {}, {"PIFFT_WIL_FUSE":"1"}]'
run() { echo "=== $*"; timeout -k 10 200 python -u tools/tune.py "$@" --variants "$V"; }
{ run --log-n 20 --prec 64 --workers 8 --steps 200 --warmup 20 &&
  run --log-n 20 --prec 32 --workers 8 --steps 200 --warmup 20 &&
  run --log-n 22 --prec 64 --workers 8 --steps 50 --warmup 10 &&
  run --log-n 24 --prec 64 --workers 8 --steps 30 --warmup 5 &&
  run --log-n 20 --prec 64 --workers 16 --steps 200 --warmup 20 &&
  run --log-n 28 --prec 64 --workers 8 --steps 5 --warmup 2 --tune-ws 4; } > "$out/ab.log" 2>&1 || { tail "$out/ab.log"; exit 1; }
grep -E "===|wall" "$out/ab.log"
