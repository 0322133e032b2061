#!/bin/bash
# tools/gpu_smallr_tile.sh -- fp64 strided passes of R <= 256 at a 4096- vs
# 8192-value tile (PIFFT_SMALLR_TILE64): R = 256 at C = 32 spills 20 B/lane at
# 128 VGPRs; C = 16 runs 256 threads at 138 VGPRs, 3 workgroups per CU
set -o pipefail
V='[{"PIFFT_SMALLR_TILE64":"8192"}, {"PIFFT_SMALLR_TILE64":"4096"}, {"PIFFT_SMALLR_TILE64":"8192"}, {"PIFFT_SMALLR_TILE64":"4096"}]'
for ln in 21 22 23 24 25 26; do
  echo "== fp64 2^$ln P=1"
  timeout -k 10 120 python -u tools/tune.py --log-n $ln --prec 64 --steps 10 --warmup 3 --variants "$V" || exit 1
done
for w in 8 16; do for ln in 26 28; do
  echo "== fp64 2^$ln worker 0 of $w"
  timeout -k 10 120 python -u tools/tune.py --log-n $ln --prec 64 --workers $w --count 1 --steps 10 --warmup 3 --variants "$V" || exit 1
done; done
echo "== fp64 2^32 worker 0 of 16"
timeout -k 10 120 python -u tools/tune.py --log-n 32 --prec 64 --workers 16 --count 1 --steps 5 --warmup 2 --variants "$V" || exit 1
