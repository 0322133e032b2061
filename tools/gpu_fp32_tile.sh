#!/bin/bash
# tools/gpu_fp32_tile.sh -- fp32 multi-pass plans at the 8192-value tile (128^4
# at 2^28) vs a 16384-value tile (1024 threads x 16 values, one workgroup per
# CU: 3 passes 1024-512-512 at C = 16/32/32) and forced pass counts
set -o pipefail
V='[{}, {"PIFFT_TILE32":"16384"}, {"PIFFT_TILE32":"16384","PIFFT_PASSES":"3"}, {"PIFFT_PASSES":"3"}, {}, {"PIFFT_TILE32":"16384"}]'
for ln in 24 26 28; do
  echo "== fp32 2^$ln P=1"
  timeout -k 10 120 python -u tools/tune.py --log-n $ln --prec 32 --steps 10 --warmup 3 --variants "$V" | grep wall || exit 1
done
