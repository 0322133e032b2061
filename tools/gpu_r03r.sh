#!/bin/bash
# tools/gpu_r03r.sh -- round-3 session r: the new last pass of fp64 / fp32 2^28
# (the 1024-point pass, 128-B segments on both sides): its streaming form
# (PIFFT_LAST_NT 0 plain, 2 nt loads, 3 nt stores; default 1 nt both) and its
# XCD tile grouping (PIFFT_LAST_XCD_GROUP, log2 tiles per XCD run; default 2)
set -o pipefail
out=gpurun_out/r03r
mkdir -p "$out"
V='[{}, {"PIFFT_LAST_NT":"0"}, {"PIFFT_LAST_NT":"2"}, {"PIFFT_LAST_NT":"3"}, {"PIFFT_LAST_XCD_GROUP":"0"}, {"PIFFT_LAST_XCD_GROUP":"1"}, {"PIFFT_LAST_XCD_GROUP":"3"}, {"PIFFT_LAST_XCD_GROUP":"4"}, {}]'
{ echo "=== fp64 2^28"; timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 64 --steps 10 --warmup 3 --variants "$V";
  echo "=== fp32 2^28"; timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 32 --steps 10 --warmup 3 --variants "$V"; } > "$out/last_pass.log" 2>&1 || { tail "$out/last_pass.log"; exit 1; }
grep -E "===|wall" "$out/last_pass.log"
