#!/bin/bash
# tools/gpu_r03j.sh -- round-3 session j: fp32 2^28 three-pass plans with the
# packed VPT-32 passes (two butterflies per register pair) vs the 4-pass plan
# and the 1024-thread three-pass plan; bitwise test
set -o pipefail
out=gpurun_out/r03j
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k packed_vpt32 -x -v --timeout 200 --timeout-method thread > "$out/test.log" 2>&1 || { tail -30 "$out/test.log"; exit 1; }
tail -2 "$out/test.log"
V='[{}, {"PIFFT_TILE32":"16384","PIFFT_PASSES":"3"}, {"PIFFT_TILE32":"16384","PIFFT_PASSES":"3","PIFFT_VPT32":"1"}, {"PIFFT_TILE32":"16384","PIFFT_VPT32":"1"}, {}, {"PIFFT_TILE32":"16384","PIFFT_PASSES":"3","PIFFT_VPT32":"1"}]'
{ echo "=== fp32 2^28"; timeout -k 10 200 python -u tools/tune.py --log-n 28 --prec 32 --steps 10 --warmup 3 --variants "$V";
  echo "=== fp32 2^26"; timeout -k 10 200 python -u tools/tune.py --log-n 26 --prec 32 --steps 10 --warmup 3 --variants "$V";
  echo "=== fp32 2^30"; timeout -k 10 200 python -u tools/tune.py --log-n 30 --prec 32 --steps 5 --warmup 2 --variants "$V"; } > "$out/pack32.log" 2>&1 || { tail "$out/pack32.log"; exit 1; }
grep -E "===|wall" "$out/pack32.log"
