#!/bin/bash
# tools/gpu_r03q.sh -- round-3 session q: the planner's position-aware pass
# rates (1024-point pass last at 2^28 / 2^29) vs the round-2 model
# (PIFFT_POS_MODEL=0), alternating fresh plans; fp64 9,9,10 with the last
# pass at C = 16 (256-B segments, one workgroup per CU); then the evidence
# session (GPU tests, bench, rocprofv3 check)
set -o pipefail
out=gpurun_out/r03q
mkdir -p "$out"
V='[{}, {"PIFFT_POS_MODEL":"0"}, {}, {"PIFFT_POS_MODEL":"0"}, {}, {"PIFFT_POS_MODEL":"0"}, {"PIFFT_RADIX_LOGS":"9,9,10","PIFFT_COL_C64":"16"}]'
{ echo "=== fp64 2^28"; timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 64 --steps 10 --warmup 3 --variants "$V";
  echo "=== fp32 2^28"; timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 32 --steps 10 --warmup 3 --variants '[{}, {"PIFFT_POS_MODEL":"0"}, {}, {"PIFFT_POS_MODEL":"0"}]'; } > "$out/pos_model.log" 2>&1 || { tail "$out/pos_model.log"; exit 1; }
grep -E "===|wall" "$out/pos_model.log"
bash tools/gpu_r03.sh r03q
