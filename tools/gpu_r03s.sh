#!/bin/bash
# tools/gpu_r03s.sh -- round-3 session s: the radix order at 2^28 WITH workspace
# placement tuning (as bench.py runs it): position model (512-512-1024) vs the
# round-2 model (1024-512-512, PIFFT_POS_MODEL=0), alternating fresh plans,
# four of each, fp64 and fp32
set -o pipefail
out=gpurun_out/r03s
mkdir -p "$out"
V='[{}, {"PIFFT_POS_MODEL":"0"}, {}, {"PIFFT_POS_MODEL":"0"}, {}, {"PIFFT_POS_MODEL":"0"}, {}, {"PIFFT_POS_MODEL":"0"}]'
{ echo "=== fp64 2^28, tuned workspace"; timeout -k 10 400 python -u tools/tune.py --log-n 28 --prec 64 --steps 20 --warmup 3 --tune-ws 4 --variants "$V";
  echo "=== fp32 2^28, tuned workspace"; timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 32 --steps 20 --warmup 3 --tune-ws 4 --variants "$V";
  echo "=== fp64 2^29, tuned workspace"; timeout -k 10 400 python -u tools/tune.py --log-n 29 --prec 64 --steps 10 --warmup 3 --tune-ws 4 --variants '[{}, {"PIFFT_POS_MODEL":"0"}, {}, {"PIFFT_POS_MODEL":"0"}]'; } > "$out/order_tuned.log" 2>&1 || { tail "$out/order_tuned.log"; exit 1; }
grep -E "===|wall" "$out/order_tuned.log"
