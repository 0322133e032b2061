#!/bin/bash
# tools/gpu_r04p_steps.sh -- round-4 session p: step time of configs 3 and 1
# against the timed loop's length (tools/tune.py, 5 warm-up steps), the data
# behind bench.py's 1000-step loops for the 10-50 us configs
# (profiles/r04p_loop_length.log).
set -o pipefail
for k in 50 200 1000 50 200; do
  timeout -k 10 120 python3 -u tools/tune.py --log-n 12 --prec 32 --batch 4096 --steps $k --warmup 5 --variants '[{}]' 2>&1 | grep -v "amdgpu.ids\|torch copy" | sed "s/^/C3 steps=$k /" || exit 1
done
for k in 50 200 1000; do
  timeout -k 10 120 python3 -u tools/tune.py --log-n 20 --prec 64 --steps $k --warmup 5 --variants '[{}]' 2>&1 | grep -v "amdgpu.ids\|torch copy" | sed "s/^/C1 steps=$k /" || exit 1
done
