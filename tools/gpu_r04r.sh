#!/bin/bash
# tools/gpu_r04r.sh -- round-4 session r: the secondary configs' timed-loop
# length and warm-up (BENCH_SMALL_STEPS / BENCH_SMALL_WARMUP), A/B on one box.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04r
mkdir -p "$out"
for v in "50 5" "200 50" "200 5" "50 5" "200 50" "1000 100"; do
  set -- $v
  BENCH_SMALL_STEPS=$1 BENCH_SMALL_WARMUP=$2 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > "$out/b_$1_$2.log" 2>&1 || { tail -20 "$out/b_$1_$2.log"; exit 1; }
  grep '^{' "$out/b_$1_$2.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('steps $1 warmup $2: headline', d['ms_per_step'], ' '.join(f'{k} {v[\"ms_per_step\"]*1e3:.2f}' for k, v in d['config']['secondary'].items() if k != 'C4_f32'))" | tee -a "$out/summary.txt"
done
