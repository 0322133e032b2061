#!/bin/bash
# tools/gpu_r03ab.sh -- round-3 session ab: the headline's run-to-run spread
# with 8 workspace placements tried (BENCH_W_TRIES default 8): three bench
# processes (headline only), then the driver-style full bench line
set -o pipefail
out=gpurun_out/r03ab
mkdir -p "$out"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-secondary --no-cpu-baseline --steps 20 --warmup 5 > "$out/h$i.log" 2>&1 || { tail "$out/h$i.log"; exit 1; }
  grep '^{' "$out/h$i.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('run', $i, d['ms_per_step'], d['value'], [l['ms'] for l in d['config']['launches']], d['roofline']['frac'], d['roofline']['step_frac'])"
done
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > "$out/bench.log" 2>&1 || { tail "$out/bench.log"; exit 1; }
grep '^{' "$out/bench.log" > "$out/r03ab_bench.json"
python3 -c "import json; d=json.loads(open('$out/r03ab_bench.json').readline()); print('full', d['ms_per_step'], d['value'], [l['ms'] for l in d['config']['launches']], d['roofline']['frac'])"
