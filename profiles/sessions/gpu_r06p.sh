# round 6, session p: the headline step by the number of workspace placements
# pifft_plan_tune_workspace tries before the warm-up (BENCH_W_TRIES; default 8)
set -o pipefail
out=gpurun_out/r06p
mkdir -p $out
for rep in 1 2; do
  for t in 1 8 16 32; do
    BENCH_W_TRIES=$t timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-secondary --no-cpu-baseline --detail '' > $out/w$t.$rep.txt 2>&1 || exit 1
    echo "tries=$t rep=$rep $(grep '^{' $out/w$t.$rep.txt | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["mean_ms"])')" >> $out/summary.txt
  done
done
