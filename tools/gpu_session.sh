#!/bin/bash
# tools/gpu_session.sh <tag> <stages> [tests...] -- one GPU evidence session (rounds 5-6).
# stages: any of t (GPU tests + smoke), b (bench.py as the driver runs it; the
#   printed line, and its sidecar with the per-launch detail),
#   s (rocprofv3 --kernel-trace --stats of bench.py in the same session, then
#      tools/check_rooflines.py on both lines),
#   p (PMC traffic, tools/pmc_traffic.py, FETCH_SIZE / WRITE_SIZE passes, of
#      every config's plan: C4 fp64 and fp32, C3, C1, C2, C2's slice, and one
#      rank's plan of the 2-, 4- and 8-GPU split at 2^28 -- the keys bench.py
#      reads roofline.traffic by),
#   q (only the per-rank 2^28 plans of p).
# Every GPU step has its own time limit; the first failure ends the job.
set -o pipefail
tag="${1:-r05}"
stages="${2:-tbs}"
shift 2
tests="${*:-tests}"
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p "$out"
{ echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "memory.max: $(cat /sys/fs/cgroup/memory.max 2>/dev/null)";
  echo "nproc: $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; } > "$out/host.txt"
cat "$out/host.txt"
if [[ "$stages" == *t* ]]; then
  timeout -k 10 900 python -u -m pytest $tests -m gpu -x -v --timeout 200 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -60 "$out/gpu_tests.log"; exit 1; }
  tail -3 "$out/gpu_tests.log"
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || { cat "$out/smoke.txt"; exit 1; }
  tail -1 "$out/smoke.txt"
fi
if [[ "$stages" == *b* ]]; then
  timeout -k 10 900 python -u bench.py --detail "$out/${tag}_bench_detail.json" > "$out/bench.log" 2>&1 || { tail -20 "$out/bench.log"; exit 1; }
  grep '^{' "$out/bench.log" | tail -1 > "$out/${tag}_bench.json" || exit 1
  python3 -c "import json; s=open('$out/${tag}_bench.json').read(); d=json.loads(s); print('chars', len(s), 'value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic']); [print(k, v.get('ms_per_step'), (v.get('roofline') or {}).get('frac'), (v.get('roofline') or {}).get('traffic'), (v.get('cpu_baseline') or {}).get('value')) for k, v in d['config']['secondary'].items()]; print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
fi
if [[ "$stages" == *s* ]]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/stats_sec" -o sec -- \
      python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --detail "$out/stats_detail.json" > "$out/stats_sec.log" 2>&1 || { tail -20 "$out/stats_sec.log"; exit 1; }
  rocpd2summary -i "$out/stats_sec/sec_results.db" -f csv -d "$out/sum_sec" -o sec > /dev/null 2>&1 || exit 1
  grep '^{' "$out/stats_sec.log" | tail -1 > "$out/${tag}_bench_under_rocprof.json" || true
  if [ -f "$out/${tag}_bench.json" ]; then
    python3 tools/check_rooflines.py "$out/${tag}_bench.json" "$out/sum_sec" "$out/stats_sec/sec_results.db" > "$out/${tag}_roofline_check.txt" 2>&1
    cat "$out/${tag}_roofline_check.txt"
  fi
  python3 tools/check_rooflines.py "$out/${tag}_bench_under_rocprof.json" "$out/sum_sec" "$out/stats_sec/sec_results.db" --same-run > "$out/${tag}_roofline_check_traced_run.txt" 2>&1
  cat "$out/${tag}_roofline_check_traced_run.txt"
fi
pmc() {  # one config's PMC passes
  local name="$1"; shift
  timeout -k 10 300 python3 -u tools/pmc_traffic.py --tag "$tag" --outdir "$out/pmc_$name" "$@" > "$out/pmc_$name.log" 2>&1 || { tail -20 "$out/pmc_$name.log"; return 1; }
  cp "$out/pmc_$name"/*traffic*.json "$out/" && echo "pmc $name ok"
}
if [[ "$stages" == *p* ]]; then
  pmc c4 --log-n 28 --prec 64 || exit 1
  pmc c4f32 --log-n 28 --prec 32 || exit 1
  pmc c3 --log-n 12 --prec 32 --batch 4096 || exit 1
  pmc c1 --log-n 20 --prec 64 --workers 1 || exit 1
  pmc c2 --log-n 20 --prec 64 --workers 8 || exit 1
  pmc c2slice --log-n 20 --prec 64 --as-rank 0/8 || exit 1
fi
if [[ "$stages" == *p* || "$stages" == *q* ]]; then
  for g in 2 4 8; do
    pmc rank0of$g --log-n 28 --prec 64 --as-rank 0/$g || exit 1
  done
fi
ls "$out"/*traffic*.json 2>/dev/null || true
