#!/bin/bash
# tools/gpu_r03.sh <tag> [tests...] -- one GPU session of round-3 evidence:
#   0. the box's host share (cgroup CPU/memory limits, affinity)
#   1. the GPU tests given (default: the whole -m gpu suite)
#   2. bench.py as the driver runs it (C4 + secondary configs + CPU baselines
#      at the reference's p_to = 32)
#   3. rocprofv3 --kernel-trace --stats of bench.py with the secondary configs
#      (no CPU baselines), in the SAME session: every roofline in the line is
#      checked against it (tools/check_rooflines.py)
# Every GPU step has its own time limit; the first failure ends the job.
set -o pipefail
tag="${1:-r03}"
shift
tests="${*:-tests}"
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p "$out"
{ echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "memory.max: $(cat /sys/fs/cgroup/memory.max 2>/dev/null)";
  echo "nproc: $(nproc)"; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; } > "$out/host.txt"
cat "$out/host.txt"
if [ "$tests" != "none" ]; then
timeout -k 10 900 python -u -m pytest $tests -m gpu -x -v --timeout 200 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
tail -3 "$out/gpu_tests.log"
fi
timeout -k 10 900 python -u bench.py > "$out/bench.log" 2>&1 || { tail -20 "$out/bench.log"; exit 1; }
grep '^{' "$out/bench.log" > "$out/${tag}_bench.json" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$out/stats_sec" -o sec -- \
    python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$out/stats_sec.log" 2>&1 || exit 1
rocpd2summary -i "$out/stats_sec/sec_results.db" -f csv -d "$out/sum_sec" -o sec > /dev/null 2>&1 || exit 1
grep '^{' "$out/stats_sec.log" > "$out/${tag}_bench_under_rocprof.json" || true
python3 tools/check_rooflines.py "$out/${tag}_bench.json" "$out/sum_sec" "$out/stats_sec/sec_results.db" > "$out/${tag}_roofline_check.txt" 2>&1
cat "$out/${tag}_roofline_check.txt"
python3 tools/check_rooflines.py "$out/${tag}_bench_under_rocprof.json" "$out/sum_sec" "$out/stats_sec/sec_results.db" > "$out/${tag}_roofline_check_traced_run.txt" 2>&1
cat "$out/${tag}_roofline_check_traced_run.txt"
