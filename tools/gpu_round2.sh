#!/bin/bash
# tools/gpu_round2.sh <tag> -- one GPU session of round-2 evidence:
#   1. the GPU test suite (new full-size / gather / sweep tests first)
#   2. smoke()
#   3. bench.py as the driver runs it (C4 + secondary configs + CPU baselines)
#   4. rocprofv3 --kernel-trace --stats of the headline bench command, in the
#      SAME session, so the line's roofline.frac can be checked against it
# Every GPU step has its own time limit; the first failure ends the job.
set -o pipefail
tag="${1:-r02}"
export TMPDIR=/tmp
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_bench.py tests -m gpu -x -v \
    --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -40 "$out/gpu_tests.log"; exit 1; }
tail -3 "$out/gpu_tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { cat "$out/smoke.log"; exit 1; }
timeout -k 10 900 python -u bench.py > "$out/bench.log" 2>&1 || { tail -20 "$out/bench.log"; exit 1; }
grep '^{' "$out/bench.log" > "$out/${tag}_bench.json" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/stats_c4" -o c4 -- \
    python3 -u bench.py --no-cpu-baseline --no-secondary --steps 10 --warmup 3 > "$out/stats_c4.log" 2>&1 || exit 1
rocpd2summary -i "$out/stats_c4/c4_results.db" -f csv -d "$out/sum_c4" -o c4 > /dev/null 2>&1 || exit 1
grep '^{' "$out/stats_c4.log" > "$out/${tag}_bench_under_rocprof.json" || true
cat "$out/sum_c4/"*.csv | head -8
python3 tools/rocpd_timed_avg.py "$out/stats_c4/c4_results.db" 10 "$out/${tag}_kernel_timed_avg.csv" || exit 1
cat "$out/${tag}_kernel_timed_avg.csv"
# the secondary configs' kernels (C1, C2, C2 slice, C3) under the same trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/stats_sec" -o sec -- \
    python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > "$out/stats_sec.log" 2>&1 || exit 1
rocpd2summary -i "$out/stats_sec/sec_results.db" -f csv -d "$out/sum_sec" -o sec > /dev/null 2>&1 || exit 1
cat "$out/sum_sec/"*.csv | head -16
