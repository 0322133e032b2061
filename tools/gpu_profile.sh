#!/bin/bash
# tools/gpu_profile.sh -- the measurement job behind profiles/<tag>_*:
#   1. bench.py as the driver runs it (N=1, C4) -> <tag>_bench.json
#   2. rocprofv3 --kernel-trace --stats of the same command -> per-kernel averages
#   3. PMC HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes) for C4 and for
#      one rank's plan of the 2/4/8-GPU jobs (bench.py --as-rank 0/G)
#   4. kernel stats of the 8-GPU rank plan
# Copied into profiles/ as <tag>_bench.json, <tag>_kernel_stats_*.csv, <tag>_traffic_*.json.
# Every GPU step has its own time limit; the first failure ends the job.
#   gpurun --timeout 1100 -- bash tools/gpu_profile.sh r01
set -o pipefail
tag="${1:-r01}"
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
mkdir -p "$out"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > "$out/bench.log" 2>&1 || exit 1
grep '^{' "$out/bench.log" > "$out/${tag}_bench.json" || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$out/stats_c4" -o c4 -- \
    python -u bench.py --no-cpu-baseline --steps 10 --warmup 3 > "$out/stats_c4.log" 2>&1 || exit 1
timeout -k 10 240 python -u tools/pmc_traffic.py --tag "$tag" --outdir "$out/pmc_p1" > "$out/pmc_p1.log" 2>&1 || exit 1
for g in 2 4 8; do
    timeout -k 10 240 python -u tools/pmc_traffic.py --tag "$tag" --outdir "$out/pmc_p$g" --as-rank "0/$g" \
        > "$out/pmc_p$g.log" 2>&1 || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$out/stats_p8" -o p8 -- \
    python -u bench.py --as-rank 0/8 --steps 10 --warmup 3 > "$out/stats_p8.log" 2>&1 || exit 1
# rocprofv3 writes a rocpd database; the per-kernel summary as CSV (no GPU use)
for t in c4 p8; do
    rocpd2summary -i "$out/stats_$t/${t}_results.db" -f csv -d "$out/sum_$t" -o "$t" > /dev/null 2>&1 || exit 1
done
cat "$out/${tag}_bench.json"
