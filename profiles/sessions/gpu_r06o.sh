# round 6, session o: bench.py exactly as the driver runs it at N = 1 (the
# headline line with the reference's -O0 build beside the -O2 one)
set -o pipefail
out=gpurun_out/r06o
mkdir -p $out
s=$(date +%s); timeout -k 10 600 python -u bench.py --detail $out/r06o_bench_detail.json > $out/bench.log 2>&1; rc=$?; echo "wall $(( $(date +%s) - s )) s rc $rc" >> $out/bench.log; exit $rc
