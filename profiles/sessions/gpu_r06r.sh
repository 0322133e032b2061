# round 6, session r: bench.py's multi-rank paths after the rank-0 rooflines
# gained their PMC traffic (the gloo rehearsals on one GPU, the RCCL
# world-size-1 run) -- tests/test_bench.py
set -o pipefail
out=gpurun_out/r06r
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_bench.py > $out/bench_tests.txt 2>&1
