# round 6, session q: config 5's per-GPU plan at HEAD -- worker 0 of the
# 8-way split of fp64 N = 2^32 (64 GiB replica) on one MI355X (--as-rank 0/8),
# and its PMC traffic (FETCH_SIZE / WRITE_SIZE passes) for the 8-GPU line
set -o pipefail
out=gpurun_out/r06q
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --log-n 32 --as-rank 0/8 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --detail $out/c5_rank0of8_detail.json > $out/c5_rank0of8.txt 2>&1 && \
timeout -k 10 600 python3 -u tools/pmc_traffic.py --tag r06q --outdir $out/pmc_c5 --log-n 32 --prec 64 --as-rank 0/8 > $out/pmc_c5.log 2>&1 && \
cp $out/pmc_c5/*traffic*.json $out/
