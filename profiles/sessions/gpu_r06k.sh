# round 6, session k: the RCCL code path at the headline's full size on one
# GPU -- bench.py --pg --dist-backend nccl at fp64 2^28 (1-rank nccl group:
# the timed region, device all-reduce, all_gather_object, the self-check, the
# 4 GiB all_gather_into_tensor, configs 2 and 3 as the multi-GPU job runs them)
set -o pipefail
out=gpurun_out/r06k
mkdir -p $out
timeout -k 10 400 python -u bench.py --pg --dist-backend nccl --steps 20 --warmup 5 --no-cpu-baseline --detail $out/pg_nccl_detail.json > $out/pg_nccl.txt 2>&1
