#!/bin/bash
# tools/gpu_r05_sweep.sh [tag] -- round 5: the reference's experiment sweeps
#  re-run on MI355X after this round's small all-worker
# plans (one fused launch up to 8192 values, two launches from 2^11 points
# per worker): the reference's CUDA grid (cuda/run-experiments:16-17, n =
# 2^10-2^13, p = 1-32), its pthreads/Xeon Phi range (n = 2^11-2^17) and the
# larger one (2^20-2^24), each with the cost-law fits of analyze-results.R.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05s}
mkdir -p "$out"
S=cs87project-msolano2_amd/pifft_sweep.py
B=cs87project-msolano2_amd/pifft
timeout -k 10 400 python3 -u $S run --bin $B --T 3 --n-from 1024 --n-to 8192 --p-from 1 --p-to 32 --out "$out/sweep_cuda_grid.tsv" || exit 1
timeout -k 10 400 python3 -u $S run --bin $B --T 3 --n-from 2048 --n-to 131072 --p-from 1 --p-to 32 --out "$out/sweep_ref_range.tsv" || exit 1
timeout -k 10 400 python3 -u $S run --bin $B --T 3 --n-from 1048576 --n-to 16777216 --p-from 1 --p-to 32 --out "$out/sweep_large.tsv" || exit 1
for f in sweep_cuda_grid sweep_ref_range sweep_large; do
  python3 $S analyze "$out/$f.tsv" > "$out/${f}_analysis.txt" || exit 1
done
cat "$out"/*_analysis.txt
