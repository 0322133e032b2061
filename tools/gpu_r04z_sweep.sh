#!/bin/bash
# tools/gpu_r04z_sweep.sh -- round-4 session z: the reference's experiment
# sweep (run-experiments-and-analyze-results:27-69) run
# with the MI355X CLI on one GPU -- the reference's own ranges (n = 2^11 ..
# 2^17, p = 1 .. 32, its data_t fp32) and a larger one (n = 2^20 .. 2^24) --
# then the cost-law fits of analyze-results.R:31-83 (pifft_sweep.py analyze).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r04z}
mkdir -p "$out"
S=cs87project-msolano2_amd/pifft_sweep.py
B=cs87project-msolano2_amd/pifft
timeout -k 10 400 python3 -u $S run --bin $B --T 3 --n-from 2048 --n-to 131072 --p-from 1 --p-to 32 --out "$out/sweep_ref_range.tsv" || exit 1
timeout -k 10 400 python3 -u $S run --bin $B --T 3 --n-from 1048576 --n-to 16777216 --p-from 1 --p-to 32 --out "$out/sweep_large.tsv" || exit 1
python3 $S analyze "$out/sweep_ref_range.tsv" > "$out/sweep_ref_range_analysis.txt" || exit 1
python3 $S analyze "$out/sweep_large.tsv" > "$out/sweep_large_analysis.txt" || exit 1
cat "$out/sweep_ref_range_analysis.txt" "$out/sweep_large_analysis.txt"
