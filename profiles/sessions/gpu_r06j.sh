# round 6, session j: config 2's fused tree pass with the factored two-level
# tree twiddles (PIFFT_WIL_TREE_MIN_LOG=0: ~2 sqrt(N) table entries instead of
# the N (1 - 1/P)-entry reference-formula table read beside the data, 1.44x
# its algorithmic bytes) now that each level's lookups are fetched at once;
# outputs checked against the default plan's (tune.py --check)
set -o pipefail
out=gpurun_out/r06j
mkdir -p $out
for shape in "--log-n 20 --workers 8" "--log-n 19 --workers 8" "--log-n 20 --workers 4" "--log-n 20 --workers 2" "--log-n 18 --workers 8"; do
  timeout -k 10 200 python -u tools/tune.py $shape --steps 1000 --warmup 250 --check \
    --variants '[{}, {"PIFFT_WIL_TREE_MIN_LOG": "0"}, {}, {"PIFFT_WIL_TREE_MIN_LOG": "0"}]' >> $out/c2_factored_tree.txt 2>&1 || exit 1
done
