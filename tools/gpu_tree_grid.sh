set -o pipefail
V='[{}, {"PIFFT_TREE_GRID_DIV":"2"}, {"PIFFT_TREE_GRID_DIV":"4"}, {"PIFFT_TREE_GRID_DIV":"8"}, {"PIFFT_TREE_GRID_DIV":"16"}, {}]'
for spec in "--log-n 28 --workers 8" "--log-n 28 --workers 16" "--log-n 28 --workers 4" "--log-n 20 --workers 8" "--log-n 24 --workers 8"; do
  echo "== $spec"
  timeout -k 10 120 python -u tools/tune.py $spec --steps 10 --warmup 3 --variants "$V" | grep wall | sed 's/ radix.*:: tree/ tree/; s/ | pass.*//' || exit 1
done
