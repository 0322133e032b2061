#!/bin/bash
# tools/gpu_interleave_ab.sh -- slice-major -> natural order forms on MI355X:
# k_interleave (one thread per output), k_interleave_rows (P <= 16, one thread
# per k) and k_interleave_tile (LDS tile of all P slices x 2048/P k), as the
# last launch of all-worker plans; then the interleave/gather parity tests.
set -o pipefail
V='[{"PIFFT_INTERLEAVE_TILE_MIN64":"0","PIFFT_INTERLEAVE_TILE_MIN32":"0"},{"PIFFT_INTERLEAVE_TILE_MIN64":"1","PIFFT_INTERLEAVE_TILE_MIN32":"1"},{},{"PIFFT_INTERLEAVE_TILE_MIN64":"0","PIFFT_INTERLEAVE_TILE_MIN32":"0"},{"PIFFT_INTERLEAVE_TILE_MIN64":"1","PIFFT_INTERLEAVE_TILE_MIN32":"1"},{}]'
for spec in "--log-n 20 --workers 8" "--log-n 24 --workers 8" "--log-n 28 --workers 2" "--log-n 28 --workers 8" "--log-n 28 --workers 64" "--log-n 24 --workers 256" "--log-n 24 --prec 32 --workers 8" "--log-n 12 --prec 32 --batch 4096 --workers 64"; do
  echo "== $spec"
  timeout -k 10 120 python -u tools/tune.py $spec --steps 20 --warmup 5 --variants "$V" | grep wall | sed 's/ radix.*interleave/ interleave/' || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or allgather or group or batched or config or large_p or size_sweep" 2>&1 | tail -1
