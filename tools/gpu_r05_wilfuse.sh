#!/bin/bash
# tools/gpu_r05_wilfuse.sh [tag] -- round 5: the all-worker tree fused into
# the first worker-interleaved pass (MODE 11).  First the parity tests of the
# all-worker plans (oracle + the unfused plan), then per-launch times of the
# fused plan (default), at J = 8 (PIFFT_WIL_FUSE_J) and with the tree as its
# own launch (PIFFT_WIL_FUSE=0), on config 2 and larger all-worker shapes.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05l}
mkdir -p "$out"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fused_all_worker or worker_interleaved or config2 or fuzz" > "$out/tests.log" 2>&1 || { tail -40 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"
V='[{}, {"PIFFT_WIL_FUSE_J":"8"}, {"PIFFT_WIL_FUSE":"0"}, {}, {"PIFFT_WIL_FUSE_J":"8"}, {"PIFFT_WIL_FUSE":"0"}]'
for shape in "--log-n 20 --prec 64 --workers 8 --steps 2000 --warmup 500" "--log-n 20 --prec 32 --workers 8 --steps 2000 --warmup 500" "--log-n 21 --prec 64 --workers 8 --steps 1000 --warmup 200" "--log-n 22 --prec 64 --workers 16 --steps 1000 --warmup 200" "--log-n 24 --prec 64 --workers 8 --steps 200 --warmup 50" "--log-n 28 --prec 64 --workers 8 --steps 20 --warmup 5" "--log-n 28 --prec 32 --workers 8 --steps 20 --warmup 5" "--log-n 26 --prec 64 --workers 4 --steps 50 --warmup 10"; do
  echo "=== $shape" >> "$out/wilfuse.log"
  timeout -k 10 300 python3 -u tools/tune.py $shape --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/wilfuse.log" || { tail -20 "$out/wilfuse.log"; exit 1; }
done
cat "$out/wilfuse.log"
