#!/bin/bash
# tools/gpu_r05_p16.sh [tag] -- round 5: P = 16 fused all-worker plans (fp32 J
# = 4 at a 1024-point remainder, fp64 J = 2 at 32-64 MiB): the all-worker GPU
# tests, then each against the separate tree launch (PIFFT_WIL_FUSE=0) and the
# previous J, outputs checked against each other.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05p16}
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "fused_all_worker or single_pass_all_worker or tiny" > "$out/tests.txt" 2>&1 || { tail -40 "$out/tests.txt"; exit 1; }
tail -2 "$out/tests.txt"
V='[{}, {"PIFFT_WIL_FUSE":"0"}, {"PIFFT_WIL_FUSE_J":"8"}, {}, {"PIFFT_WIL_FUSE":"0"}, {"PIFFT_WIL_FUSE_J":"8"}]'
for s in "32 21 16 1" "64 21 16 1" "64 22 16 1" "64 20 16 2" "32 20 16 2"; do
  set -- $s
  echo "=== fp$1 2^$2 P = $3 batch $4" >> "$out/p16.log"
  timeout -k 10 120 python3 -u tools/tune.py --log-n $2 --prec $1 --workers $3 --batch $4 --steps 1000 --warmup 300 --check \
    --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/p16.log" || exit 1
done
echo done
