#!/bin/bash
# tools/gpu_r05_tiny.sh [tag] -- round 5: (1) the small all-worker plan tests
# (one fused launch for P M <= 8192, the two-pass worker-interleaved plans),
# (2) the one-launch plan against the three-launch one (PIFFT_WIL_ONE_LAUNCH=0)
# over the reference's GPU sweep grid (n = 2^10-2^13, P = 2..16, both
# precisions), (3) the fused all-worker pass's tree twiddles (reference-formula
# table vs factored, PIFFT_WIL_TREE_MIN_LOG=0) at 2^16-2^20 -- outputs checked
# against each other (tools/tune.py --check).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05z}
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "tiny or single_pass_all_worker or fused_all_worker" > "$out/tests.txt" 2>&1 || { tail -40 "$out/tests.txt"; exit 1; }
tail -2 "$out/tests.txt"
V='[{}, {"PIFFT_WIL_ONE_LAUNCH":"0"}, {}, {"PIFFT_WIL_ONE_LAUNCH":"0"}]'
for prec in 64 32; do
  for n in 10 11 12 13; do
    for P in 2 4 8 16; do
      echo "=== fp$prec 2^$n P = $P" >> "$out/tiny.log"
      timeout -k 10 120 python3 -u tools/tune.py --log-n $n --prec $prec --workers $P --steps 2000 --warmup 500 --check \
        --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/tiny.log" || exit 1
    done
  done
done
V='[{}, {"PIFFT_WIL_TREE_MIN_LOG":"0"}, {}, {"PIFFT_WIL_TREE_MIN_LOG":"0"}]'
for prec in 64 32; do
  for n in 16 18 20; do
    for P in 2 8; do
      echo "=== fp$prec 2^$n P = $P" >> "$out/wiltw.log"
      timeout -k 10 120 python3 -u tools/tune.py --log-n $n --prec $prec --workers $P --steps 2000 --warmup 500 --check \
        --variants "$V" 2>&1 | grep -v amdgpu.ids >> "$out/wiltw.log" || exit 1
    done
  done
done
echo done
