#!/bin/bash
# tools/gpu_r04t.sh -- round-4 session t: the fused tree pass of small slices
# with 32 leaf loads in flight per thread and round (PIFFT_TREE_LOADS_SMALL=32,
# build abvar2/tl32.so) instead of 16: half the dependent load rounds.
# Parity under the variant first, then A/B against the in-tree library.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04t
mkdir -p "$out"
PIFFT_LIB=abvar2/tl32.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "slice_last_pass_forms or fused_tree_first_pass" -m gpu -x -q --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for a in "--log-n 20 --workers 8" "--log-n 19 --workers 8" "--log-n 21 --workers 8" "--log-n 18 --workers 4" "--log-n 21 --workers 16" "--log-n 20 --workers 2"; do
  for lib in "" abvar2/tl32.so "" abvar2/tl32.so; do
    PIFFT_LIB=$lib timeout -k 10 120 python3 -u tools/tune.py $a --prec 64 --first 0 --count 1 --steps 1000 --warmup 200 --variants '[{}]' 2>&1 | grep -v "amdgpu.ids\|torch copy" | sed "s|^|$a lib=${lib:-default} |" >> "$out/tl32.log" || exit 1
  done
done
cat "$out/tl32.log"
