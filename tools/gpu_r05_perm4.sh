#!/bin/bash
# tools/gpu_r05_perm4.sh [tag] -- round 5: the radix-4 cross-lane last stage
# (v_permlane32/16_swap) where it compiles spill-free (perm4_ok: <= 4 lines
# per workgroup or a plain first pass; abvar2/perm4.so, HEAD) against radix 2
# only (abvar2/base.so, the previous commit), on the shapes whose plans have
# such a 1024-point pass: config 1, fp32 2^20, batched 1024-point single
# passes, the fp32 fused 1024 passes; config 4 as the control.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05j}
mkdir -p "$out"
for shape in "--log-n 20 --prec 64 --workers 1 --steps 2000 --warmup 500" "--log-n 20 --prec 32 --workers 1 --steps 2000 --warmup 500" "--log-n 10 --prec 64 --batch 4096 --steps 1000 --warmup 200" "--log-n 10 --prec 32 --batch 8192 --steps 1000 --warmup 200" "--log-n 22 --prec 32 --workers 4 --first 1 --count 1 --steps 1000 --warmup 200" "--log-n 28 --prec 64 --steps 20 --warmup 5"; do
  echo "=== $shape" >> "$out/perm4.log"
  AB_ROUNDS=3 timeout -k 10 300 bash tools/ab.sh "$shape" abvar2/base.so abvar2/perm4.so >> "$out/perm4.log" 2>&1 || { tail -20 "$out/perm4.log"; exit 1; }
done
cat "$out/perm4.log"
