#!/bin/bash
# Historical in part: PIFFT_STRIDED_VPT was removed after this session; at HEAD that sweep runs the default.
# tools/gpu_r04c.sh -- round-4 session c: PMC traffic of the C4 / C4_f32 / C3
# plans (tools/gpu_r04.sh stage p), then A/B sweeps of the fp32 2^28 last pass
# (XCD tile grouping, streaming form, workspace row pad) and config 2's
# one-GPU slice with the tree unfused.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04c
mkdir -p "$out"
bash tools/gpu_r04.sh r04c p || exit 1
timeout -k 10 300 python3 -u tools/tune.py --log-n 28 --prec 32 --tune-ws 8 --steps 20 --variants \
  '[{}, {"PIFFT_LAST_XCD_GROUP": 0}, {"PIFFT_LAST_XCD_GROUP": 1}, {"PIFFT_LAST_XCD_GROUP": 3}, {"PIFFT_LAST_XCD_GROUP": 4}, {"PIFFT_LAST_NT": 0}, {"PIFFT_W_PAD": 0}, {"PIFFT_W_PAD": 1056}, {"PIFFT_W_PAD": 4128}, {}]' \
  > "$out/fp32_last_pass_sweep.log" 2>&1 || { tail "$out/fp32_last_pass_sweep.log"; exit 1; }
cat "$out/fp32_last_pass_sweep.log"
timeout -k 10 120 python3 -u tools/tune.py --log-n 20 --prec 64 --workers 8 --first 0 --count 1 --steps 200 --warmup 20 --variants \
  '[{}, {"PIFFT_FUSE_TREE": 0}, {}, {"PIFFT_FUSE_TREE": 0}]' > "$out/c2_slice_unfused.log" 2>&1 || { tail "$out/c2_slice_unfused.log"; exit 1; }
cat "$out/c2_slice_unfused.log"
# the radix-4 cross-lane last stage (v_permlane32/16_swap, PIFFT_PERMLANE=3) vs the default (radix 2 only)
AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh "--log-n 28 --prec 64 --tune-ws 8 --steps 20" abvar/base.so abvar/perm3.so > "$out/permlane4_c4.log" 2>&1 || { tail "$out/permlane4_c4.log"; exit 1; }
AB_ROUNDS=2 timeout -k 10 200 bash tools/ab.sh "--log-n 20 --prec 64 --steps 400 --warmup 20" abvar/base.so abvar/perm3.so > "$out/permlane4_c1.log" 2>&1 || { tail "$out/permlane4_c1.log"; exit 1; }
grep -v "^torch" "$out/permlane4_c4.log" "$out/permlane4_c1.log"
# strided passes at 8 values per thread (twice the waves) on the latency-bound 2^20 configs
timeout -k 10 120 python3 -u tools/tune.py --log-n 20 --prec 64 --steps 400 --warmup 20 --variants \
  '[{}, {"PIFFT_STRIDED_VPT": 8}, {}, {"PIFFT_STRIDED_VPT": 8}]' > "$out/vpt8_c1.log" 2>&1 || { tail "$out/vpt8_c1.log"; exit 1; }
timeout -k 10 120 python3 -u tools/tune.py --log-n 20 --prec 64 --workers 8 --first 0 --count 1 --steps 400 --warmup 20 --variants \
  '[{}, {"PIFFT_STRIDED_VPT": 8}, {}, {"PIFFT_STRIDED_VPT": 8}]' > "$out/vpt8_c2_slice.log" 2>&1 || { tail "$out/vpt8_c2_slice.log"; exit 1; }
grep -v "^torch" "$out/vpt8_c1.log" "$out/vpt8_c2_slice.log"
