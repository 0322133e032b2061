#!/bin/bash
# tools/gpu_r05_c1_two_wg.sh [tag] -- round 5: the round-4 verdict's untried
# idea for config 1 (fp64 2^20, P = 1): two co-resident workgroups per CU (C = 2
# lines, 128 threads each: 512 workgroups, so one workgroup's HBM loads can
# overlap the other's LDS exchanges) against the default one workgroup of
# C = 4 per CU -- step times (tools/tune.py) and workgroup clocks
# (tools/wg_clock.py, diagnostics build).  Variants: tools/mk_c1_c2_variants.sh.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05r}
mkdir -p "$out"
C2='{"PIFFT_COL_C64":"2","PIFFT_STRIDED_CMIN":"2"}'
PIFFT_LIB=abvar2/c2x.so timeout -k 10 200 python3 -u tools/tune.py --log-n 20 --prec 64 --workers 1 --steps 2000 --warmup 500 --variants "[{}, $C2, {}, $C2, {}, $C2]" 2>&1 | grep -v amdgpu.ids > "$out/c1_two_wg.log" || exit 1
echo "== workgroup clocks, C = 4 (default)" >> "$out/c1_two_wg.log"
PIFFT_LIB=abvar2/c2xclock.so timeout -k 10 120 python3 -u tools/wg_clock.py --log-n 20 2>&1 | grep -v amdgpu.ids >> "$out/c1_two_wg.log" || exit 1
echo "== workgroup clocks, C = 2 (two workgroups per CU)" >> "$out/c1_two_wg.log"
PIFFT_TUNING=1 PIFFT_COL_C64=2 PIFFT_STRIDED_CMIN=2 PIFFT_LIB=abvar2/c2xclock.so timeout -k 10 120 python3 -u tools/wg_clock.py --log-n 20 2>&1 | grep -v amdgpu.ids >> "$out/c1_two_wg.log" || exit 1
cat "$out/c1_two_wg.log"
