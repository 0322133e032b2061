#!/bin/bash
# Historical: the -DPIFFT_SINGLE_WPE variant build was removed after this session.
# tools/gpu_r04f.sh -- round-4 session f: config 3's single pass built for 8
# waves per SIMD (abvar2/wpe8.so, -DPIFFT_SINGLE_WPE=8: 64 VGPRs, 8 workgroups
# per CU instead of 7 for its 16 per CU) vs the default build, then the HEAD
# evidence set (tools/gpu_r04.sh r04f tbs).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04f
mkdir -p "$out"
AB_ROUNDS=3 timeout -k 10 300 bash tools/ab.sh "--log-n 12 --prec 32 --batch 4096 --steps 400 --warmup 20" abvar2/base.so abvar2/wpe8.so > "$out/c3_wpe8.log" 2>&1 || { tail "$out/c3_wpe8.log"; exit 1; }
grep -v "^torch" "$out/c3_wpe8.log"
bash tools/gpu_r04.sh r04f tbs
