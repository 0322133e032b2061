#!/bin/bash
# tools/gpu_r03h.sh -- workspace placement tuning on fresh C4 allocation pairs
set -o pipefail
out=gpurun_out/r03h
mkdir -p "$out"
timeout -k 10 300 python -u tools/probe_wtune.py 28 8 4 > "$out/wtune.log" 2>&1 || { tail "$out/wtune.log"; exit 1; }
cat "$out/wtune.log"
