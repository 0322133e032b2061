#!/bin/bash
# A/B: natural-order store in the last pass of all-worker plans (PassArgs::ilv_log;
# PIFFT_ILV 0 never / 1 always / unset the planner rule) vs slice-major + interleave.
set -o pipefail
V='[{"PIFFT_ILV":0}, {"PIFFT_ILV":1}, {}, {"PIFFT_ILV":0}, {"PIFFT_ILV":1}, {}]'
run() { echo "== $1"; timeout -k 10 120 python tools/tune.py $1 --variants "$V" 2>&1 | grep -v amdgpu.ids | sed -e 's/ radix=.*wall/ wall/' | cut -c1-200 || exit 1; }
run "--log-n 16 --prec 64 --workers 8 --steps 100 --warmup 10"
run "--log-n 18 --prec 64 --workers 8 --steps 100 --warmup 10"
run "--log-n 20 --prec 64 --workers 8 --steps 100 --warmup 10"
run "--log-n 20 --prec 64 --workers 2 --steps 100 --warmup 10"
run "--log-n 20 --prec 64 --workers 16 --steps 100 --warmup 10"
run "--log-n 21 --prec 64 --workers 8 --steps 50 --warmup 5"
run "--log-n 22 --prec 64 --workers 8 --steps 50 --warmup 5"
run "--log-n 23 --prec 64 --workers 8 --steps 30 --warmup 5"
run "--log-n 24 --prec 64 --workers 8 --steps 20 --warmup 3"
run "--log-n 20 --prec 32 --workers 8 --steps 100 --warmup 10"
run "--log-n 22 --prec 32 --workers 8 --steps 50 --warmup 5"
run "--log-n 12 --prec 32 --batch 4096 --workers 4 --steps 50 --warmup 5"
run "--log-n 12 --prec 64 --batch 1024 --workers 4 --steps 50 --warmup 5"
