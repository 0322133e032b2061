#!/bin/bash
# tools/ab.sh -- A/B per-launch timing of library variants on one box:
#   tools/ab.sh "<tune.py args>" variants/a.so variants/b.so ...
# runs tools/tune.py once per variant, twice round-robin (box drift shows).
set -o pipefail
args="$1"; shift
for round in $(seq 1 "${AB_ROUNDS:-2}"); do
  for lib in "$@"; do
    echo "== $lib (round $round)"
    PIFFT_LIB="$lib" timeout -k 10 120 python tools/tune.py $args 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
