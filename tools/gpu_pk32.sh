#!/bin/bash
# A/B of packed fp32 complex arithmetic (abvar/pk32.so) against the scalar
# forms (abvar/base.so): the fp32 configs, plus an fp64 control.
set -o pipefail
libs="abvar/base.so abvar/pk32.so"
run() { echo "#### $1"; AB_ROUNDS=2 bash tools/ab.sh "$2" $libs || exit 1; }
run "fp32 4096 x 512 (C3 share of 8)" "--log-n 12 --prec 32 --batch 512 --steps 100 --warmup 10"
run "fp32 4096 x 4096 (C3)" "--log-n 12 --prec 32 --batch 4096 --steps 50 --warmup 5"
run "fp32 2^20 P=1" "--log-n 20 --prec 32 --steps 100 --warmup 10"
run "fp32 2^24 P=8" "--log-n 24 --prec 32 --workers 8 --steps 30 --warmup 5"
run "fp32 2^28 P=1" "--log-n 28 --prec 32 --steps 5 --warmup 2"
run "fp64 2^20 P=1 (control)" "--log-n 20 --prec 64 --steps 100 --warmup 10"
