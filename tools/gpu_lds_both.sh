#!/bin/bash
# Historical: PIFFT_LDS_BOTH_MAX was removed after this A/B; kept as the record of how its log was taken.
# A/B of the both-components LDS exchange (PIFFT_LDS_BOTH_MAX) on the small
# configs and C4: tools/mkvariant.sh builds, copied to abvar/.
set -o pipefail
libs="abvar/base.so abvar/both40k.so abvar/both80k.so"
run() { echo "#### $1"; AB_ROUNDS=2 bash tools/ab.sh "$2" $libs || exit 1; }
run "fp32 4096 x 512 (C3 share of 8)" "--log-n 12 --prec 32 --batch 512 --steps 100 --warmup 10"
run "fp32 4096 x 4096 (C3)" "--log-n 12 --prec 32 --batch 4096 --steps 50 --warmup 5"
run "fp64 2^20 P=1 (C1)" "--log-n 20 --prec 64 --steps 100 --warmup 10"
run "fp64 2^20 P=8 (C2)" "--log-n 20 --prec 64 --workers 8 --steps 100 --warmup 10"
run "fp64 2^22 P=1" "--log-n 22 --prec 64 --steps 50 --warmup 5"
run "fp64 2^12 x 1024" "--log-n 12 --prec 64 --batch 1024 --steps 100 --warmup 10"
run "fp64 2^28 (C4)" "--log-n 28 --prec 64 --steps 5 --warmup 2"
