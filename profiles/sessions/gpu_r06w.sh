# round 6, session w: what the LDS hand-offs between stages cost the
# latency-bound configs -- HEAD vs a timing-only build without them
# (PIFFT_DIAG_NO_XCHG=1: wrong results; the upper bound of any register
# exchange), A/B round robin
set -o pipefail
out=gpurun_out/r06w
mkdir -p $out
export AB_ROUNDS=3
tools/ab.sh "--log-n 20 --prec 64 --steps 300 --warmup 20" abvar/base.so abvar/noxchg.so > $out/c1.txt 2>&1 &&
tools/ab.sh "--log-n 20 --prec 64 --workers 8 --steps 300 --warmup 20" abvar/base.so abvar/noxchg.so > $out/c2.txt 2>&1 &&
tools/ab.sh "--log-n 20 --prec 64 --workers 8 --count 1 --steps 300 --warmup 20" abvar/base.so abvar/noxchg.so > $out/c2_slice.txt 2>&1 &&
tools/ab.sh "--log-n 12 --prec 32 --batch 4096 --steps 300 --warmup 20" abvar/base.so abvar/noxchg.so > $out/c3.txt 2>&1 &&
AB_ROUNDS=2 tools/ab.sh "--log-n 28 --prec 64 --steps 10 --warmup 3" abvar/base.so abvar/noxchg.so > $out/c4.txt 2>&1
