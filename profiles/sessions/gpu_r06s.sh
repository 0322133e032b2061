# round 6, session s: stage-twiddle prefetch (PIFFT_TW_PREFETCH=2) at HEAD on the
# latency-bound configs (C1, C2) and the streaming ones (C3, C4), A/B round robin
set -o pipefail
out=gpurun_out/r06s
mkdir -p $out
export AB_ROUNDS=3
tools/ab.sh "--log-n 20 --prec 64 --steps 200 --warmup 20" abvar/base.so abvar/twpre2.so > $out/c1.txt 2>&1 &&
tools/ab.sh "--log-n 20 --prec 64 --workers 8 --steps 200 --warmup 20" abvar/base.so abvar/twpre2.so > $out/c2.txt 2>&1 &&
tools/ab.sh "--log-n 12 --prec 32 --batch 4096 --steps 200 --warmup 20" abvar/base.so abvar/twpre2.so > $out/c3.txt 2>&1 &&
AB_ROUNDS=2 tools/ab.sh "--log-n 28 --prec 64 --steps 10 --warmup 3" abvar/base.so abvar/twpre2.so > $out/c4.txt 2>&1
