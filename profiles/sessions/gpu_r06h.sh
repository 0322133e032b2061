# round 6, session h: the packed fp32 passes' schedule -- a scheduling barrier
# after each butterfly pair (abvar/pkser.so, PIFFT_PK_SERIAL=1), the LDS
# addresses kept instead of recomputed per component (abvar/pkremat0.so,
# PIFFT_PK_REMAT=0) -- against the product on fp32 2^28 and 2^27
set -o pipefail
out=gpurun_out/r06h
mkdir -p $out
AB_ROUNDS=3 timeout -k 10 500 bash tools/ab.sh "--log-n 28 --prec 32 --steps 20 --warmup 5 --tune-ws 4" cs87project-msolano2_amd/libpifft.so abvar/pkser.so abvar/pkremat0.so > $out/ab_fp32_sched_2e28.txt 2>&1 && \
AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh "--log-n 27 --prec 32 --steps 20 --warmup 5" cs87project-msolano2_amd/libpifft.so abvar/pkser.so abvar/pkremat0.so > $out/ab_fp32_sched_2e27.txt 2>&1
