# round 6, session l: the AMDGPU machine scheduler's strategies for the whole
# library (abvar/schedilp.so: -amdgpu-sched-strategy=max-ilp,
# abvar/schedmem.so: =max-memory-clause) against the product's default, on
# the BASELINE configs' plans
set -o pipefail
out=gpurun_out/r06l
mkdir -p $out
L="cs87project-msolano2_amd/libpifft.so abvar/schedilp.so abvar/schedmem.so"
AB_ROUNDS=2 timeout -k 10 400 bash tools/ab.sh "--log-n 28 --prec 32 --steps 20 --warmup 5 --tune-ws 4" $L > $out/ab_fp32_2e28.txt 2>&1 && \
AB_ROUNDS=2 timeout -k 10 400 bash tools/ab.sh "--log-n 28 --prec 64 --steps 20 --warmup 5 --tune-ws 4" $L > $out/ab_fp64_2e28.txt 2>&1 && \
AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh "--log-n 20 --prec 64 --steps 1000 --warmup 250" $L > $out/ab_c1.txt 2>&1 && \
AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh "--log-n 20 --prec 64 --workers 8 --steps 1000 --warmup 250" $L > $out/ab_c2.txt 2>&1 && \
AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh "--log-n 12 --prec 32 --batch 4096 --steps 200 --warmup 50" $L > $out/ab_c3.txt 2>&1
