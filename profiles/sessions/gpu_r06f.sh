# round 6, session f: the packed fp32 passes with LDS layouts from the bank
# model (tools/lds_model.hip now covers VPT 32; profiles/r06_lds_model_vpt32.txt):
# fp32 parity at full size and the fuzz, the A/B against the previous
# layouts (abvar/lds_old.so) on fp32 2^28 and 2^27, each pass against its copy
# again, and the LDS bank-conflict counters of both builds
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r06f
mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -k "f32 or fp32 or float" > $out/fp32_tests.txt 2>&1 && \
AB_ROUNDS=3 timeout -k 10 400 bash tools/ab.sh "--log-n 28 --prec 32 --steps 20 --warmup 5 --tune-ws 4" abvar/lds_old.so cs87project-msolano2_amd/libpifft.so > $out/ab_fp32_2e28.txt 2>&1 && \
AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh "--log-n 27 --prec 32 --steps 20 --warmup 5" abvar/lds_old.so cs87project-msolano2_amd/libpifft.so > $out/ab_fp32_2e27.txt 2>&1 && \
timeout -k 10 200 ./tools/probe_c4_passes_bin 3 > $out/c4_pass_ceilings.log 2>&1 && \
for v in old new; do
  lib=cs87project-msolano2_amd/libpifft.so; [ $v = old ] && lib=abvar/lds_old.so
  PIFFT_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $out/pmc_$v -o pmc -- python3 tools/tune.py --log-n 28 --prec 32 --steps 3 --warmup 1 > $out/pmc_$v.log 2>&1 || exit 1
  python3 tools/lds_pmc_summary.py $out/pmc_$v > $out/lds_conflicts_$v.txt 2>&1 || exit 1
done
