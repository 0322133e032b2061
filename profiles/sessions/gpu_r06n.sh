# round 6, session n: the packed fp32 MODE 2 first stage with the inter-pass
# base factor folded into the powers (abvar/pkfold.so, PIFFT_PK_FOLD=1: 31
# instead of 42 complex products per butterfly) -- A/B on fp32 2^28 / 2^27 and
# the fp32 parity tests through that build
set -o pipefail
out=gpurun_out/r06n
mkdir -p $out
AB_ROUNDS=3 timeout -k 10 400 bash tools/ab.sh "--log-n 28 --prec 32 --steps 20 --warmup 5 --tune-ws 4" cs87project-msolano2_amd/libpifft.so abvar/pkfold.so > $out/ab_fp32_2e28.txt 2>&1 && \
AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh "--log-n 27 --prec 32 --steps 20 --warmup 5" cs87project-msolano2_amd/libpifft.so abvar/pkfold.so > $out/ab_fp32_2e27.txt 2>&1 && \
PIFFT_LIB=$PWD/abvar/pkfold.so timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -k "f32 or fp32 or float" > $out/fp32_tests_pkfold.txt 2>&1
