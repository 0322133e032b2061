# round 6, session g: where the packed fp32 MODE 2 passes' 5-7 % over their
# copies goes -- the C4 pass probe built four ways (timing only, WRONG
# results): the kernel as is, without twiddles (PIFFT_DIAG_NO_TW), without
# butterflies (PIFFT_DIAG_NO_DFT), without both (data movement + the LDS
# exchanges only)
set -o pipefail
out=gpurun_out/r06g
mkdir -p $out
for b in "" _dnotw _dnodft _dnotwdnodft; do
  echo "== probe_c4_passes_bin$b" >> $out/fp32_diag.log
  timeout -k 10 200 ./tools/probe_c4_passes_bin$b 2 >> $out/fp32_diag.log 2>&1 || exit 1
done
