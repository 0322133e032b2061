# round 6, session y6: output hashes of one worker's slice plans (the
# one-worker fused tree pass, MODE 3) through the build before its stage-twiddle
# prefetch (abvar/base.so) and HEAD's (abvar/head.so)
set -o pipefail
out=gpurun_out/r06y6
mkdir -p $out
for v in base head; do
  PIFFT_LIB=abvar/$v.so timeout -k 10 120 python tools/bitwise_libs.py --set slice > $out/bitwise_slice_$v.txt 2>&1 || exit 1
done
