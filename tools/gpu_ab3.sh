set -o pipefail
mkdir -p gpurun_out
AB_ROUNDS=3 timeout -k 10 400 bash tools/ab.sh "--log-n 28 --prec 64" variants/pre_chunk.so variants/perm0.so variants/cur.so > gpurun_out/ab3_c4.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/ab3_c4.log | cut -c1-200
