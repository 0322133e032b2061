# round 6, session m: the tree-twiddle fetch keeps the results bit for bit --
# the same plans through the round-5 kernels (abvar/r5kernels.so) and HEAD's,
# output SHA-256 compared
set -o pipefail
out=gpurun_out/r06m
mkdir -p $out
PIFFT_LIB=abvar/r5kernels.so timeout -k 10 200 python3 -u tools/bitwise_libs.py > $out/r5.txt 2>&1 && \
timeout -k 10 200 python3 -u tools/bitwise_libs.py > $out/head.txt 2>&1 && \
{ diff <(grep -v amdgpu $out/r5.txt | awk '{print $1,$2,$3,$4,$NF}') <(grep -v amdgpu $out/head.txt | awk '{print $1,$2,$3,$4,$NF}') > $out/diff.txt && echo "BITWISE EQUAL" >> $out/diff.txt || echo "DIFFER" >> $out/diff.txt; }
