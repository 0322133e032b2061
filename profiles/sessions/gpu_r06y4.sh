# round 6, session y4: config 3 (fp32 4096 x 4096) as a packed VPT-32 single
# pass (128 threads per transform, 128 VGPRs: 8 workgroups per CU, so 16
# transforms per CU run in exactly two rounds) against HEAD's VPT-16 pass (6
# per CU, 2.67 rounds); experiment library abvar/c3pk.so, output compared
set -o pipefail
out=gpurun_out/r06y4
mkdir -p $out
V='[{}, {"PIFFT_SINGLE_VPT":"32"}]'
for r in 1 2 3; do
  PIFFT_LIB=abvar/c3pk.so PIFFT_TUNING=1 timeout -k 10 120 python tools/tune.py --log-n 12 --prec 32 --batch 4096 --steps 300 --warmup 20 --variants "$V" --check >> $out/c3.txt 2>&1 || exit 1
done
for b in 512 1024 8192; do
  PIFFT_LIB=abvar/c3pk.so PIFFT_TUNING=1 timeout -k 10 120 python tools/tune.py --log-n 12 --prec 32 --batch $b --steps 300 --warmup 20 --variants "$V" --check >> $out/f32_4096_b$b.txt 2>&1 || exit 1
done
