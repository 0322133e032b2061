# round 6, session v: per-workgroup clocks of config 3's single pass (fp32
# 4096 x 4096) and config 1 at HEAD (diagnostics build abvar/wgclock.so)
set -o pipefail
out=gpurun_out/r06v
mkdir -p $out
PIFFT_LIB=abvar/wgclock.so timeout -k 10 120 python tools/wg_clock.py --log-n 12 --prec 32 --batch 4096 --dump $out/c3_dump.csv > $out/wg_clock_c3.txt 2>&1 &&
PIFFT_LIB=abvar/wgclock.so timeout -k 10 120 python tools/wg_clock.py --log-n 20 --prec 64 > $out/wg_clock_c1.txt 2>&1
