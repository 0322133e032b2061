#!/bin/bash
# tools/gpu_r04j.sh -- round-4 session j: the clean-loop roofline (bench tests,
# bench line, rocprofv3 check), the workgroup timeline of configs 1 / 2 / 2's
# slice (diagnostics build abvar2/wgclock.so, tools/wg_clock.py) and the
# slice's last pass at 8 values per thread (PIFFT_LAST_VPT / PIFFT_LAST_C).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r04j
mkdir -p "$out"
bash tools/gpu_r04.sh r04j tbs tests/test_bench.py tests/test_gpu_parity.py::test_launch_loop_times_and_restores_the_result || exit 1
for a in "--log-n 20" "--log-n 20 --workers 8 --count 1" "--log-n 20 --workers 8"; do
  PIFFT_LIB=abvar2/wgclock.so timeout -k 10 120 python3 -u tools/wg_clock.py $a >> "$out/wg_clock.txt" 2>&1 || { tail -20 "$out/wg_clock.txt"; exit 1; }
done
cat "$out/wg_clock.txt"
timeout -k 10 300 python3 -u tools/tune.py --log-n 20 --prec 64 --workers 8 --first 0 --count 1 --steps 200 --warmup 20 \
  --variants '[{}, {"PIFFT_LAST_VPT":"8"}, {"PIFFT_LAST_VPT":"8","PIFFT_LAST_C":"8"}, {"PIFFT_LAST_C":"8"}, {}, {"PIFFT_LAST_VPT":"8"}, {"PIFFT_LAST_VPT":"8","PIFFT_LAST_C":"8"}]' \
  > "$out/slice_last_vpt.log" 2>&1 || { tail -20 "$out/slice_last_vpt.log"; exit 1; }
cat "$out/slice_last_vpt.log"
