#!/bin/bash
# tools/gpu_nt_sweep.sh -- non-temporal streaming (PIFFT_NT) on launches whose
# data fit the Infinity Cache: the kernel boundary writes back what a
# predecessor leaves dirty in L2 (MI355X_MICROARCH.md: + B / 6 TB/s)
set -o pipefail
mkdir -p gpurun_out/nt
V='[{"PIFFT_NT":"0"}, {"PIFFT_NT":"1"}, {"PIFFT_NT":"0"}, {"PIFFT_NT":"1"}]'
{
for ln in 16 18 20 22 24; do
  echo "== fp64 2^$ln P=1"
  timeout -k 10 120 python -u tools/tune.py --log-n $ln --prec 64 --steps 50 --warmup 10 --variants "$V" || exit 1
  echo "== fp64 2^$ln P=8 all workers"
  timeout -k 10 120 python -u tools/tune.py --log-n $ln --prec 64 --workers 8 --steps 50 --warmup 10 --variants "$V" || exit 1
  echo "== fp64 2^$ln worker 0 of 8"
  timeout -k 10 120 python -u tools/tune.py --log-n $ln --prec 64 --workers 8 --count 1 --steps 50 --warmup 10 --variants "$V" || exit 1
done
for b in 256 512 1024 2048 4096 8192; do
  echo "== fp32 4096 x $b"
  timeout -k 10 120 python -u tools/tune.py --log-n 12 --prec 32 --batch $b --steps 50 --warmup 10 --variants "$V" || exit 1
done
} > gpurun_out/nt/sweep.log 2>&1 || { tail -20 gpurun_out/nt/sweep.log; exit 1; }
grep -E "==|wall" gpurun_out/nt/sweep.log | sed 's/(sum of launches/(launches/; s/ :: .*//'
