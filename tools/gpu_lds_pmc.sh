#!/bin/bash
# tools/gpu_lds_pmc.sh -- LDS counters of the pass kernels (one --pmc pass per
# plan, SQ block only): C4 and rank 0's plan of the 8-GPU job.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/lds
C="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/lds/c4 -o pmc -- \
    python -u bench.py --no-cpu-baseline --no-secondary --steps 2 --warmup 1 > gpurun_out/lds/c4.out 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d gpurun_out/lds/p8 -o pmc -- \
    python -u bench.py --no-cpu-baseline --no-secondary --as-rank 0/8 --steps 2 --warmup 1 > gpurun_out/lds/p8.out 2>&1 || exit 1
python3 tools/lds_pmc_summary.py gpurun_out/lds/c4 > gpurun_out/lds/summary.txt
python3 tools/lds_pmc_summary.py gpurun_out/lds/p8 >> gpurun_out/lds/summary.txt
cat gpurun_out/lds/summary.txt
