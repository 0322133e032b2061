#!/bin/bash
# tools/gpu_r03v.sh -- round-3 session v: (1) the new 1024-point last pass with
# two sub-tiles per workgroup (PIFFT_SUBTILES_LAST=2: 256-B effective row
# segments, one workgroup per CU), tuned workspaces, alternating; (2) PMC HBM
# traffic of the new 2^28 plan (FETCH_SIZE / WRITE_SIZE in separate passes,
# tools/pmc_traffic.py); (3) the evidence session (bench + rocprofv3 check)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r03v
mkdir -p "$out"
V='[{}, {"PIFFT_SUBTILES_LAST":"2"}, {}, {"PIFFT_SUBTILES_LAST":"2"}, {}, {"PIFFT_SUBTILES_LAST":"2"}]'
{ echo "=== fp64 2^28, tuned workspace (4)"; timeout -k 10 400 python -u tools/tune.py --log-n 28 --prec 64 --steps 20 --warmup 3 --tune-ws 4 --variants "$V"; } > "$out/sub_last.log" 2>&1 || { tail "$out/sub_last.log"; exit 1; }
grep -E "===|wall" "$out/sub_last.log"
timeout -k 10 400 python tools/pmc_traffic.py --tag r03v --steps 3 --outdir gpurun_out/r03v/pmc > "$out/pmc.log" 2>&1 || { tail -20 "$out/pmc.log"; exit 1; }
grep -E '"kernel"|per_launch|"[0-9]": [0-9]' "$out/pmc.log" | head -12
bash tools/gpu_r03.sh r03v none
