#!/bin/bash
# tools/gpu_r02h.sh -- HEAD evidence at the end of the round-2 session:
# tools/gpu_round2.sh (GPU tests, smoke, bench, rocprofv3 stats of the same
# command) + PMC HBM traffic of the C4 plan and of the 2-GPU rank plan (both
# with padded W), tag r02h.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_round2.sh r02h || exit 1
out=gpurun_out/r02h/pmc
mkdir -p "$out"
timeout -k 10 240 python -u tools/pmc_traffic.py --tag r02h --outdir "$out/p1" > "$out/p1.log" 2>&1 || { tail "$out/p1.log"; exit 1; }
timeout -k 10 240 python -u tools/pmc_traffic.py --tag r02h --outdir "$out/p2" --as-rank "0/2" > "$out/p2.log" 2>&1 || { tail "$out/p2.log"; exit 1; }
for g in 1 2; do python3 -c "
import json,glob
f=glob.glob('$out/p$g/r02h_traffic_*.json')[0]; d=json.load(open(f))
print(d['config_key'], [(k, round(v['fetch_bytes_corrected']+v['write_bytes']), v['algorithmic_bytes']) for k,v in d['kernels'].items()])"; done
