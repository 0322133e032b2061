#!/bin/bash
# tools/gpu_pmc_r02.sh -- PMC HBM traffic (FETCH_SIZE, WRITE_SIZE in separate
# passes) of the C4 plan and of one rank's plan of the 2/4/8-GPU jobs, round-2 kernels
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_r02
mkdir -p "$out"
timeout -k 10 240 python -u tools/pmc_traffic.py --tag r02 --outdir "$out/p1" > "$out/p1.log" 2>&1 || { tail "$out/p1.log"; exit 1; }
for g in 2 4 8; do
  timeout -k 10 240 python -u tools/pmc_traffic.py --tag r02 --outdir "$out/p$g" --as-rank "0/$g" > "$out/p$g.log" 2>&1 || { tail "$out/p$g.log"; exit 1; }
done
for g in 1 2 4 8; do python3 -c "
import json,glob
f=glob.glob('$out/p$g/r02_traffic_*.json')[0]; d=json.load(open(f))
print(d['config_key'], [(k, round(v['fetch_bytes_corrected']+v['write_bytes']), v['algorithmic_bytes']) for k,v in d['kernels'].items()])"; done
