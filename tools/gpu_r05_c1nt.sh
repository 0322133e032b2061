#!/bin/bash
# tools/gpu_r05_c1nt.sh [tag] -- round 5: config 1's last pass
# (k_pass<double,1024,4,2,1,0,16>, 64-B row segments) writes 1.30x its
# algorithmic bytes with non-temporal stores (profiles/r05b_traffic_n2^20_f64_
# b1_P1_q1.json).  Its streaming forms by time (tools/tune.py, 4 rounds) and
# by PMC bytes (tools/pmc_traffic.py with PIFFT_LAST_NT=0: plain loads and
# stores; default 1: non-temporal both -- the only two forms instantiated).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r05f}
mkdir -p "$out"
timeout -k 10 200 python3 -u tools/tune.py --log-n 20 --prec 64 --workers 1 --steps 2000 --warmup 500 --variants '[{}, {"PIFFT_LAST_NT":"0"}, {}, {"PIFFT_LAST_NT":"0"}, {}, {"PIFFT_LAST_NT":"0"}]' 2>&1 | grep -v "amdgpu.ids" > "$out/c1_nt.log" || exit 1
for v in 0; do
  PIFFT_TUNING=1 PIFFT_LAST_NT=$v timeout -k 10 200 python3 -u tools/pmc_traffic.py --tag "${1:-r05f}_lastnt$v" --outdir "$out/pmc_nt$v" --log-n 20 --prec 64 --workers 1 > "$out/pmc_nt$v.log" 2>&1 || { tail -20 "$out/pmc_nt$v.log"; exit 1; }
  cp "$out/pmc_nt$v"/*traffic*.json "$out/"
done
cat "$out/c1_nt.log"
