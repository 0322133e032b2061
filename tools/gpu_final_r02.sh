#!/bin/bash
# tools/gpu_final_r02.sh -- the whole GPU suite (as the driver runs it), smoke
# and one default bench line at HEAD, end of the round-2 session.
set -o pipefail
out=gpurun_out/final
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$out/gpu_tests.log" 2>&1 || { tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { cat "$out/smoke.log"; exit 1; }
timeout -k 10 600 python -u bench.py > "$out/bench.log" 2>&1 || { tail -20 "$out/bench.log"; exit 1; }
grep '^{' "$out/bench.log" > "$out/bench.json"
python3 -c "
import json; d=json.load(open('$out/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], [l['ms'] for l in d['config']['launches']])"
