#!/bin/bash
# tools/gpu_r04h.sh -- round-4 session h: the driver's multi-GPU bench lines at
# full headline size, rehearsed with gloo ranks on one GPU (--same-device):
# every worker split checks itself (config.verify); config 5 refuses cleanly
# (its 2^32 replicas do not fit 8 ranks on one GPU).  Then the C host's split
# check at 2^24 (pifft -t -g 8 -R).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-r04h}
mkdir -p "$out"
timeout -k 10 600 python3 -u bench.py --gpus 8 --same-device --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > "$out/bench_g8_rehearsal.log" 2>&1 || { tail -30 "$out/bench_g8_rehearsal.log"; exit 1; }
grep '^{' "$out/bench_g8_rehearsal.log" > "$out/r04h_bench_g8_rehearsal.json" || exit 1
timeout -k 10 300 python3 -u bench.py --gpus 2 --same-device --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > "$out/bench_g2_rehearsal.log" 2>&1 || { tail -30 "$out/bench_g2_rehearsal.log"; exit 1; }
grep '^{' "$out/bench_g2_rehearsal.log" > "$out/r04h_bench_g2_rehearsal.json" || exit 1
python3 - "$out" <<'PY'
import json, sys
for g in (8, 2):
    d = json.load(open(f"{sys.argv[1]}/r04h_bench_g{g}_rehearsal.json"))
    print(g, "ranks: value", d["value"], "verify", json.dumps(d["config"]["verify"]))
    for k, v in d["config"]["secondary"].items():
        print("  ", k, "error" in v and v["error"][:120], json.dumps(v.get("verify")))
PY
timeout -k 10 120 cs87project-msolano2_amd/pifft -t -n 16777216 -p 8 -g 8 -R -f 64 > "$out/cli_split_check_2e24.log" 2>&1 || exit 1
grep -E "Split check" "$out/cli_split_check_2e24.log"
# (keep what merges back under gpurun's 64-MiB limit: the lines and summaries, the logs' tails)
for f in "$out"/*.log; do tail -c 100000 "$f" > "$f.tail" && mv "$f.tail" "$f"; done
