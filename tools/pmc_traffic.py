#!/usr/bin/env python3
"""tools/pmc_traffic.py -- HBM traffic per launch from rocprofv3 PMC counters.

Recipe (MI355X_MICROARCH.md, HBM / rocprofv3 PMC slots):
  * FETCH_SIZE and WRITE_SIZE (units: KiB) do not fit in one TCC pass, so each
    is collected in its own `rocprofv3 --pmc` run (no tracing options beside
    --pmc);
  * gfx950 correction: FETCH_SIZE reports exactly half of the bytes of a wide
    (16 B/lane) coalesced streaming read -> x2 for the fp64 kernels here;
    WRITE_SIZE is exact for 16 B/lane streaming stores.  The fp32 kernels'
    8 B/lane reads are calibrated on the fp32 2^28 plan (round 4,
    profiles/r04c_traffic_n2^28_f32_b1_P1_q1.json): each pass streams 2 GiB in,
    8x the Infinity Cache, so every input byte must come from memory at least
    once, yet raw FETCH_SIZE is 0.500x those bytes in all three passes -- the
    same half count -> x2 as well (WRITE_SIZE: 1.000x, exact).

Runs bench.py under each counter pass, finds every full execution of the
plan among the dispatches (its launches in order, by the kernel names the
bench line records -- bench.py's single-kernel roofline loops are left out),
averages each launch over them, and writes profiles/<tag>_traffic.json,
which bench.py reads for roofline.traffic.  (Round 4, r04w: the earlier
"last steps x launches dispatches" rule took the roofline loops' dispatches
once bench.py added them.)

usage: python tools/pmc_traffic.py --tag r01 [bench.py args...]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OURS = ("k_pass", "k_tree", "k_interleave")


def run_pass(counter: str, outdir: str, bench_args: list[str]) -> tuple[list[dict], dict]:
    """rocprofv3 --pmc <counter> -- python bench.py ...; returns (rows, bench JSON line).
    This process never touches the GPU (rocprofv3 and bench.py are children)."""
    os.makedirs(outdir, exist_ok=True)
    side = os.path.join(outdir, "bench_detail.json")
    cmd = ["rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", outdir, "-o", "pmc", "--",
           sys.executable, os.path.join(ROOT, "bench.py")] + bench_args + ["--detail", side]
    r = subprocess.run(cmd, check=True, cwd=ROOT, stdout=subprocess.PIPE, text=True)
    if not any(ln.startswith("{") and '"metric"' in ln for ln in r.stdout.splitlines()):
        raise SystemExit("bench.py printed no JSON line")
    with open(side) as f:  # the full record (per-launch bytes and kernel names): bench.py's sidecar
        line = json.load(f)
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {outdir}")
    rows = []
    for f in files:
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows, line


def per_dispatch(rows: list[dict], counter: str) -> list[tuple[int, str, float]]:
    acc: dict[int, list] = {}
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        did = int(r.get("Dispatch_Id", r.get("Correlation_Id", 0)))
        name = r.get("Kernel_Name", "")
        v = float(r.get("Counter_Value", 0.0))
        if did in acc:
            acc[did][1] += v
        else:
            acc[did] = [name, v]
    return [(d, acc[d][0], acc[d][1]) for d in sorted(acc)]


def correction(prec: int) -> str:
    return ("FETCH_SIZE KiB x1024 x2 (gfx950 16 B/lane streaming read), WRITE_SIZE KiB x1024" if prec == 64 else
            "FETCH_SIZE KiB x1024 x2 (gfx950 8 B/lane streaming read: half-counted, calibrated on the fp32 2^28 "
            "passes -- raw 0.500x the compulsory bytes of a stream 8x the Infinity Cache), WRITE_SIZE KiB x1024")


def recorrect(path: str, out: str) -> None:
    """Rewrites a summary with the current correction (the raw counter values
    are kept in every summary)."""
    d = json.load(open(path))
    prec = int(d["config_key"].split("_f")[1].split("_")[0])
    for i, k in d["kernels"].items():
        k["fetch_bytes_corrected"] = k["FETCH_SIZE_KiB"] * 1024 * 2
        k["write_bytes"] = k["WRITE_SIZE_KiB"] * 1024
        d["per_launch_bytes"][i] = k["fetch_bytes_corrected"] + k["write_bytes"]
    d["correction"] = correction(prec)
    with open(out, "w") as f:
        json.dump(d, f, indent=1)


def main() -> None:
    if len(sys.argv) == 4 and sys.argv[1] == "--recorrect":
        return recorrect(sys.argv[2], sys.argv[3])
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--outdir", default=os.path.join(ROOT, "gpurun_out", "pmc"))
    args, rest = ap.parse_known_args()
    bench_args = ["--steps", str(args.steps), "--warmup", "1", "--no-cpu-baseline", "--no-secondary"] + rest

    ba = argparse.ArgumentParser()
    ba.add_argument("--prec", type=int, default=64)
    b, _ = ba.parse_known_args(rest)
    result = {"counters": {}, "kernels": {}}
    per_launch = defaultdict(dict)
    line = None
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        rows, line = run_pass(counter, os.path.join(args.outdir, counter.lower()), bench_args)
        launches = line["config"]["launches"]
        nl = len(launches)
        disp = [d for d in per_dispatch(rows, counter) if any(o in d[1] for o in OURS)]
        names = line["config"].get("kernel_names")
        if names:
            # every full execution of the plan: nl consecutive dispatches with
            # the plan's kernels in order (workspace tuning, warm-up, timed and
            # profiling loops; not bench.py's single-kernel roofline loops)
            execs, i = [], 0
            while i + nl <= len(disp):
                if all(disp[i + j][1] == names[j] for j in range(nl)):
                    execs.append(disp[i:i + nl])
                    i += nl
                else:
                    i += 1
            if not execs:
                raise SystemExit(f"no full execution of {names} among {len(disp)} dispatches")
        else:  # (lines before round 4: the timed loop is the tail)
            tail = disp[-args.steps * nl:]
            execs = [tail[s * nl:(s + 1) * nl] for s in range(len(tail) // nl)]
        for i in range(nl):
            vals = [e[i][2] for e in execs]
            per_launch[i][counter] = sum(vals) / len(vals)
            per_launch[i]["kernel"] = execs[-1][i][1]
        per_launch[0].setdefault("executions", {})[counter] = len(execs)
        result["counters"][counter] = len(disp)
    cfg = line["config"]
    key = f"n2^{cfg['n'].bit_length() - 1}_f{b.prec}_b{cfg['batch']}_P{cfg['workers']}_q{cfg['workers_per_gpu']}"
    result["config_key"] = key
    result["executions_averaged"] = per_launch[0].get("executions")
    result["bench_line"] = line
    nl = len(cfg["launches"])
    launch_bytes = [l.get("bytes") for l in cfg["launches"]]
    out = {}
    for i in range(nl):
        f_kib = per_launch[i].get("FETCH_SIZE", 0.0)
        w_kib = per_launch[i].get("WRITE_SIZE", 0.0)
        fetch = f_kib * 1024 * 2
        write = w_kib * 1024
        out[str(i)] = fetch + write
        result["kernels"][str(i)] = {"kernel": per_launch[i]["kernel"], "FETCH_SIZE_KiB": f_kib,
                                     "WRITE_SIZE_KiB": w_kib, "fetch_bytes_corrected": fetch,
                                     "write_bytes": write, "algorithmic_bytes": launch_bytes[i]}
    result["per_launch_bytes"] = out
    result["correction"] = correction(b.prec)
    # written under gpurun_out/ (merged back from the GPU box); copy into profiles/ to commit
    os.makedirs(args.outdir, exist_ok=True)
    path = os.path.join(args.outdir, f"{args.tag}_traffic_{key}.json")
    with open(path, "w") as f:
        json.dump(result, f, indent=1)
    print(json.dumps(result, indent=1))


if __name__ == "__main__":
    main()
