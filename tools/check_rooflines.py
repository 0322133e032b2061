#!/usr/bin/env python3
"""tools/check_rooflines.py <bench.json> <rocpd2summary dir> <rocpd .db> --
checks every roofline of a bench line against rocprofv3 --kernel-trace of the
same bench command in the same session (tools/gpu_r03.sh).

The traced run executes the configs in bench.py's order (headline, then the
secondary configs).  Dispatches are split into one cluster per config at each
input generation (k_generate: every config's Job starts with one; its warm-up,
timed and clean loops follow).  For each roofline the dominant kernel (by the
demangled name bench.py records, pifft_plan_kernel_name) is averaged over its
cluster's back-to-back dispatches (those starting within BACK_TO_BACK_US of the
previous dispatch's end: the timed loop's context) and over all dispatches of
that name (what --stats prints); the bench line's mean launch time is compared
with the first.
Done when every frac is within 3 % of rocprof's."""
import csv
import glob
import json
import os
import sqlite3
import sys

TOL = 0.03
BACK_TO_BACK_US = 2.0


def rooflines(line):
    """(config key, roofline dict, step ms) of the line, in bench.py's order."""
    out = [("headline", line["roofline"], line["ms_per_step"])]
    sec = (line.get("config") or {}).get("secondary") or {}
    for key, rec in sec.items():
        rf = rec.get("roofline") or rec.get("roofline_rank0")
        if rf:
            out.append((key, rf, rec.get("ms_per_step")))
    return out


def main():
    line = json.loads(open(sys.argv[1]).read().strip().splitlines()[0])
    stats = {}
    for f in glob.glob(os.path.join(sys.argv[2], "**", "*kernel*s*.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            avg = r.get("AverageNs") or r.get("Average (Nsec)")
            stats[r["Name"]] = (int(r["Calls"]), float(avg) * 1e-6)
    con = sqlite3.connect(sys.argv[3])
    clusters, last_end = [], None
    for n, s, e in con.execute("select name, start, end from kernels order by start"):
        gap = (s - last_end) * 1e-3 if last_end is not None else 1e9  # us since the previous dispatch ended
        last_end = e
        if "k_generate" in n:  # every config (bench.py Job) starts by generating its input
            clusters.append([])
        elif clusters:
            clusters[-1].append((n, (e - s) * 1e-6, gap))
    rfs = rooflines(line)
    print(f"{len(clusters)} dispatch clusters in the trace, {len(rfs)} rooflines in the line")
    worst, ok = 0.0, True
    print(f"{'config':10s} {'bench ms':>10s} {'trace ms':>10s} {'stats ms':>10s} {'frac':>7s} {'frac(tr)':>8s} "
          f"{'diff':>7s}  kernel")
    for i, (key, rf, step_ms) in enumerate(rfs):
        name = rf.get("kernel_name")
        if rf.get("frac") is None or not name:
            print(f"{key:10s} no frac in the line: {rf.get('error', 'no kernel name')}")
            ok = False
            continue
        cl = clusters[i] if i < len(clusters) else []
        # back-to-back dispatches only (the timed loop's context; a dispatch
        # after one with bound events starts ~9 us late, isolated)
        durs = [d for n, d, gap in cl if n == name and gap < BACK_TO_BACK_US]
        tr = sum(durs) / len(durs) if durs else None
        st = stats.get(name, (0, None))[1]
        ref = tr if tr is not None else st
        if ref is None:
            print(f"{key:10s} kernel not in the trace: {name}")
            ok = False
            continue
        frac_tr = rf["algorithmic_bytes"] / (ref * 1e-3) / 1e9 / rf["peak"]
        diff = rf["frac"] / frac_tr - 1.0
        worst = max(worst, abs(diff))
        ok = ok and abs(diff) <= TOL
        print(f"{key:10s} {rf.get('mean_ms', rf['algorithmic_bytes'] / (rf['achieved'] * 1e9) * 1e3):10.5f} {ref:10.5f} {st if st is not None else float('nan'):10.5f} "
              f"{rf['frac']:7.4f} {frac_tr:8.4f} {diff:+7.2%}  {name}  ({len(durs)} dispatches)")
    print(f"worst |frac difference| {worst:.2%}: {'OK' if ok else 'FAIL'} (tolerance {TOL:.0%})")
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
