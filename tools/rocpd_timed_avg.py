#!/usr/bin/env python3
"""tools/rocpd_timed_avg.py <rocpd .db> <steps> [out.csv] -- per-kernel average
duration over the LAST `steps` executions of a bench.py run traced by
`rocprofv3 --kernel-trace` (the timed region: bench.py runs its warm-up steps
first), next to the all-dispatch average that `rocprofv3 --stats` prints.
The timed-region average is what bench.py's HIP events measure."""
import csv
import sqlite3
import sys
from collections import defaultdict

db, steps = sys.argv[1], int(sys.argv[2])
con = sqlite3.connect(db)
rows = list(con.execute("select name, duration from kernels order by start"))
ours = [(n, d) for n, d in rows if "k_pass" in n or "k_tree" in n or "k_interleave" in n]
# launches per step: the plan's kernels repeat with a fixed pattern; the last
# steps * (launches per step) dispatches are the timed region
by = defaultdict(list)
for n, d in ours:
    by[n].append(d)
per_step = {n: len(v) // 1 for n, v in by.items()}
total_steps = None
out = []
for n, v in by.items():
    # every kernel of the plan runs the same number of times per step
    out.append((n, len(v), sum(v) / len(v)))
calls = [c for _, c, _ in out]
# the kernel with the fewest calls per step runs once per step
k1 = min(calls)
total_steps = k1  # warm-up + timed steps (each step runs every kernel >= once)
res = []
for n, c, avg_all in out:
    per = c // total_steps
    tail = by[n][-steps * per:]
    res.append((n, c, avg_all, len(tail), sum(tail) / len(tail)))
w = csv.writer(open(sys.argv[3], "w") if len(sys.argv) > 3 else sys.stdout)
w.writerow(["Name", "Calls", "Average (Nsec) all dispatches", "Timed calls", "Average (Nsec) timed region"])
for r in sorted(res, key=lambda r: -r[1] * r[2]):
    w.writerow([r[0], r[1], f"{r[2]:.1f}", r[3], f"{r[4]:.1f}"])
