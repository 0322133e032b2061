"""tools/instance_sweep.py -- which compiled k_pass instances the planner uses.

Plans (host-side only, pifft_plan_dry_run_instances: no GPU) every shape of
the planner's domain with the default settings (no tuning variable):
  N = 2^1 .. 2^32, P = 2^0 .. 2^12 (<= N), worker ranges [0, count) and
  [P - count, P) for every power-of-two count <= P, natural-order /
  slice-major / bit-reversed output, with and without PIFFT_SEPARATE_TREE
  (CLI -u), batches 1 .. 4096 (BATCHES; batch * N <= 2^32), fp32 and fp64,
and prints the set of instances they launch.  tests/test_instances.py checks
that every compiled instance is launched either by some plan of this domain or
by a plan the GPU tests build with their tuning variables (the recorded list
tests/golden/instances_tests.txt, conftest.py's PIFFTTEST_RECORD_INSTANCES); instances
neither uses are not generated (tools/gen_instances.py).

  python tools/instance_sweep.py [--out FILE] [--plans FILE.json] [--jobs 8]
  python tools/instance_sweep.py --compare A.json B.json
"""
from __future__ import annotations

import argparse
import os
import sys
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))

def _batches() -> tuple:
    """1 .. 32, then a geometric grid (ratio 1.07, each point and its
    successor) up to 4096: the planner's batch-dependent choices (workgroup
    counts, byte thresholds) change between these points at most where a
    denser grid found nothing new (round 6: 175 batches reach 768 instances,
    23 batches 766)."""
    b = set(range(1, 33))
    x = 32.0
    while x < 4096:
        x *= 1.07
        b.update((int(x), int(x) + 1))
    b.add(4096)
    return tuple(sorted(v for v in b if v <= 4096))


BATCHES = _batches()


def shapes(log_n: int):
    """(n, P, first, count, batch, prec, flags) of the domain at one N."""
    import pifft
    n = 1 << log_n
    for prec in (pifft.F32, pifft.F64):
        for lp in range(0, min(log_n, 12) + 1):
            P = 1 << lp
            for batch in BATCHES:
                if batch * n > (1 << 32):
                    continue
                for sep in (0, pifft.SEPARATE_TREE):
                    c = P
                    while c >= 1:
                        outs = ((pifft.OUT_NATURAL, pifft.OUT_SLICES, pifft.OUT_BITREV) if c == P else
                                (pifft.OUT_SLICES, pifft.OUT_BITREV))
                        for first in ((0,) if c == P else (0, P - c)):
                            for out in outs:
                                yield n, P, first, c, batch, prec, out | sep
                        c //= 2


def random_shapes(k: int, seed: int = 6):
    """k seeded random shapes beyond the grid: any batch up to 65536, any
    aligned worker range, any output order."""
    import random
    import pifft
    rng = random.Random(seed)
    out = []
    while len(out) < k:
        log_n = rng.randint(1, 32)
        lp = rng.randint(0, min(log_n, 12))
        P = 1 << lp
        batch = rng.randint(1, min(65536, (1 << 32) >> log_n))
        c = 1 << rng.randint(0, lp)
        first = c * rng.randrange(P // c)
        outs = (pifft.OUT_NATURAL, pifft.OUT_SLICES, pifft.OUT_BITREV) if c == P else (pifft.OUT_SLICES, pifft.OUT_BITREV)
        flags = rng.choice(outs) | rng.choice((0, pifft.SEPARATE_TREE))
        out.append((1 << log_n, P, first, c, batch, rng.choice((pifft.F32, pifft.F64)), flags))
    return out


def sweep_one(log_n: int, plans: bool = False):
    """{instance index: first shape that launches it} at one N (a worker
    process: the library's planner state is per process); with plans, also
    every shape's plan as its launches' instance descriptors."""
    import pifft
    table = pifft.instances()
    used, by_shape = {}, {}
    errors = 0
    for shp in (shapes(log_n) if isinstance(log_n, int) else log_n):
        n, P, first, count, batch, prec, flags = shp
        try:
            ids = pifft.dry_run_instances(n, P, batch, prec, first=first, count=count, flags=flags)
        except pifft.PifftError:
            errors += 1  # shapes the ABI refuses (e.g. too large for one launch) plan nothing
            if plans:
                by_shape[shp] = None
            continue
        for i in ids:
            if i >= 0 and i not in used:
                used[i] = shp
        if plans:
            by_shape[shp] = tuple(table[i] if i >= 0 else None for i in ids)
    # the instances these plans depend on: every one the planner found while
    # choosing (pifft_instance_found), launched or not
    for i in pifft.instances_found():
        used.setdefault(i, None)
    return used, errors, by_shape


def _sweep_plans(log_n: int):
    return sweep_one(log_n, True)


def _default_planner_env():
    """Worker-process initializer: the default planner, no tuning variable
    (the caller's own environment is left as it is)."""
    for k in list(os.environ):
        if k.startswith("PIFFT_") and k != "PIFFT_LIB":
            del os.environ[k]


def sweep(jobs: int = 8, logs=range(1, 33), with_plans: bool = False):
    """Every instance the default planner launches or finds over the domain:
    ({index: one shape using it (None: found while choosing)}), with the
    registry table and the count of shapes the ABI refuses."""
    import multiprocessing
    import pifft
    table = pifft.instances()
    used = {}
    errors = 0
    plans = {}
    # fresh worker processes (spawn): each starts with an empty found-log
    # and the default planner's environment
    ctx = multiprocessing.get_context("spawn")
    with ProcessPoolExecutor(max_workers=jobs, mp_context=ctx, initializer=_default_planner_env) as ex:
        for got, err, by_shape in ex.map(_sweep_plans if with_plans else sweep_one, list(logs)):
            errors += err
            plans.update(by_shape)
            for i, shp in got.items():
                used.setdefault(i, shp)
    return (table, used, errors, plans) if with_plans else (table, used, errors)


def fmt(desc) -> str:
    return "prec=%d R=%d C=%d mode=%d nts=%d lp=%d vpt=%d" % tuple(desc)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", default="", help="write the used instances' descriptors here (one per line)")
    ap.add_argument("--jobs", type=int, default=8)
    ap.add_argument("--plans", default="", help="write every shape's plan (its launches' instances) as JSON here")
    ap.add_argument("--random", type=int, default=0, help="also plan this many seeded random shapes (--plans)")
    ap.add_argument("--compare", nargs=2, metavar=("A", "B"),
                    help="compare two --plans files: every shape must plan the same launches")
    args = ap.parse_args()
    if args.compare:
        import json
        a, b = (json.load(open(f)) for f in args.compare)
        diff = [k for k in set(a) | set(b) if a.get(k) != b.get(k)]
        print(f"{len(a)} / {len(b)} shapes, {len(diff)} planned differently")
        for k in sorted(diff)[:20]:
            print(" ", k, a.get(k), "->", b.get(k))
        return 1 if diff else 0
    logs = list(range(1, 33))
    if args.random:
        rs = random_shapes(args.random)
        logs += [rs[k::args.jobs] for k in range(args.jobs)]
    table, used, errors, plans = sweep(args.jobs, logs=logs, with_plans=True)
    if args.plans:
        import json
        with open(args.plans, "w") as f:
            json.dump({str(k): v for k, v in plans.items()}, f)
    print(f"{len(table)} compiled instances; the default planner launches {len(used)} over the domain "
          f"({errors} shapes refused)")
    grid = {fmt(table[i]) for i, shp in used.items()}
    if args.random:
        _, grid_used, _ = sweep(args.jobs)
        grid = {fmt(table[i]) for i in grid_used}
        extra = {fmt(table[i]) for i in used} - grid
        print(f"the {args.random} random shapes launch {len(extra)} instances the grid does not: {sorted(extra)[:8]}")
        used = grid_used
    if args.out:
        with open(args.out, "w") as f:
            for line in sorted(fmt(table[i]) for i in used):
                f.write(line + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
