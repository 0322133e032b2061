#!/usr/bin/env python3
"""tools/probe_ybits.py -- does the fast/slow state of C4 passes 2 and 3
follow the output's virtual address?

One plan (its padded workspace W fixed) and many fresh outputs y (4 GiB
each, all kept alive so each lands elsewhere): per y, the three pass times
(HIP events, 8 steps, the faster of 2 reps) and y's virtual address, so the
state can be matched against address bits of y (W is fixed).  A probe, not
product.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))

import torch  # noqa: E402

import pifft  # noqa: E402

N_Y = int(os.environ.get("PROBE_NY", "20"))
STEPS = 8


def main():
    torch.cuda.set_device(0)
    n = 1 << 28
    s = torch.cuda.current_stream()
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, seed=11, stream=s)
    plan = pifft.Plan(n, 1, 1, pifft.F64, device=0)
    keep = []
    for t in range(N_Y):
        y = torch.empty(n, dtype=torch.complex128, device="cuda")
        keep.append(y)
        best = None
        for rep in range(2):
            for _ in range(2):
                plan.execute_device(x.data_ptr(), y.data_ptr(), s)
            torch.cuda.synchronize()
            plan.profile_start(STEPS, pifft.PROFILE_ALL)  # every launch of every execution
            for _ in range(STEPS):
                plan.execute_device(x.data_ptr(), y.data_ptr(), s)
            used, sums, cnt = plan.profile_read()
            ms = [v / c for v, c in zip(sums, cnt)]
            if best is None or sum(ms) < sum(best):
                best = ms
        va = y.data_ptr()
        print(f"y {t:2d} va {va:#014x} (GiB {va / 2**30:10.3f})  passes " + " ".join(f"{v:.3f}" for v in best) +
              f"  2+3 {best[1] + best[2]:.3f}", flush=True)


if __name__ == "__main__":
    main()
