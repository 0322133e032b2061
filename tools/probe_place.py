#!/usr/bin/env python3
"""tools/probe_place.py -- is the C4 pass-3 time a property of where the
buffers landed?

Pass 3 of the fp64 2^28 plan reads the plan's workspace W and writes the
caller's output at the SAME 8 MiB-strided offsets; the pass has measured
1.57-1.90 ms box to box and run to run (traced runs 1.84-1.90 ms on a box
whose untraced run took 1.58 ms).  Each trial here allocates a fresh input,
output (with 2 MiB of slack) and plan (fresh W), keeps the earlier trials'
buffers alive so the allocations land elsewhere, and times the three passes
(HIP events) with the output shifted by several offsets inside its slack.
A probe, not product.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))

import torch  # noqa: E402

import pifft  # noqa: E402

LOG_N = int(os.environ.get("PROBE_LOG_N", "28"))
TRIALS = int(os.environ.get("PROBE_TRIALS", "5"))
OFFS = [0, 4 << 10, 64 << 10, 256 << 10, 1 << 20, (1 << 20) + (96 << 10)]
STEPS = 8


def main():
    torch.cuda.set_device(0)
    n = 1 << LOG_N
    keep = []
    s = torch.cuda.current_stream()
    for t in range(TRIALS):
        x = torch.empty(n, dtype=torch.complex128, device="cuda")
        pifft.generate_device(x.data_ptr(), n, n, pifft.F64, seed=11, stream=s)
        ybig = torch.empty(n + (2 << 20) // 16, dtype=torch.complex128, device="cuda")
        plan = pifft.Plan(n, 1, 1, pifft.F64, device=0)
        keep.append((x, ybig, plan))
        for off in OFFS:
            yp = ybig.data_ptr() + off
            for _ in range(2):
                plan.execute_device(x.data_ptr(), yp, s)
            torch.cuda.synchronize()
            plan.profile_start(STEPS)
            for _ in range(STEPS):
                plan.execute_device(x.data_ptr(), yp, s)
            used, sums = plan.profile_read()
            ms = [v / used for v in sums]
            print(f"trial {t} x={x.data_ptr() & ((1 << 30) - 1):#x} y={ybig.data_ptr() & ((1 << 30) - 1):#x} "
                  f"off {off >> 10:5d} KiB  passes " + " ".join(f"{v:.3f}" for v in ms) +
                  f"  total {sum(ms):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
