#!/usr/bin/env python3
"""tools/host_boundary.py -- the PCIe-inclusive rate of the host boundary.

pifft_execute (the reference's run() shape: host in, host out, CPU.c:312-380)
on fp64 N=2^28 with pageable numpy buffers, as the reference's malloc'd
in/out would be: wall time per call (H2D copy of the input, the transform,
D2H copy of the output) next to the kernels' own time (the two stage timers
the call returns).  Never bench.py's value (that is device-resident); this
is DESIGN.md's PCIe-inclusive note.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import pifft  # noqa: E402
import pifft_oracle as oracle  # noqa: E402  (the input generator only)


def main():
    log_n = int(os.environ.get("PROBE_LOG_N", "28"))
    n = 1 << log_n
    x = oracle.generate(n, np.complex128)
    out = np.empty_like(x)
    for P in (1, 8):
        plan = pifft.Plan(n, P, 1, pifft.F64)
        plan.execute(x, out)  # warm-up: staging buffers, code objects
        walls, kern = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            t1, t2 = plan.execute(x, out)
            walls.append((time.perf_counter() - t0) * 1e3)
            kern.append(t1 + t2)
        w, k = min(walls), min(kern)
        gf = 5.0 * n * log_n / (w * 1e-3) / 1e9
        print(f"fp64 N=2^{log_n} P={P}: pifft_execute wall {w:.1f} ms ({gf:.0f} GFLOP/s PCIe-inclusive), kernels "
              f"{k:.2f} ms, host<->device copies {w - k:.1f} ms = {2 * n * 16 / ((w - k) * 1e-3) / 1e9:.1f} GB/s "
              f"for 2 x {n * 16 / 2**30:.0f} GiB", flush=True)
        plan.close()


if __name__ == "__main__":
    main()
