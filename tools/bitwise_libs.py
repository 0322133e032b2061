#!/usr/bin/env python3
"""tools/bitwise_libs.py LIB -- run a list of plans through this process's
libpifft (PIFFT_LIB) and write each output's SHA-256 to stdout; two runs with
two builds, diffed, show whether a kernel change kept the results bit for bit
(round 6: the one-round-trip tree twiddle fetch, tree_tw_fetch, against the
round-5 kernels; the stage-twiddle prefetch, PIFFT_TW_PREFETCH=3, against
HEAD's kernels on one-worker plans: --set single; and on one worker's
slice of a split, the one-worker fused tree pass: --set slice).
usage: PIFFT_LIB=abvar/x.so python3 tools/bitwise_libs.py [--set tree|single|slice]"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))

import torch  # noqa: E402  (before libpifft: one HIP runtime)
import pifft  # noqa: E402

SHAPES = [(20, 8, 1, 64), (19, 8, 1, 64), (20, 4, 1, 64), (18, 4, 1, 64), (22, 8, 1, 64), (20, 2, 1, 64),
          (20, 8, 1, 32), (18, 8, 1, 32), (21, 8, 1, 32), (12, 8, 64, 64), (17, 8, 16, 64), (24, 8, 1, 64)]
# one-worker plans: single and first passes of every radix the planner picks at these sizes
SINGLE = [(20, 1, 1, 64), (12, 1, 4096, 32), (12, 1, 64, 64), (10, 1, 512, 32), (11, 1, 256, 64), (13, 1, 64, 64),
          (16, 1, 1, 64), (18, 1, 1, 64), (22, 1, 1, 64), (20, 1, 1, 32), (22, 1, 1, 32), (24, 1, 1, 32),
          (9, 1, 1024, 64), (14, 1, 16, 32), (26, 1, 1, 64)]
# one worker's slice (the one-worker fused tree pass, MODE 3): (log n, P, batch, prec, first worker)
SLICE = [(20, 8, 1, 64, 0), (20, 8, 1, 64, 5), (19, 8, 1, 64, 0), (20, 4, 1, 64, 1), (22, 8, 1, 64, 0),
         (20, 2, 1, 64, 1), (20, 8, 1, 32, 0), (21, 8, 1, 32, 3), (12, 8, 64, 64, 0), (18, 16, 1, 64, 7),
         (24, 8, 1, 64, 0), (16, 4, 1, 32, 2)]
SET = sys.argv[sys.argv.index("--set") + 1] if "--set" in sys.argv else "tree"
if SET == "single":
    SHAPES = SINGLE
elif SET == "slice":
    SHAPES = SLICE

for shape in SHAPES:
    logn, P, batch, prec = shape[:4]
    first = shape[4] if len(shape) > 4 else 0
    n = 1 << logn
    cdt = torch.complex128 if prec == 64 else torch.complex64
    x = torch.empty(n * batch, dtype=cdt, device="cuda")
    pifft.generate_device(x.data_ptr(), n * batch, n, prec, seed=logn * 7 + P)
    plan = pifft.Plan(n, P, batch, prec, first=first, count=1) if SET == "slice" else pifft.Plan(n, P, batch, prec)
    y = torch.empty(plan.describe()["out_elems"], dtype=cdt, device="cuda")
    plan.execute_device(x.data_ptr(), y.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    h = hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"n=2^{logn} P={P} first={first} batch={batch} f{prec} {plan.kernel_name(0)[:60]} {h}", flush=True)
    plan.close()
