#!/usr/bin/env python3
"""tools/probe_wpad.py -- C4 (fp64 2^28) with padded workspace rows
(PIFFT_W_PAD elements per W row, PassArgs::in_pad/out_pad) against unpadded,
over several placements of the workspace.

Each trial allocates a fresh output y; then, for every pad, a plan is
created (its W allocated) and timed (HIP events per pass, 8 steps x 2 reps,
the faster rep) and its output checked bitwise against the first one.
Nothing is freed, so every (W, y) pair is a new placement (the pass-2/3 time
is a property of the pair: tools/probe_place.py).  A probe, not product.
Historical in part: PIFFT_INPLACE_LAST was removed after round 2 (PIFFT_W_PAD
remains).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))

import torch  # noqa: E402

import pifft  # noqa: E402

LOG_N = int(os.environ.get("PROBE_LOG_N", "28"))
PREC = int(os.environ.get("PROBE_PREC", "64"))
TRIALS = int(os.environ.get("PROBE_TRIALS", "5"))
PADS = os.environ.get("PROBE_PADS", "0,16,272,1040,8208,65552").split(",")
P = int(os.environ.get("PROBE_P", "1"))  # workers; the plan holds worker 0 only when P > 1
STEPS = 8


def main():
    torch.cuda.set_device(0)
    n = 1 << LOG_N
    prec = pifft.F64 if PREC == 64 else pifft.F32
    cdt = torch.complex128 if PREC == 64 else torch.complex64
    s = torch.cuda.current_stream()
    x = torch.empty(n, dtype=cdt, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, prec, seed=11, stream=s)
    ref = None
    keep = []
    sums_by_pad = {p: [] for p in PADS}
    for t in range(TRIALS):
        y = torch.empty(n // P, dtype=cdt, device="cuda")
        keep.append(y)
        row = []
        for pad in PADS:
            # "<pad>ip": the last pass in place in the output (PIFFT_INPLACE_LAST)
            os.environ["PIFFT_W_PAD"] = pad[:-2] if pad.endswith("ip") else pad
            os.environ["PIFFT_INPLACE_LAST"] = "1" if pad.endswith("ip") else "0"
            plan = pifft.Plan(n, P, 1, prec, first=0, count=1, device=0,
                              flags=pifft.OUT_NATURAL if P == 1 else pifft.OUT_SLICES)
            best = None
            for rep in range(2):
                for _ in range(2):
                    plan.execute_device(x.data_ptr(), y.data_ptr(), s)
                torch.cuda.synchronize()
                plan.profile_start(STEPS, pifft.PROFILE_ALL)
                for _ in range(STEPS):
                    plan.execute_device(x.data_ptr(), y.data_ptr(), s)
                used, sums, _ = plan.profile_read()
                ms = [v / used for v in sums]
                if best is None or sum(ms) < sum(best):
                    best = ms
            if ref is None:
                ref = y.clone()
            same = bool(torch.equal(torch.view_as_real(y), torch.view_as_real(ref)))
            info = plan.describe()
            keep.append(plan)
            sums_by_pad[pad].append(sum(best))
            row.append(f"[{pad}] " + " ".join(f"{v:.3f}" for v in best) + f" ={sum(best):.3f}{'' if same else ' MISMATCH'}")
            if not same:
                print("MISMATCH at pad", pad, "workspace", info.get("workspace_bytes"), flush=True)
        print(f"trial {t}: " + "  ".join(row), flush=True)
    for pad in PADS:
        v = sums_by_pad[pad]
        print(f"pad {pad:>8s}: mean {sum(v) / len(v):.3f} ms  min {min(v):.3f}  max {max(v):.3f}", flush=True)


if __name__ == "__main__":
    main()
