#!/usr/bin/env python3
"""tools/probe_wtune.py -- workspace placement tuning (pifft_plan_tune_workspace)
on fresh C4 allocation pairs: for each trial a fresh output y and plan (fresh
W), the plan's time before and after keeping the fastest of `tries` W
placements (mean of 10 back-to-back executions each).  Shows how often the
slow DRAM-bank pairing occurs and whether the tuning removes it."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))


def main():
    import torch
    import pifft
    log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 28
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 6
    tries = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    n = 1 << log_n
    st = torch.cuda.current_stream()
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, stream=st)

    def wall(plan, y, k=10):
        for _ in range(2):
            plan.execute_device(x.data_ptr(), y.data_ptr(), st)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            plan.execute_device(x.data_ptr(), y.data_ptr(), st)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / k

    keep = []
    for t in range(trials):
        y = torch.empty(n, dtype=torch.complex128, device="cuda")
        plan = pifft.Plan(n, 1, 1, pifft.F64)
        before = wall(plan, y)
        t0 = time.perf_counter()
        best = plan.tune_workspace(x.data_ptr(), y.data_ptr(), st, tries)
        tune_s = time.perf_counter() - t0
        after = wall(plan, y)
        print(f"trial {t}: {before:.3f} ms -> tuned ({tries} placements, {tune_s * 1e3:.0f} ms) {after:.3f} ms "
              f"(tuner's best {best:.3f})", flush=True)
        keep.append((y, plan))  # keep earlier allocations alive: every trial gets new memory
        if len(keep) > 2:
            keep.pop(0)


if __name__ == "__main__":
    main()
