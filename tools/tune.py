#!/usr/bin/env python3
"""tools/tune.py -- per-launch GB/s of plan variants in one process.

Each variant is a dict of PIFFT_* planner environment variables (read at plan
creation).  For each: build the plan, run W warm-ups, time every launch in
context (PIFFT_PROFILE_SAMPLED) and K back-to-back executions; print
per-launch ms and algorithmic GB/s.

usage: python tools/tune.py --log-n 28 --prec 64 --variants '[{"PIFFT_COL_C64":"4"}, {}]'
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=28)
    ap.add_argument("--prec", type=int, default=64)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--first", type=int, default=0)
    ap.add_argument("--count", type=int, default=0)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--variants", default="[{}]")
    ap.add_argument("--flags", type=int, default=-1, help="plan flags (default: natural / slices)")
    ap.add_argument("--check", action="store_true",
                    help="each variant's output against the first variant's (relative L2)")
    ap.add_argument("--tune-ws", type=int, default=0,
                    help="workspace placements tried per plan (pifft_plan_tune_workspace, as bench.py does)")
    args = ap.parse_args()
    import torch
    import pifft
    n = 1 << args.log_n
    prec = pifft.F64 if args.prec == 64 else pifft.F32
    cdt = torch.complex128 if args.prec == 64 else torch.complex64
    x = torch.empty(n * args.batch, dtype=cdt, device="cuda")
    pifft.generate_device(x.data_ptr(), n * args.batch, n, prec)
    y = None
    yref = None
    # reference ceiling: torch's device copy of the same bytes
    z = torch.empty_like(x)
    for _ in range(3):
        z.copy_(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        z.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"torch copy: {ms:.3f} ms {2 * x.numel() * x.element_size() / ms / 1e6:.0f} GB/s", flush=True)
    del z
    for var in json.loads(args.variants):
        for k in [k for k in os.environ if k.startswith("PIFFT_")]:
            del os.environ[k]
        os.environ.update({k: str(v) for k, v in var.items()})
        os.environ["PIFFT_TUNING"] = "1"
        count = args.count or args.workers
        plan = pifft.Plan(n, args.workers, args.batch, prec, first=args.first, count=count, device=0,
                          flags=None if args.flags < 0 else args.flags)
        d = plan.describe()
        if y is None or y.numel() != d["out_elems"]:
            y = torch.empty(d["out_elems"], dtype=cdt, device="cuda")
        if args.tune_ws > 0:
            plan.tune_workspace(x.data_ptr(), y.data_ptr(), tries=args.tune_ws)
        for _ in range(args.warmup):
            plan.execute_device(x.data_ptr(), y.data_ptr())
        torch.cuda.synchronize()
        # in-context per-launch durations: sampled dispatches back to back (PIFFT_PROFILE_SAMPLED)
        samples = max(args.steps // 2, 3)
        execs = 2 * d["num_launches"] * samples
        plan.profile_start(execs, pifft.PROFILE_SAMPLED)
        for _ in range(execs):
            plan.execute_device(x.data_ptr(), y.data_ptr())
        _, sums, cnt = plan.profile_read()
        avg = [t / c for t, c in zip(sums, cnt)]
        tot = sum(avg)
        # back-to-back executions, no per-launch events (what bench.py times)
        e0.record()
        for _ in range(args.steps):
            plan.execute_device(x.data_ptr(), y.data_ptr())
        e1.record()
        torch.cuda.synchronize()
        wall = e0.elapsed_time(e1) / args.steps
        # consecutive launches of one kind (chunked pairs) summed into one entry
        groups = []
        for i in range(d["num_launches"]):
            k = d["launch_kind"][i]
            k = "chunked" if k.startswith("chunk") else k
            if groups and k == "chunked" and groups[-1][0] == "chunked":
                groups[-1][1] += avg[i]
                groups[-1][2] += d["launch_bytes"][i]
                groups[-1][3] += 1
            else:
                groups.append([k, avg[i], d["launch_bytes"][i], 1])
        per = " | ".join(f"{k}{'x' + str(c) if c > 1 else ''} {ms:.3f}ms {b / ms / 1e6:.0f}GB/s"
                         for k, ms, b, c in groups)
        gf = 5.0 * n * args.log_n * args.batch / (wall * 1e-3) / 1e9
        chk = ""
        if args.check:
            if yref is None:
                yref = y.clone()
            else:
                rel = ((y - yref).abs().pow(2).sum() / yref.abs().pow(2).sum()).sqrt().item()
                chk = f" [vs first variant: rel L2 {rel:.2e}]"
        print(f"{json.dumps(var)} radix={d['radix']} lines={d['lines']} vpt={d.get('vpt')} wall {wall:.3f} ms "
              f"{gf:.0f} GFLOP/s (sum of launches {tot:.3f} ms) :: {per}{chk}", flush=True)
        del plan


if __name__ == "__main__":
    main()
