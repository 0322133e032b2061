#!/usr/bin/env python3
"""bench.py -- the headline benchmark of BASELINE.json:

  "GFLOP/s (5N log2N / t) + % HBM roofline, fp64 complex N=2^28 @1/2/4/8 GPU"

One step = one complete pi-FFT of ONE fp64 complex N=2^28 transform (config 4
at --gpus 1).  With --gpus G (one process per GPU, torchrun) the same transform
is split over P=G workers the reference's way: rank q computes worker q's
N/P output bins (its tree over the whole, replicated input + an N/P-point FFT),
with no data-path collective; the time is the slowest rank's (max over ranks),
value = 5 N log2 N / t for the one transform ("strong" scaling: the total work
is fixed).  Inputs are generated on the device (splitmix64, the oracle's
generator) and resident in HBM before the timed region.

--shard batch (config 3, e.g. --log-n 12 --prec 32 --batch 4096): the batch of
independent transforms is split by transform instead, rank r running B/G whole
transforms (P = --workers, default 1) -- again no data-path collective.

Adds to the JSON line:
  roofline     : the dominant kernel's algorithmic bytes / its mean duration
                 (HIP events on the launch stream, inside the timed region),
                 vs 8 TB/s; traffic = PMC-measured HBM bytes per launch from the
                 committed rocprofv3 summary (profiles/), else null
  cpu_baseline : the reference CPU path (oracle/_ref, compiled from the
                 reference source) on a bounded sample, rank 0 at --gpus 1 only
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def _baseline_metric():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        return json.load(f)["metric"]


def cpu_baseline(log_n: int, threads: int) -> dict | None:
    """Reference CPU path (oracle/_ref, -Dfloat=double) on N=2^log_n with P=threads."""
    import pifft_oracle as oracle
    n = 1 << log_n
    flops = 5.0 * n * log_n
    exe = oracle.reference_binary(64)
    host = {"cpu_model": _cpu_model(), "host_cpus": os.cpu_count()}

    def run_ref(path):
        t0 = time.perf_counter()
        r = subprocess.run([path, "-n", str(n), "-p", str(threads), "-o"], capture_output=True, text=True,
                           timeout=900)
        wall = time.perf_counter() - t0
        if r.returncode != 0:
            return None, wall
        return float(r.stdout.strip().splitlines()[-1].split("\t")[2]), wall

    if exe:
        ms, wall = run_ref(exe)
        if ms is not None:
            out = {"value": round(flops / (ms * 1e6), 4), "unit": "GFLOP/s", "cores": threads,
                   "kind": "reference",
                   "sample": f"reference fourier-parallel-pi-cpu-pthreads built -O2 -Dfloat=double, "
                             f"fp64 N=2^{log_n}, p={threads} pthreads; worker 0's tree+cylinder time "
                             f"{ms:.1f} ms (the reference's own timer); process wall {wall:.1f} s", **host}
            # the same at the reference Makefile's own flags (-g, no -O; cpu/Makefile:21)
            o0 = exe + "-O0"
            if os.path.exists(o0):
                ms0, wall0 = run_ref(o0)
                if ms0 is not None:
                    out["value_O0"] = round(flops / (ms0 * 1e6), 4)
                    out["sample_O0"] = (f"same sample, reference built with its Makefile's flags (-g, -O0): "
                                        f"worker 0 {ms0:.1f} ms, process wall {wall0:.1f} s")
            return out
    # fallback: the C restatement (bitwise-equal arithmetic)
    import numpy as np
    x = oracle.generate(n, np.complex128)
    _, (t1, t2, wall) = oracle.fft(x, P=threads, nthreads=threads, timing=True)
    ms = t1 + t2
    return {"value": round(flops / (ms * 1e6), 4), "unit": "GFLOP/s", "cores": threads, "kind": "port",
            "sample": f"oracle/pifft_oracle.c (restated reference) fp64 N=2^{log_n}, {threads} threads; "
                      f"worker 0 tree+cylinder {ms:.1f} ms, join wall {wall:.1f} ms", **host}


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_traffic(config_key: str, launch_indices):
    """HBM bytes per launch of the dominant kernel (mean over its launches) from
    the committed PMC summary."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("config_key") == config_key:
            per = d.get("per_launch_bytes", {})
            vals = [per.get(str(i)) for i in launch_indices]
            if vals and all(v is not None for v in vals):
                return float(sum(vals)) / len(vals), os.path.relpath(f, ROOT)
    return None, None


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=28)
    ap.add_argument("--prec", type=int, default=64, choices=(32, 64))
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--workers", type=int, default=0, help="P (default: number of ranks)")
    ap.add_argument("--seed", type=int, default=0x5EED)
    ap.add_argument("--shard", choices=("workers", "batch"), default="workers",
                    help="split one transform's workers over the ranks (the reference's pi split), or a "
                         "batch of independent transforms by transform (config 3)")
    ap.add_argument("--allgather", action="store_true", help="also time the optional RCCL all-gather")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-log-n", type=int, default=26)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) or gloo")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses cuda:0 (use with --dist-backend gloo)")
    ap.add_argument("--as-rank", default="",
                    help="q/G: run only rank q's plan of a G-GPU job, on this one GPU and without a process "
                         "group (per-rank profiling, e.g. tools/pmc_traffic.py); never a job-level number")
    args = ap.parse_args()

    import torch
    import pifft

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    emulated = None
    if args.as_rank:
        if world > 1:
            raise SystemExit("--as-rank is a single-process option")
        emulated = tuple(int(v) for v in args.as_rank.split("/"))
        if len(emulated) != 2 or not 0 <= emulated[0] < emulated[1]:
            raise SystemExit("--as-rank wants q/G with 0 <= q < G")
    gpu = 0 if args.same_device else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    def barrier():
        if dist is not None:
            if args.dist_backend == "nccl":
                dist.barrier(device_ids=[gpu])
            else:
                dist.barrier()

    n = 1 << args.log_n
    import pifft_dist
    q_rank, g_world = emulated if emulated else (rank, world)
    b_first, b_count = 0, args.batch  # transforms of the batch on this rank
    if args.shard == "batch":
        P = args.workers or 1
        first, count = 0, P
        b_first, b_count = pifft_dist.batch_range(q_rank, g_world, args.batch)
    else:
        P = args.workers or g_world
        first, count = pifft_dist.worker_range(q_rank, g_world, P)
    prec = pifft.F64 if args.prec == 64 else pifft.F32
    cdt = torch.complex128 if prec == pifft.F64 else torch.complex64
    esz = 16 if prec == pifft.F64 else 8

    if count == P:
        plan = pifft.Plan(n, P, b_count, prec, first=0, count=P, device=gpu, flags=pifft.OUT_NATURAL)
    else:
        plan = pifft.Plan(n, P, b_count, prec, first=first, count=count, device=gpu,
                          flags=pifft.OUT_SLICES)
    desc = plan.describe()
    stream = torch.cuda.current_stream(dev)
    # this rank's transforms of the global batch: elements [b_first n, (b_first + b_count) n)
    x = torch.empty(n * b_count, dtype=cdt, device=dev)
    pifft.generate_device(x.data_ptr(), n * b_count, n, prec, seed=args.seed, first=b_first * n, stream=stream)
    y = torch.empty(desc["out_elems"], dtype=cdt, device=dev)
    for _ in range(args.warmup):
        plan.execute_device(x.data_ptr(), y.data_ptr(), stream)
    torch.cuda.synchronize(dev)

    nl = desc["num_launches"]
    # per-launch HIP events on the launch stream, recorded inside the timed
    # region without host syncs (pifft_profile_start/read)
    plan.profile_start(args.steps)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.execute_device(x.data_ptr(), y.data_ptr(), stream)
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    recorded, sums = plan.profile_read()
    assert recorded == args.steps, recorded
    red_dev = dev if args.dist_backend == "nccl" else None  # gloo reduces on the CPU
    elapsed = pifft_dist.max_over_ranks(elapsed, red_dev)
    ms_per_step = elapsed * 1e3 / args.steps

    allgather_ms = None
    if args.allgather and dist is not None and args.shard == "batch":
        # whole transforms per rank: the gathered batch is already in order
        torch.cuda.synchronize(dev)
        barrier()
        ta = time.perf_counter()
        gathered = pifft_dist.allgather_slices(y)
        torch.cuda.synchronize(dev)
        allgather_ms = pifft_dist.max_over_ranks((time.perf_counter() - ta) * 1e3, red_dev)
        del gathered
    elif args.allgather and dist is not None and count < P:
        torch.cuda.synchronize(dev)
        barrier()
        ta = time.perf_counter()
        gathered = pifft_dist.allgather_slices(y)
        natural = torch.empty(n * args.batch, dtype=cdt, device=dev)
        pifft.interleave_device(gathered.data_ptr(), natural.data_ptr(), n, P, args.batch, prec, stream)
        torch.cuda.synchronize(dev)
        allgather_ms = pifft_dist.max_over_ranks((time.perf_counter() - ta) * 1e3, red_dev)
        del gathered, natural

    avg = [s / args.steps for s in sums]
    # dominant kernel = the kernel function with the largest share of the step
    # (its launches grouped as rocprofv3 --stats groups them); achieved = its
    # algorithmic bytes per launch / its mean launch duration
    by_fn = {}
    for i in range(nl):
        by_fn.setdefault(desc["launch_fn"][i], []).append(i)
    dom_launches = max(by_fn.values(), key=lambda ls: sum(avg[i] for i in ls)) if nl else [0]
    dom = dom_launches[0]
    dom_ms = sum(avg[i] for i in dom_launches) / len(dom_launches)
    dom_bytes = sum(desc["launch_bytes"][i] for i in dom_launches) // len(dom_launches)
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
    flops = 5.0 * n * args.log_n * args.batch  # the whole job's batch (every rank's share)
    value = flops / (ms_per_step * 1e-3) / 1e9
    config_key = f"n2^{args.log_n}_f{args.prec}_b{b_count}_P{P}_q{count}"
    traffic, traffic_src = load_traffic(config_key, dom_launches)

    launches = []
    for i in range(nl):
        kind = desc["launch_kind"][i] if i < len(desc["launch_kind"]) else "?"
        b = desc["launch_bytes"][i] if i < len(desc["launch_bytes"]) else 0
        launches.append({"kind": kind, "bytes": b, "ms": round(avg[i], 4),
                         "GB/s": round(b / (avg[i] * 1e-3) / 1e9, 1) if avg[i] > 0 else None})
    total_bytes = sum(desc["launch_bytes"][:nl])

    if rank == 0:
        line = {
            "metric": _baseline_metric(),
            "value": round(value, 2),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 6),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64" if prec == pifft.F64 else "f32",
            "data": "synthetic: splitmix64 U[-1,1]/sqrt(N) complex input generated in HBM (the oracle's generator)",
            "config": {
                "workload": (f"config 4: one fp64 complex N=2^{args.log_n} pi-FFT" if args.log_n == 28 and
                             args.prec == 64 and args.batch == 1 else
                             f"config 3: batched fp32 {args.batch} x N=4096" if args.log_n == 12 and
                             args.prec == 32 and args.batch == 4096 else
                             f"pi-FFT N=2^{args.log_n} f{args.prec} batch {args.batch}")
                            + (f", P={P} workers, {b_count} whole transforms per GPU (batch-sharded, no "
                               f"data-path collective)" if args.shard == "batch" else
                               f", P={P} workers, {count} per GPU (no data-path collective)"),
                "n": n, "workers": P, "workers_per_gpu": count, "batch": args.batch,
                "batch_per_gpu": b_count, "shard": args.shard,
                "local_n": desc["local_n"], "passes": desc["num_passes"], "radix": desc["radix"],
                "lines_per_workgroup": desc["lines"],
                "hbm_bytes_per_step_algorithmic": total_bytes,
                "hbm_GBps_per_step_algorithmic": round(total_bytes / (ms_per_step * 1e-3) / 1e9, 1),
                "launches": launches,
                "parallelism": (f"batch-split {args.batch}/{world} per GPU, p{P}" if args.shard == "batch" else
                                f"pi-split p{P} over {world} GPU(s)"),
                "allgather_ms": None if allgather_ms is None else round(allgather_ms, 3),
                "emulated_rank": args.as_rank or None,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": (f"{launches[dom]['kind'] if launches else '?'} kernel of launches {dom_launches} "
                           f"(mean launch {dom_ms:.4f} ms, HIP events on the launch stream)"),
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes": dom_bytes,
            },
            "cpu_baseline": None,
        }
        if world == 1 and not emulated and not args.no_cpu_baseline:
            threads = args.cpu_threads
            ncpu = os.cpu_count() or 1
            while threads > ncpu:
                threads //= 2
            try:
                line["cpu_baseline"] = cpu_baseline(args.cpu_log_n, max(1, threads))
            except Exception as e:  # reported, never silently replaced
                line["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
