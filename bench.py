#!/usr/bin/env python3
"""bench.py -- the headline benchmark of BASELINE.json:

  "GFLOP/s (5N log2N / t) + % HBM roofline, fp64 complex N=2^28 @1/2/4/8 GPU"

One step = one complete pi-FFT of ONE fp64 complex N=2^28 transform (config 4
at --gpus 1).  With --gpus G the same transform is split over P=G workers the
reference's way, one process per GPU: rank q computes worker q's N/P output
bins (its tree over the whole, replicated input + an N/P-point FFT), with no
data-path collective; the time is the slowest rank's (max over ranks), value =
5 N log2 N / t for the one transform ("strong" scaling: the total work is
fixed).  Inputs are generated on the device (splitmix64, the oracle's
generator) and resident in HBM before the timed region.

--gpus G without a torchrun environment: this process launches G ranks
(python -m torch.distributed.run, 127.0.0.1) and exits with their status; it
never touches a GPU itself.  Under torchrun, WORLD_SIZE must equal --gpus.

--shard batch (config 3, e.g. --log-n 12 --prec 32 --batch 4096): the batch of
independent transforms is split by transform instead, rank r running B/G whole
transforms (P = --workers, default 1) -- again no data-path collective.

At G > 1 the optional final exchange (RCCL all-gather over xGMI + the
stride-P interleave into natural order) runs once after the timed region and
is reported as config.allgather_ms (never part of value; --no-allgather skips
it).  Every rank's own time and dominant-kernel roofline go to config.per_rank.

Adds to the JSON line:
  roofline     : the dominant kernel's algorithmic bytes / its mean duration,
                 vs 8 TB/s.  The duration: after the timed region, a clean
                 loop of that kernel's launches alone, back to back on the
                 launch stream between two marker events (pifft_launch_loop,
                 ~20 ms of them), so nothing but the kernel and its dispatch
                 gaps is timed.  Every launch's own duration (config launches)
                 comes from a profiling loop that times one launch per odd
                 execution with events bound to that dispatch
                 (PIFFT_PROFILE_SAMPLED).  Refused (frac null) if the kernel's
                 launches would take longer than the step.  traffic =
                 PMC-measured HBM bytes per launch from the committed
                 rocprofv3 summary (profiles/)
  cpu_baseline : the reference CPU path (oracle/_ref, compiled from the
                 reference source) at the SAME N, rank 0 of every job, at the
                 fastest p the box's CPU share supports (p = 16 under a
                 16-CPU quota), the reference's own p_to = 32 beside it
  secondary    : (--gpus 1, default on) configs 1, 2 (whole and one GPU's
                 slice) and 3 timed in the same run, each with its own
                 dominant-kernel roofline and a reference CPU baseline at the
                 same N
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# a roofline is refused when the dominant kernel's launches, timed back to back
# in a clean loop, take longer than the step by more than this (timing noise;
# tools/check_rooflines.py's tolerance)
REFUSE_TOL = 0.03
# The reference's own processor sweep: p = 1 .. 32 (run-experiments-and-analyze-
# results:29, p_to=32), skipping p above the machine's online CPUs
# (how-many-cpu-cores.c; CPU.c:200, 835-837 refuses p > sysconf(ONLN))
REF_P_TO = 32
# A GPU-box command is killed above ~270 GiB of host memory (the pool's
# per-command cap, not visible to the process): the reference's footprint is
# planned below this, and below 0.8 x MemAvailable and any cgroup limit
HOST_CMD_CAP = 256 << 30
BENCH_PROC_RESERVE = 8 << 30  # this process (torch + HIP runtime) beside the reference


def _baseline_metric():
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        return json.load(f)["metric"]


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _physical_cores() -> int | None:
    """Distinct (physical id, core id) pairs of /proc/cpuinfo."""
    try:
        cores, phys = set(), None
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    cores.add((phys, line.split(":", 1)[1].strip()))
        return len(cores) or None
    except OSError:
        return None


def _cgroup_cpu_quota() -> float | None:
    """CPUs' worth of time this cgroup may use (cpu.max), None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return None


def _cgroup_mem_limit() -> int | None:
    try:
        v = open("/sys/fs/cgroup/memory.max").read().strip()
        return None if v == "max" else int(v)
    except (OSError, ValueError):
        return None


def _mem_available() -> int:
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 8 << 30


def _host() -> dict:
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {"cpu_model": _cpu_model(), "host_cpus": os.cpu_count(), "physical_cores": _physical_cores(),
            "cpu_affinity": affinity, "cgroup_cpu_quota": _cgroup_cpu_quota(),
            "mem_available_GiB": round(_mem_available() / 2**30, 1),
            "cgroup_mem_limit_GiB": None if _cgroup_mem_limit() is None else round(_cgroup_mem_limit() / 2**30, 1)}


def _host_budget() -> int:
    """Host bytes the reference may touch: 0.8 x MemAvailable, the cgroup
    limit and the box's per-command cap, less this process's own share."""
    b = min(int(_mem_available() * 0.8), int(HOST_CMD_CAP * 0.9))
    lim = _cgroup_mem_limit()
    if lim is not None:
        b = min(b, int(lim * 0.9))
    return b - BENCH_PROC_RESERVE


def _child_peak_rss() -> int:
    """Peak RSS (bytes) of the largest child process that has exited so far."""
    import resource
    return resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss * 1024


def _run_ref(path: str, n: int, p: int, timeout: int = 900):
    """One run of the reference CLI; (worker 0's tree+cylinder ms by its own timer, wall s)."""
    t0 = time.perf_counter()
    r = subprocess.run([path, "-n", str(n), "-p", str(p), "-o"], capture_output=True, text=True, timeout=timeout)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"reference exited {r.returncode}: {r.stderr.strip()[-300:]}")
    return float(r.stdout.strip().splitlines()[-1].split("\t")[2]), wall


def _union_len(iv) -> int:
    tot, end = 0, -1
    for a, b in sorted(iv):
        if b <= end:
            continue
        tot += b - max(a, end)
        end = b
    return tot


def ref_touched_elems(n: int, p: int) -> int:
    """Elements of host memory the reference touches with p workers (-o runs):
    `in` (written by initialize_data, CPU.c:220-247; `out` stays untouched
    without -t) and, per worker, all of tmp_in (copy_to, CPU.c:407) plus the
    tmp_out pages its tree levels and cylinder stages write (CPU.c:419-478,
    the two scratchpads swapping after every level)."""
    lp = p.bit_length() - 1
    m = n // p
    total = n
    for q in range(p):
        written = [[], []]  # ranges written into the original tmp_in / tmp_out
        cur, size, it = 1, n, lp
        while size > m:
            off = (q >> it) * size
            left = ((q >> (it - 1)) & 1) == 0
            written[cur].append((off, off + size // 2) if left else (off + size // 2, off + size))
            cur ^= 1
            size //= 2
            it -= 1
        size = m
        while size > 1:
            written[cur].append((q * m, q * m + m))
            cur ^= 1
            size //= 2
        total += n + _union_len(written[1])
    return total


def _cpu_share() -> int:
    """CPUs this process may actually run on at once: the online CPUs, the
    affinity mask and the cgroup's CPU quota (cpu.max), whichever is least."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        pass
    q = _cgroup_cpu_quota()
    if q is not None:
        n = min(n, max(1, int(q)))
    return n


def ref_workers(log_n: int, esz: int, threads: int | None = None, share: bool = True) -> int:
    """The reference's worker count for the CPU baseline: the largest p of its
    own sweep (1, 2, 4, ... up to REF_P_TO = 32, run-experiments-and-analyze-
    results:29) that the host's CPU share runs without time-sharing (online
    CPUs as how_many_cores rules, CPU.c:200, the affinity mask and the cgroup
    quota; share=False: online CPUs only, the reference's own rule), halved
    until the host memory it touches (ref_touched_elems) fits _host_budget()."""
    cap = threads or min(REF_P_TO, _cpu_share() if share else (os.cpu_count() or 1))
    p = 1
    while p * 2 <= cap:
        p *= 2
    budget = _host_budget()
    while p > 1 and ref_touched_elems(1 << log_n, p) * esz > budget:
        p //= 2
    need = ref_touched_elems(1 << log_n, p) * esz
    if need > budget:
        raise RuntimeError(f"N=2^{log_n} needs {need / 2**30:.0f} GiB of host memory, "
                           f"{budget / 2**30:.0f} GiB available")
    return p


def cpu_baseline(log_n: int, prec: int, threads: int | None = None, workers: int | None = None, repeat: int = 1,
                 batch: int = 1, slice_of: int = 0) -> dict:
    """The reference CPU path at N = 2^log_n: oracle/_ref (CPU.c built -O2,
    -Dfloat=double for fp64) with P = `workers` pthreads (default:
    ref_workers -- the reference's own p_to = 32 where the host allows).  Its
    own timer (worker 0's tree + cylinder, CPU.c:414-491) gives the time.
    repeat > 1 takes the median of that many runs; batch > 1 scales one
    transform's time to the batch (the reference has no batch: a batch is a
    loop of run()).  slice_of = P: the time is ONE worker's share of a
    P-worker split (worker 0's own time), reported as the rate of the whole
    transform at that time."""
    import pifft_oracle as oracle
    n = 1 << log_n
    esz = 16 if prec == 64 else 8
    flops = 5.0 * n * log_n * batch
    p = workers or ref_workers(log_n, esz, threads)
    exe = oracle.reference_binary(prec)
    if exe is None:  # fallback: the C restatement (bitwise-equal arithmetic)
        import numpy as np
        x = oracle.generate(n, np.complex128 if prec == 64 else np.complex64)
        _, (t1, t2, wall) = oracle.fft(x, P=p, nthreads=p, timing=True)
        ms = (t1 + t2) * batch
        return {"value": round(flops / (ms * 1e6), 4), "unit": "GFLOP/s", "cores": p, "kind": "port",
                "sample": f"oracle/pifft_oracle.c (restated reference) f{prec} N=2^{log_n}, P={p}; worker 0 "
                          f"tree+cylinder {ms:.1f} ms, join wall {wall:.1f} ms", **_host()}
    runs = [_run_ref(exe, n, p) for _ in range(repeat)]
    ms1 = statistics.median(r[0] for r in runs)
    ms = ms1 * batch
    what = (f"reference fourier-parallel-pi-cpu-pthreads built -O2{' -Dfloat=double' if prec == 64 else ''} "
            f"(oracle/_ref, from the reference source), f{prec} N=2^{log_n}, p={p} pthreads")
    if repeat > 1:
        what += f"; median of {repeat} runs of worker 0's tree+cylinder time {ms1:.3f} ms"
    else:
        what += f"; worker 0's tree+cylinder time {ms1:.1f} ms (the reference's own timer)"
    if batch > 1:
        what += f" x {batch} transforms (the reference has no batch) = {ms:.1f} ms"
    if slice_of:
        what += f"; one worker's share of the {slice_of}-way split, rated as the whole transform"
    what += f"; process wall {sum(r[1] for r in runs):.1f} s"
    return {"value": round(flops / (ms * 1e6), 4), "unit": "GFLOP/s", "cores": p, "kind": "reference",
            "ms": round(ms, 3), "sample": what, "host_bytes_touched": ref_touched_elems(n, p) * esz,
            "child_peak_rss_GiB": round(_child_peak_rss() / 2**30, 2), **_host()}


def headline_cpu_baseline(log_n: int, prec: int, batch: int = 1, threads: int | None = None) -> dict:
    """cpu_baseline of a bench line: the reference's best on this host.  It
    runs at the largest p of its sweep that the host's CPU share (online CPUs,
    affinity, cgroup quota: 16 CPUs on the GPU box) runs without time-sharing,
    and -- when the reference's own rule (p_to = 32 up to the online CPUs,
    CPU.c:200) allows more -- at that p too; `value` is the faster of the two,
    the other is reported beside it ("alternative"), with the quota stated."""
    cl = log_n
    rec = cpu_baseline(cl, prec, threads, batch=batch, repeat=1 if cl > 16 else 15)
    rec["cpu_share"] = _cpu_share()
    rec["selection"] = ("the largest p of the reference's sweep within the host's CPU share (online CPUs, "
                        "affinity, cgroup quota)" if not threads else "--cpu-threads")
    if rec.get("kind") != "reference" or threads:
        return rec
    try:
        p_ref = ref_workers(cl, 16 if prec == 64 else 8, share=False)
    except RuntimeError:
        p_ref = rec["cores"]
    if p_ref > rec["cores"]:
        try:
            alt = cpu_baseline(cl, prec, workers=p_ref, batch=batch, repeat=1 if cl > 16 else 15)
            keep = ("value", "cores", "ms", "sample", "host_bytes_touched", "child_peak_rss_GiB")
            if alt["value"] > rec["value"]:  # lead with the reference's best on this host
                other = {k: rec[k] for k in keep if k in rec}
                rec.update({k: alt[k] for k in keep if k in alt})
                rec["alternative"] = other
            else:
                rec["alternative"] = {k: alt[k] for k in keep if k in alt}
        except Exception as e:  # reported, never silently replaced
            rec["alternative"] = {"value": None, "cores": p_ref, "error": repr(e)}
    # the reference Makefile's own flags (-g, i.e. -O0, cpu/Makefile:21) beside
    # the -O2 build, at the same p; fp64 (oracle/_ref's -O0 build)
    if prec == 64 and batch == 1 and os.environ.get("BENCH_CPU_O0", "1") == "1":
        try:
            import pifft_oracle as oracle
            exe0 = os.path.join(os.path.dirname(oracle.reference_binary(64)), "fourier-parallel-pi-cpu-pthreads-f64-O0")
            ms0, wall0 = _run_ref(exe0, 1 << cl, rec["cores"])
            rec["O0"] = {"value": round(5.0 * (1 << cl) * cl / (ms0 * 1e6), 4), "cores": rec["cores"],
                         "ms": round(ms0, 3), "wall_s": round(wall0, 1)}
        except Exception as e:  # reported, never silently replaced
            rec["O0"] = {"value": None, "error": repr(e)[:200]}
    return rec


def load_traffic(config_key: str, launch_indices, kernel_names=None):
    """HBM bytes per launch of the dominant kernel (mean over its launches) from
    the committed PMC summary (the last profiles/*traffic*.json of this plan by
    name: round tags sort in order).  With kernel_names, a summary counts only
    if it profiled those very kernels at those launches (a planner change
    gives the same config a different plan)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic*.json")))  # r02_* after r01_*
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("config_key") == config_key:
            per = d.get("per_launch_bytes", {})
            if kernel_names is not None and [d.get("kernels", {}).get(str(i), {}).get("kernel")
                                             for i in launch_indices] != list(kernel_names):
                continue
            vals = [per.get(str(i)) for i in launch_indices]
            if vals and all(v is not None for v in vals):
                return float(sum(vals)) / len(vals), os.path.relpath(f, ROOT)
    return None, None


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(gpus: int) -> int:
    """--gpus G outside torchrun: one rank process per GPU (this parent never
    initialises a GPU; it only waits for its children)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


class Job:
    """One pi-FFT plan on this rank's GPU with its input resident in HBM."""

    def __init__(self, pifft, torch, gpu, *, n, P, prec, first, count, batch_local, b_first, seed):
        self.pifft, self.torch, self.n, self.P = pifft, torch, n, P
        self.prec, self.count, self.batch_local = prec, count, batch_local
        self.dev = torch.device("cuda", gpu)
        flags = pifft.OUT_NATURAL if count == P else pifft.OUT_SLICES
        self.plan = pifft.Plan(n, P, batch_local, prec, first=first, count=count, device=gpu, flags=flags)
        self.desc = self.plan.describe()
        self.stream = torch.cuda.current_stream(self.dev)
        cdt = torch.complex128 if prec == pifft.F64 else torch.complex64
        # this rank's transforms of the global batch: elements [b_first n, (b_first + b_local) n)
        self.x = torch.empty(n * batch_local, dtype=cdt, device=self.dev)
        pifft.generate_device(self.x.data_ptr(), n * batch_local, n, prec, seed=seed, first=b_first * n,
                              stream=self.stream)
        self.y = torch.empty(self.desc["out_elems"], dtype=cdt, device=self.dev)
        # placement tuning before the warm-up (pifft_plan_tune_workspace: the
        # fastest of 8 workspace allocations for this output; ~0.2 s at 2^28,
        # profiles/r03_workspace_tuning.log: C4 4.62-4.81 -> 4.59-4.62 ms)
        self.tuned_ms = self.plan.tune_workspace(self.x.data_ptr(), self.y.data_ptr(), self.stream,
                                                 int(os.environ.get("BENCH_W_TRIES", "8")))

    def step(self):
        self.plan.execute_device(self.x.data_ptr(), self.y.data_ptr(), self.stream)

    def run(self, steps, warmup, barrier=lambda: None):
        """W untimed steps, then exactly K steps between barrier + synchronize
        on both sides; nothing but the plan's launches in the timed region.
        Returns this rank's seconds."""
        torch = self.torch
        for _ in range(warmup):
            self.step()
        torch.cuda.synchronize(self.dev)
        barrier()
        torch.cuda.synchronize(self.dev)
        t0 = time.perf_counter()
        for _ in range(steps):
            self.step()
        torch.cuda.synchronize(self.dev)
        barrier()
        return time.perf_counter() - t0

    def time_launches(self, samples: int):
        """Every launch's in-context duration (ms): a profiling loop after the
        timed region in which odd executions time one launch each, round
        robin, with start/stop events bound to that dispatch
        (PIFFT_PROFILE_SAMPLED) -- every timed dispatch runs back to back
        after untimed ones, as in the timed loop (a timed dispatch delays the
        next by ~9 us; launches timed one after another ran 1-6 % faster than
        back to back, round-3 trace).  `samples` per launch."""
        nl = self.desc["num_launches"]
        execs = 2 * nl * samples
        self.plan.profile_start(execs, self.pifft.PROFILE_SAMPLED)
        for _ in range(execs):
            self.step()
        used, sums, cnt = self.plan.profile_read()
        assert used == execs and min(cnt) == samples, (used, cnt)
        self.avg = [t / c for t, c in zip(sums, cnt)]
        self.samples = samples

    def loop(self, launches) -> tuple:
        """(mean ms, rounds) of a clean loop of these launches alone, back to
        back (pifft_launch_loop): ~20 ms of them, 10 - 4000 rounds sized from
        the bytes at 4 TB/s, so the count is a function of the plan alone (a
        trace of another run of the same command cuts at the same place)."""
        d = self.desc
        nbytes = sum(d["launch_bytes"][i] for i in launches)
        reps = int(min(4000, max(10, 20e-3 / (nbytes / 4e12))))
        return self.plan.launch_loop(launches, reps, self.x.data_ptr(), self.y.data_ptr(), self.stream), reps

    def roofline(self, ms_per_step: float) -> dict:
        """The dominant kernel: the kernel function (its launches grouped as
        rocprofv3 --stats groups them) with the largest time per step in a
        clean back-to-back loop of its launches (Job.loop; marker events
        around the loop only, so the figure holds under a tracer too:
        rocprofv3 reproduces it on the same dispatches to 0.04 %, round 4,
        profiles/r04i_roofline_check_traced_run.txt).  frac = algorithmic
        bytes per launch / that mean launch time; the dominant kernel's loop
        runs last, so a trace ends with it.  Self-check: no frac when the
        kernel's launches take longer than the measured step."""
        d = self.desc
        nl = d["num_launches"]
        raw_step_ms = sum(self.avg[:nl])
        avg = self.scaled(ms_per_step)
        by_fn = {}
        for i in range(nl):
            by_fn.setdefault(d["launch_fn"][i], []).append(i)
        shares = {tuple(ls): self.loop(ls)[0] * len(ls) for ls in by_fn.values()} if len(by_fn) > 1 else {}
        dom_launches = list(max(shares, key=shares.get)) if shares else next(iter(by_fn.values()))
        sampled_ms = sum(avg[i] for i in dom_launches) / len(dom_launches)
        dom_bytes = sum(d["launch_bytes"][i] for i in dom_launches) // len(dom_launches)
        dom_ms, reps = self.loop(dom_launches)
        dom_step_ms = dom_ms * len(dom_launches)
        kernel_step_ms = sum(avg[:nl])
        achieved = dom_bytes / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
        rec = {"bound": "hbm",
               "kernel": (f"{d['launch_kind'][dom_launches[0]]} kernel of launches {dom_launches} "
                          f"(mean launch {dom_ms:.5f} ms: a clean loop of {reps} x {len(dom_launches)} launches "
                          f"back to back on the launch stream, marker events around the loop)"),
               "launches": dom_launches, "mean_ms": round(dom_ms, 6), "loop_reps": reps,
               "sampled_mean_ms": round(sampled_ms, 6),
               "kernel_name": self.plan.kernel_name(dom_launches[0]),
               "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(achieved / HBM_PEAK_GBS, 4), "algorithmic_bytes": dom_bytes,
               "kernel_ms_per_step": round(dom_step_ms, 6), "all_launches_ms_per_step": round(kernel_step_ms, 6),
               "step_ms": round(ms_per_step, 6), "event_ms_per_step": round(raw_step_ms, 6),
               "event_overhead_subtracted_ms": round(raw_step_ms - kernel_step_ms, 6),
               # the loop's place in this config's dispatches of the kernel:
               # its timed rounds, then one full execution (the last
               # len(launches) of them) -- tools/check_rooflines.py cuts a
               # trace to exactly the timed rounds
               "trace_loop_dispatches": reps * len(dom_launches)}
        # the whole step beside the dominant kernel: every launch's algorithmic
        # bytes over the measured step time (a plan may trade one kernel's
        # frac for a shorter step, e.g. the narrow-segment pass moved last)
        step_bytes = sum(d["launch_bytes"][:nl])
        rec["step_achieved"] = round(step_bytes / (ms_per_step * 1e-3) / 1e9, 1) if ms_per_step > 0 else None
        rec["step_frac"] = round(rec["step_achieved"] / HBM_PEAK_GBS, 4) if rec["step_achieved"] else None
        # self-checks, both recorded: the dominant kernel's launches, back to
        # back, cannot take longer than the step they run in (beyond
        # REFUSE_TOL: refused), and every kernel function's clean loop
        # together -- and the sampled per-launch event times -- should fit in
        # it too (recorded, with the tolerance, so a reader sees when the
        # tolerance was used)
        loops_ms = sum(shares.values()) if shares else dom_step_ms
        rec["loops_ms_per_step"] = round(loops_ms, 6)
        rec["checks"] = {"tol": REFUSE_TOL,
                         "dominant_fits_step": bool(dom_step_ms <= ms_per_step),
                         "dominant_fits_step_tol": bool(dom_step_ms <= ms_per_step * (1 + REFUSE_TOL)),
                         "all_loops_fit_step_tol": bool(loops_ms <= ms_per_step * (1 + REFUSE_TOL)),
                         "sampled_events_fit_step": bool(raw_step_ms <= ms_per_step)}
        if dom_ms <= 0 or dom_step_ms > ms_per_step * (1 + REFUSE_TOL):
            rec.update({"achieved": None, "frac": None,
                        "error": f"refused: the kernel's {len(dom_launches)} launches take {dom_step_ms:.6f} ms "
                                 f"back to back per {ms_per_step:.6f}-ms step"})
        return rec

    def scaled(self, ms_per_step: float) -> list:
        """Per-launch ms with the event overhead taken out: a dispatch with
        bound events ends a little later than an unbound one (its timestamps
        wait for the end-of-kernel release), a roughly fixed cost per timed
        dispatch.  When the launches' event times add up to more than the
        measured step, the excess is taken off every launch equally (at most
        half of any launch) -- not in proportion, which would over-credit the
        long dominant kernel.  Raw times stay in the line (event_ms)."""
        nl = self.desc["num_launches"]
        raw = sum(self.avg[:nl])
        if raw <= ms_per_step or nl == 0:
            return list(self.avg)
        per = (raw - ms_per_step) / nl
        return [t - min(per, 0.5 * t) for t in self.avg]

    def launches(self, ms_per_step: float) -> list:
        d, out = self.desc, []
        avg = self.scaled(ms_per_step)
        for i in range(d["num_launches"]):
            b = d["launch_bytes"][i]
            out.append({"kind": d["launch_kind"][i], "bytes": b, "ms": round(avg[i], 4),
                        "event_ms": round(self.avg[i], 4),
                        "GB/s": round(b / (avg[i] * 1e-3) / 1e9, 1) if avg[i] > 0 else None})
        return out

    def free(self):
        self.plan.close()
        self.x = self.y = None
        self.torch.cuda.empty_cache()


def secondary_configs(pifft, torch, gpu, steps, warmup, seed, cpu_threads, with_cpu) -> dict:
    """Configs 1-3 of BASELINE.json on this one GPU, each a separate timed loop
    (same contract as the headline step) with its own roofline and a reference
    CPU baseline at the same N."""
    F64, F32 = pifft.F64, pifft.F32
    cases = [
        ("C1", "config 1: fp64 N=2^20, 1 worker", dict(log_n=20, prec=F64, P=1, first=0, count=1, batch=1),
         dict(log_n=20, prec=64, workers=1, repeat=3)),
        ("C2", "config 2: fp64 N=2^20, 8 workers on one GPU (natural order)",
         dict(log_n=20, prec=F64, P=8, first=0, count=8, batch=1), dict(log_n=20, prec=64, workers=8, repeat=5)),
        ("C2_slice", "config 2, one GPU's slice: worker 0 of the 8-way split (rated as the whole transform)",
         dict(log_n=20, prec=F64, P=8, first=0, count=1, batch=1),
         dict(log_n=20, prec=64, workers=8, repeat=5, slice_of=8)),
        ("C3", "config 3: batched fp32 4096 x N=4096", dict(log_n=12, prec=F32, P=1, first=0, count=1, batch=4096),
         dict(log_n=12, prec=32, workers=1, repeat=31, batch=4096)),
        ("C4_f32", "config 4 in the reference's own data_t: one fp32 complex N=2^28 transform",
         dict(log_n=28, prec=F32, P=1, first=0, count=1, batch=1), dict(log_n=28, prec=32)),
    ]
    out = {}
    for key, what, g, c in cases:
        rec = {"workload": what}
        try:
            n = 1 << g["log_n"]
            job = Job(pifft, torch, gpu, n=n, P=g["P"], prec=g["prec"], first=g["first"], count=g["count"],
                      batch_local=g["batch"], b_first=0, seed=seed)
            # small steps: more of them, so the timed loop is the steady state:
            # 1000 steps of the 10-50 us configs (10-45 ms, after 250 warm-up
            # steps).  Measured on one box (profiles/r04r_loop_length.txt):
            # 50 / 200 / 1000 steps -> config 3 45.4 / 48.2 / 44.4 us, config
            # 2's slice 12.6 / 12.3 / 12.25 us, config 2 30.0 / 29.4 / 29.1 us
            k = max(steps, int(os.environ.get("BENCH_SMALL_STEPS", "1000"))) if g["log_n"] < 24 else max(steps, 20)
            elapsed = job.run(k, max(warmup, int(os.environ.get("BENCH_SMALL_WARMUP", str(k // 4)))))  # (a quarter of the loop)
            ms = elapsed * 1e3 / k
            # the 10-50 us configs: 200 samples per launch (a few ms), so their
            # means hold to ~1 % against the rocprofv3 trace
            job.time_launches(200 if g["log_n"] < 24 else max(5, k // 2))
            flops = 5.0 * n * g["log_n"] * g["batch"]
            rf = job.roofline(ms)
            # PMC traffic of this very plan's dominant kernel, when a committed summary profiled it
            tkey = f"n2^{g['log_n']}_f{32 if g['prec'] == F32 else 64}_b{g['batch']}_P{g['P']}_q{g['count']}"
            rf["traffic"], rf["traffic_source"] = load_traffic(tkey, rf["launches"],
                                                               [job.plan.kernel_name(i) for i in rf["launches"]])
            rec.update({"value": round(flops / (ms * 1e-3) / 1e9, 2), "unit": "GFLOP/s", "ms_per_step": round(ms, 6),
                        "steps": k, "dtype": "f64" if g["prec"] == F64 else "f32", "n": n, "workers": g["P"],
                        "workers_in_plan": g["count"], "batch": g["batch"], "passes": job.desc["num_passes"],
                        "radix": job.desc["radix"], "launches": job.launches(ms), "roofline": rf})
            job.free()
        except Exception as e:  # reported, never silently replaced
            rec["error"] = repr(e)
        if with_cpu:
            try:
                rec["cpu_baseline"] = cpu_baseline(threads=cpu_threads, **c)
            except Exception as e:
                rec["cpu_baseline"] = {"value": None, "error": repr(e)}
        out[key] = rec
    return out


def _with_traffic(job, rf: dict, log_n: int, prec_bits: int) -> dict:
    """rf with the PMC traffic of this rank's plan (load_traffic: the committed
    profile of these very kernels, named by traffic_source), when one exists."""
    key = f"n2^{log_n}_f{prec_bits}_b{job.batch_local}_P{job.P}_q{job.count}"
    try:
        rf["traffic"], rf["traffic_source"] = load_traffic(key, rf["launches"],
                                                           [job.plan.kernel_name(i) for i in rf["launches"]])
    except Exception as e:  # (optional: never costs the config its numbers)
        rf["traffic"], rf["traffic_source"] = None, f"error: {e!r}"[:160]
    return rf


C5_HEADROOM = 4 << 30  # HBM left free beside config 5's largest phase


def c5_hbm_need(n: int, world: int, esz: int = 16) -> int:
    """Config 5's peak HBM per GPU: the timed phase holds the input replica, the
    slice and the plan's workspace (n + 2 n/world values), and rank 0's
    verification replays another rank's plan beside them (+ 2 n/world); the
    exchange, after the replica and the plan are freed, holds the slice, the
    gathered buffer and the natural-order result (n/world + 2 n)."""
    return max(n + 4 * (n // world), n // world + 2 * n) * esz + C5_HEADROOM


def all_ranks_ok(ok: bool, dist, red_dev) -> bool:
    """True only if every rank says ok (one all-reduce, so that all ranks take
    the same branch and no collective is left waiting on a rank that skipped)."""
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=red_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def config5(pifft, torch, dist, gpu, rank, world, steps, warmup, seed, barrier, red_dev, log_n=32,
            same_device=False) -> dict:
    """Config 5 on a multi-GPU job: fp64 N=2^32 split over `world` GPUs (one
    worker per GPU, 64 GiB input replica each), then the RCCL all-gather and
    interleave into natural order (timed separately).  log_n < 32: a smaller
    rehearsal of the same code path.  Every rank first checks its free HBM
    against the config's peak (c5_hbm_need); if any rank is short, all ranks
    report the error instead of allocating (no out-of-memory mid-collective)."""
    import pifft_dist
    n = 1 << log_n
    rec = {"workload": f"config 5: fp64 N=2^{log_n} over {world} GPUs, one worker each (no data-path collective), "
                       f"then the all-gather ({'RCCL' if dist.get_backend() == 'nccl' else dist.get_backend()}) "
                       f"+ interleave"}
    torch.cuda.empty_cache()
    free, total = torch.cuda.mem_get_info(gpu)
    need = c5_hbm_need(n, world)
    if same_device:
        need = need * world  # every rehearsal rank shares one GPU
    rec["hbm_need_GiB"], rec["hbm_free_GiB"] = round(need / 2**30, 2), round(free / 2**30, 2)
    if not all_ranks_ok(free >= need, dist, red_dev):
        rec["error"] = (f"not run: config 5 needs {need / 2**30:.1f} GiB of HBM per GPU and at least one rank has "
                        f"less free (this rank {free / 2**30:.1f} of {total / 2**30:.1f} GiB)")
        return rec
    job = Job(pifft, torch, gpu, n=n, P=world, prec=pifft.F64, first=rank, count=1, batch_local=1, b_first=0,
              seed=seed)
    local_s = job.run(steps, warmup, barrier)
    elapsed = pifft_dist.max_over_ranks(local_s, red_dev)
    ms = elapsed * 1e3 / steps
    job.time_launches(max(3, steps))
    rec.update({"value": round(5.0 * n * log_n / (ms * 1e-3) / 1e9, 2), "unit": "GFLOP/s",
                "ms_per_step": round(ms, 6), "steps": steps, "launches": job.launches(local_s * 1e3 / steps),
                "roofline_rank0": _with_traffic(job, job.roofline(local_s * 1e3 / steps), log_n, 64)
                if rank == 0 else None})

    def _drop_replica():
        job.x = None  # the 64 GiB replica is not needed by the exchange
        job.plan.close()  # nor the plan's workspace
        torch.cuda.empty_cache()
    exchange_and_verify(pifft, torch, dist, job, rank, world, barrier, red_dev, rec, between=_drop_replica)
    job.free()
    return rec


def multi_secondary(pifft, torch, dist, gpu, rank, world, steps, warmup, seed, barrier, red_dev) -> dict:
    """Configs 2 and 3 on a multi-GPU job, each a timed loop with the headline's
    barrier + max-over-ranks contract: C2's 8 workers split over the GPUs
    (the reference's 8-way split on real GPUs: one worker per GPU at 8, 8/G
    at G = 1, 2, 4), C3's 4096 transforms sharded by transform over the GPUs.
    Rank 0's dominant-kernel roofline comes from the same loop; the worker
    split checks itself (exchange_and_verify, at one rank too)."""
    import pifft_dist
    F64, F32 = pifft.F64, pifft.F32
    b0, bc = pifft_dist.batch_range(rank, world, 4096)
    p2 = 8 if 8 % world == 0 else world
    f2, c2 = pifft_dist.worker_range(rank, world, p2)
    cases = [
        ("C2_split", f"config 2: fp64 N=2^20, {p2} workers split over {world} GPU(s), {c2} each (no data-path "
                     f"collective)", 20, F64, dict(P=p2, first=f2, count=c2, batch_local=1, b_first=0), 1),
        ("C3_batch", f"config 3: batched fp32 4096 x N=4096 sharded by transform over {world} GPUs",
         12, F32, dict(P=1, first=0, count=1, batch_local=bc, b_first=b0), 4096),
    ]
    out = {}
    for key, what, log_n, prec, g, batch in cases:
        rec = {"workload": what}
        try:
            job = Job(pifft, torch, gpu, n=1 << log_n, prec=prec, seed=seed, **g)
            k = max(steps, 1000)  # (as the one-GPU secondaries: the steady state)
            local_s = job.run(k, max(warmup, k // 4), barrier)
            elapsed = pifft_dist.max_over_ranks(local_s, red_dev)
            ms = elapsed * 1e3 / k
            job.time_launches(200)
            rec.update({"value": round(5.0 * (1 << log_n) * log_n * batch / (ms * 1e-3) / 1e9, 2),
                        "unit": "GFLOP/s", "ms_per_step": round(ms, 6), "steps": k, "n_gpus": world,
                        "dtype": "f64" if prec == F64 else "f32", "batch_per_gpu": g["batch_local"],
                        "roofline_rank0": _with_traffic(job, job.roofline(local_s * 1e3 / k), log_n,
                                                        64 if prec == F64 else 32) if rank == 0 else None})
            if key == "C2_split":  # a worker split: check it (slices bitwise, gathered result vs one GPU)
                exchange_and_verify(pifft, torch, dist, job, rank, world, barrier, red_dev, rec)
            job.free()
        except Exception as e:  # reported, never silently replaced
            rec["error"] = repr(e)
        out[key] = rec
    return out


# direct DFT bins instead of a whole one-GPU reference transform above this
# many elements (config 5: an all-worker 2^32 plan would need 192 GiB on rank 0)
VERIFY_WHOLE_MAX = 1 << 30


def verify_prepare(pifft, torch, dist, job, rank: int, world: int) -> dict:
    """The first multi-GPU run checks its own result (round-3 verdict), after
    the timed region.  Collective: every rank calls it.
      slices_bitwise -- every rank's slice-major result equals, bit for bit,
        the same worker range's plan replayed on rank 0's GPU over rank 0's
        replica of the input (integer digests, pifft_dist.tensor_digest; the
        kernels are deterministic, so any difference is a fault of the
        multi-GPU path: a wrong worker range, replica or device);
      the references for the natural-order result (kept on rank 0 for
        verify_finish): a one-GPU all-worker plan of the same input
        (N <= 2^30), and direct float64 DFT bins (pifft_dist.dft_bins) of each
        worker's bins (fp64, one transform: config 5 too, beyond what the
        reference can express)."""
    import pifft_dist
    torch.cuda.synchronize(job.dev)
    digests = [None] * world
    dist.all_gather_object(digests, pifft_dist.tensor_digest(job.y))
    if rank != 0:
        return {}
    _fault("verify", rank)
    st = job.stream
    same = []
    for q in range(world):
        first, count = pifft_dist.worker_range(q, world, job.P)
        if q == 0:
            same.append(True)  # (rank 0's own slice is the replay's reference)
            continue
        plan = pifft.Plan(job.n, job.P, job.batch_local, job.prec, first=first, count=count, device=job.dev.index,
                          flags=pifft.OUT_SLICES)
        out = torch.empty(plan.describe()["out_elems"], dtype=job.y.dtype, device=job.dev)
        plan.execute_device(job.x.data_ptr(), out.data_ptr(), st)
        torch.cuda.synchronize(job.dev)
        same.append(pifft_dist.tensor_digest(out) == tuple(digests[q]))
        plan.close()
        del out
    prep = {"slices_bitwise": all(same), "slices_checked": world,
            "slices_differing": [q for q, ok in enumerate(same) if not ok]}
    n, b = job.n, job.batch_local
    prep["tol"] = 1e-12 if job.prec == pifft.F64 else 1e-5 * (n.bit_length() - 1)
    if n * b <= VERIFY_WHOLE_MAX:
        plan = pifft.Plan(n, job.P, b, job.prec, device=job.dev.index)  # all P workers, natural order
        ref = torch.empty(n * b, dtype=job.y.dtype, device=job.dev)
        plan.execute_device(job.x.data_ptr(), ref.data_ptr(), st)
        torch.cuda.synchronize(job.dev)
        plan.close()
        prep["ref"] = ref
        prep["reference"] = f"one-GPU all-worker plan (P={job.P}, natural order) on rank 0, same input"
    if b == 1 and job.prec == pifft.F64:  # (cheap: also beside the whole reference)
        ks = pifft_dist.sample_bins(n, job.P)
        prep["ks"] = ks
        prep["bins"] = pifft_dist.dft_bins(job.x, ks)
        prep["x_norm"] = float(torch.linalg.vector_norm(job.x))
        prep["reference"] = (prep.get("reference", "") + "; " if "reference" in prep else "") + \
            f"{len(ks)} direct float64 DFT bins ({len(ks) // job.P} per worker, GEMM over the input)"
    return prep


def verify_finish(torch, prep: dict, natural) -> dict | None:
    """Rank 0: the gathered natural-order result against verify_prepare's
    reference: rel-L2 (<= the north star's tolerance) and/or the direct bins
    (each within 50 x tol x rms(X), rms(X) = ||x|| by Parseval; a misplaced bin
    is off by ~rms)."""
    if not prep:
        return None
    rec = {k: prep[k] for k in ("slices_bitwise", "slices_checked", "slices_differing", "tol", "reference")
           if k in prep}
    rec["rel_l2"] = rec["bins_ok"] = None
    ok = prep["slices_bitwise"]
    if natural is not None and "ref" in prep:
        ref = prep["ref"]
        err = float(torch.linalg.vector_norm(natural - ref) / torch.linalg.vector_norm(ref))
        rec["rel_l2"] = err
        ok = ok and err <= prep["tol"]
    if natural is not None and "ks" in prep:
        ks = torch.tensor(prep["ks"], dtype=torch.int64, device=natural.device)
        worst = float(torch.max(torch.abs(natural[ks] - prep["bins"])))
        bound = 50 * prep["tol"] * prep["x_norm"]
        rec.update({"bins": len(prep["ks"]), "bins_max_err": worst, "bins_bound": bound, "bins_ok": worst <= bound})
        ok = ok and worst <= bound
    if natural is None:
        rec["note"] = "no all-gather (--no-allgather): slices only"
    rec["ok"] = bool(ok)
    return rec


def exchange_and_verify(pifft, torch, dist, job, rank, world, barrier, red_dev, rec: dict, verify: bool = True,
                        gather: bool = True, between=None) -> None:
    """The optional stages after a multi-GPU timed loop, none of which may
    cost the line (round-4 verdict): the split's self-check (verify_prepare,
    rank 0 replaying the other ranks' plans), the all-gather + interleave
    and the comparison of the gathered result.  Every failure becomes
    rec["verify_error"] / rec["allgather_error"]; after each stage the ranks
    agree (all_ranks_ok, one all-reduce) whether to go on, so a stage that
    failed on one rank only (rank 0's replay running out of HBM, say) never
    leaves the others waiting in a collective.  `between`: run after the
    preparation (config 5 frees its replica there)."""
    prep = None
    if verify:
        prep = guarded(rec, "verify_error", verify_prepare, pifft, torch, dist, job, rank, world)
        if not all_ranks_ok("verify_error" not in rec, dist, red_dev):
            rec.setdefault("verify_error", "skipped: the self-check failed on another rank")
            prep = None
    if between is not None:
        between()
    natural = None
    if gather:
        def _exchange():
            ms, nat = allgather(pifft, torch, dist, job, barrier, red_dev, keep=prep is not None and rank == 0)
            _fault("allgather", rank)
            return ms, nat
        got = guarded(rec, "allgather_error", _exchange)
        if all_ranks_ok(got is not None, dist, red_dev):
            rec["allgather_ms"] = round(got[0], 3)
            natural = got[1]
        else:
            rec.setdefault("allgather_error", "skipped: the exchange failed on another rank")
    if prep is not None and "allgather_error" not in rec:
        rec["verify"] = guarded(rec, "verify_error", verify_finish, torch, prep, natural if gather else None)


def allgather(pifft, torch, dist, job, barrier, red_dev, keep: bool = False):
    """The optional final exchange: RCCL all-gather of every rank's result,
    then -- for a worker split -- the stride-P interleave into natural order on
    every GPU (ms, max over ranks).  A batch-sharded job (every plan holds all
    P workers, count == P) gathers whole transforms already in natural order:
    no interleave.  With several transforms per rank the gathered buffer is
    rank-major (rank, transform, slices) and is reordered to the
    transform-major slice layout the interleave reads.  Returns (ms, the
    natural-order result if keep else None)."""
    import pifft_dist
    torch.cuda.synchronize(job.dev)
    barrier()
    ta = time.perf_counter()
    gathered = pifft_dist.allgather_slices(job.y)
    natural = None
    if job.count < job.P:
        world = gathered.numel() // job.y.numel()
        batch = job.batch_local
        gathered = pifft_dist.slices_transform_major(gathered, world, batch)
        natural = torch.empty(job.n * batch, dtype=job.y.dtype, device=job.dev)
        pifft.interleave_device(gathered.data_ptr(), natural.data_ptr(), job.n, job.P, batch, job.prec, job.stream)
    elif keep:
        natural = gathered.reshape(-1)  # whole transforms in natural order (a world-size-1 group: its own result)
    torch.cuda.synchronize(job.dev)
    ms = pifft_dist.max_over_ranks((time.perf_counter() - ta) * 1e3, red_dev)
    del gathered
    return ms, (natural if keep else None)


# ---------------------------------------------------------------------------
# The printed line and its sidecar.  The driver keeps the last ~8 KB of
# stdout (round-4 verdict: the ~15 KB line lost configs 1 and 2 from the
# record), so the line carries each config's numbers only -- value, step,
# roofline {kernel_name, mean_ms, frac, traffic}, cpu_baseline {value, cores,
# ms} -- and the per-launch detail goes to a sidecar JSON (--detail).
LINE_MAX_CHARS = 7000

_RF_KEYS = ("bound", "kernel_name", "launches", "mean_ms", "loop_reps", "trace_loop_dispatches", "achieved",
            "peak", "unit", "frac", "traffic", "traffic_source", "algorithmic_bytes", "kernel_ms_per_step", "all_launches_ms_per_step",
            "step_ms", "step_frac", "checks", "error")
_RF_SECONDARY = ("kernel_name", "launches", "mean_ms", "loop_reps", "trace_loop_dispatches", "achieved", "peak",
                 "frac", "traffic", "traffic_source", "algorithmic_bytes", "step_frac", "error")
_CPU_KEYS = ("value", "unit", "cores", "kind", "ms", "sample", "cpu_model", "cpu_share", "error")


def _pick(d, keys):
    return None if d is None else {k: d[k] for k in keys if k in d}


def _short_sample(cb: dict) -> dict:
    """cpu_baseline for the line: the sample's first clause (what ran, at what
    size and p) stands for the full prose kept in the sidecar."""
    out = _pick(cb, _CPU_KEYS)
    if out and isinstance(out.get("sample"), str):
        out["sample"] = out["sample"].split(";")[0][:160]
    alt = cb.get("alternative") if cb else None
    if alt:
        out["alternative"] = _pick(alt, ("value", "cores", "ms", "error"))
    if cb and cb.get("O0"):
        out["O0"] = _pick(cb["O0"], ("value", "cores", "ms", "error"))
    return out


def compact_secondary(sec: dict | None) -> dict | None:
    if not sec:
        return sec
    out = {}
    for key, rec in sec.items():
        c = {k: rec[k] for k in ("value", "ms_per_step", "dtype", "n", "workers", "workers_in_plan", "batch",
                                 "batch_per_gpu", "n_gpus", "allgather_ms", "hbm_need_GiB", "hbm_free_GiB",
                                 "error", "allgather_error") if k in rec}
        for rk in ("roofline", "roofline_rank0"):
            if rec.get(rk) is not None:
                c[rk] = _pick(rec[rk], _RF_SECONDARY)
                if isinstance(rec[rk].get("checks"), dict):  # (each check in the sidecar)
                    c[rk]["checks_ok"] = all(v for k, v in rec[rk]["checks"].items() if k != "tol" and
                                             k != "sampled_events_fit_step")
        if "cpu_baseline" in rec:
            cb = rec["cpu_baseline"] or {}
            c["cpu_baseline"] = _pick(cb, ("value", "cores", "kind", "ms", "error"))
        if rec.get("verify") is not None:
            c["verify"] = _pick(rec["verify"], ("ok", "slices_bitwise", "slices_checked", "rel_l2", "bins_ok",
                                                "bins_max_err", "error", "note"))
        out[key] = c
    return out


def compact_line(full: dict) -> dict:
    """The printed line: the contract's keys, the headline config's numbers
    and each secondary config's summary; lists of launches and prose go to
    the sidecar (config.detail names it)."""
    line = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data")}
    cfg = full["config"]
    c = {k: cfg[k] for k in ("workload", "n", "workers", "workers_per_gpu", "batch", "batch_per_gpu", "shard",
                             "local_n", "passes", "parallelism", "hbm_GBps_per_step_algorithmic", "allgather_ms",
                             "allgather_error", "verify_error", "per_rank_error", "emulated_rank", "stage",
                             "detail") if k in cfg}
    if cfg.get("verify") is not None:
        c["verify"] = _pick(cfg["verify"], ("ok", "slices_bitwise", "slices_checked", "rel_l2", "bins_ok",
                                            "bins_max_err", "error", "note"))
    if cfg.get("per_rank") is not None:
        c["per_rank"] = [_pick(r, ("rank", "ms_per_step", "dominant_ms", "frac")) for r in cfg["per_rank"]]
    if cfg.get("secondary") is not None:
        c["secondary"] = compact_secondary(cfg["secondary"])
    line["config"] = c
    line["roofline"] = _pick(full["roofline"], _RF_KEYS)
    line["cpu_baseline"] = _short_sample(full["cpu_baseline"]) if full.get("cpu_baseline") else full.get("cpu_baseline")
    return line


def emit(full: dict, detail_path: str | None) -> str:
    """Writes the full record to the sidecar, prints the compact line (one
    line, flushed) and returns it.  A line still over LINE_MAX_CHARS drops
    its secondary summaries' verify objects, then the per-rank list."""
    if detail_path:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(detail_path)), exist_ok=True)
            with open(detail_path, "w") as f:
                json.dump(full, f, indent=1)
        except OSError as e:
            full["config"]["detail"] = f"not written: {e!r}"
    line = compact_line(full)
    s = json.dumps(line)
    if len(s) > LINE_MAX_CHARS:
        for rec in (line["config"].get("secondary") or {}).values():
            rec.pop("verify", None)
        s = json.dumps(line)
    if len(s) > LINE_MAX_CHARS and line["config"].get("per_rank"):
        line["config"]["per_rank"] = "in the sidecar"
        s = json.dumps(line)
    print(s, flush=True)
    return s


def guarded(rec: dict, key: str, fn, *a, **kw):
    """fn(*a, **kw), an exception becoming rec[key] (repr) and None: the
    optional stages after the timed region never cost the line."""
    try:
        return fn(*a, **kw)
    except Exception as e:  # reported, never silently replaced
        rec[key] = repr(e)[:400]
        return None


def _fault(stage: str, rank: int) -> None:
    """Test-only fault injection (BENCH_FAULT=<stage>[:rank], read only under
    PIFFT_TUNING=1 like libpifft's PIFFT_FAULT): raises in that stage on that
    rank (default rank 0), to check that the line survives."""
    spec = os.environ.get("BENCH_FAULT", "") if os.environ.get("PIFFT_TUNING") == "1" else ""
    if not spec:
        return
    st, _, r = spec.partition(":")
    if st == stage and rank == int(r or 0):
        raise RuntimeError(f"injected fault in {stage} on rank {rank} (BENCH_FAULT)")


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1, help="GPUs (= ranks, one process per GPU)")
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
    ap.add_argument("--allgather", dest="allgather", action="store_true", default=True,
                    help="at G > 1, time the optional RCCL all-gather + interleave after the timed region (default)")
    ap.add_argument("--no-allgather", dest="allgather", action="store_false")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip configs 1-3 (at 1 GPU) / 2-3 split over the GPUs and 5 (at 8 GPUs) beside the "
                         "headline step")
    ap.add_argument("--c5-log-n", type=int, default=32,
                    help="config 5 size at 8 GPUs (default 2^32; smaller only to rehearse the code path)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-log-n", type=int, default=0, help="CPU baseline size (default: the headline N)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="reference pthreads for the CPU baseline (default: the reference's own p_to = 32, "
                         "within the online CPUs and host memory)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL) or gloo")
    ap.add_argument("--pg", action="store_true",
                    help="open the process group even at one rank (with --dist-backend nccl: a world-size-1 RCCL "
                         "group on one GPU runs the multi-GPU code path -- init, barrier, device all-reduce, "
                         "all_gather_object, the all-gather and the self-check -- before any multi-GPU job does)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank uses cuda:0 (use with --dist-backend gloo)")
    ap.add_argument("--as-rank", default="",
                    help="q/G: run only rank q's plan of a G-GPU job, on this one GPU and without a process "
                         "group (per-rank profiling, e.g. tools/pmc_traffic.py); never a job-level number")
    ap.add_argument("--detail", default=os.environ.get("BENCH_DETAIL", os.path.join(ROOT, "gpurun_out",
                                                                                   "bench_detail.json")),
                    help="sidecar JSON with the full record (per-launch times, kernel names, prose); the printed "
                         "line keeps each config's numbers ('' = none)")
    args = ap.parse_args()

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and (args.gpus > 1 or args.pg):
        if args.as_rank:
            raise SystemExit("--as-rank emulates one rank on one GPU: use it without --gpus or --pg")
        return spawn_ranks(args.gpus)
    world = int(world_env or "1")
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} does not match the {world} rank(s) launched (WORLD_SIZE)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import pifft
    import pifft_dist

    emulated = None
    if args.as_rank:
        if world > 1 or args.pg:
            raise SystemExit("--as-rank is a single-process option without a process group")
        emulated = tuple(int(v) for v in args.as_rank.split("/"))
        if len(emulated) != 2 or not 0 <= emulated[0] < emulated[1]:
            raise SystemExit("--as-rank wants q/G with 0 <= q < G")
    gpu = 0 if args.same_device else local
    if not args.same_device and world > 1 and torch.cuda.device_count() < world:
        raise SystemExit(f"{world} ranks but only {torch.cuda.device_count()} GPU(s) visible "
                         f"(rehearse with --same-device --dist-backend gloo)")
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    if world > 1 or args.pg:
        import datetime
        import torch.distributed as dist
        # fail fast: a stuck collective on a first multi-GPU run ends in 3 min,
        # not at the default watchdog
        tmo = datetime.timedelta(seconds=int(os.environ.get("BENCH_DIST_TIMEOUT_S", "180")))
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
        else:
            dist.init_process_group(args.dist_backend, timeout=tmo)

    def barrier():
        if dist is not None:
            if args.dist_backend == "nccl":
                dist.barrier(device_ids=[gpu])
            else:
                dist.barrier()

    red_dev = dev if args.dist_backend == "nccl" else None  # gloo reduces on the CPU
    n = 1 << args.log_n
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

    job = Job(pifft, torch, gpu, n=n, P=P, prec=prec, first=first, count=count, batch_local=b_count,
              b_first=b_first, seed=args.seed)
    local_s = job.run(args.steps, args.warmup, barrier)
    elapsed = pifft_dist.max_over_ranks(local_s, red_dev)
    ms_per_step = elapsed * 1e3 / args.steps
    job.time_launches(max(5, args.steps // 2))  # after the timed region
    rf = job.roofline(local_s * 1e3 / args.steps)
    desc = job.desc
    kernel_names = [job.plan.kernel_name(i) for i in range(desc["num_launches"])]
    launches = job.launches(local_s * 1e3 / args.steps)
    config_key = f"n2^{args.log_n}_f{args.prec}_b{b_count}_P{P}_q{count}"
    rf["traffic"], rf["traffic_source"] = load_traffic(config_key, rf["launches"],
                                                       [job.plan.kernel_name(i) for i in rf["launches"]])

    total_bytes = sum(desc["launch_bytes"][: desc["num_launches"]])
    flops = 5.0 * n * args.log_n * args.batch  # the whole job's batch (every rank's share)
    value = flops / (ms_per_step * 1e-3) / 1e9
    full = {
        "metric": _baseline_metric(),
        "value": round(value, 2),
        "unit": "GFLOP/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 6),
        "higher_is_better": True,
        "scaling": "strong",  # the job's total work (one transform, or the global batch) is fixed
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
            "kernel_names": kernel_names,
            "hbm_bytes_per_step_algorithmic": total_bytes,
            "hbm_GBps_per_step_algorithmic": round(total_bytes / (ms_per_step * 1e-3) / 1e9, 1),
            "launches": launches,
            "parallelism": (f"batch-split {args.batch}/{world} per GPU, p{P}" if args.shard == "batch" else
                            f"pi-split p{P} over {world} GPU(s)"),
            "allgather_ms": None,
            "verify": None,
            "per_rank": None,
            "emulated_rank": args.as_rank or None,
            "secondary": None,
            "detail": os.path.relpath(args.detail, ROOT) if args.detail else None,
        },
        "roofline": rf,
        "cpu_baseline": None,
    }
    cfg = full["config"]
    if dist is not None and rank == 0:
        # the headline is complete here: print it before anything optional
        # runs (the first multi-GPU run executes the RCCL exchange for the
        # first time; CPU.c:485-492, worker 0 reports regardless of the
        # others).  The final line below repeats it with the rest.
        cfg["stage"] = "headline (the final line follows)"
        emit(full, args.detail)
    cfg["stage"] = None

    if dist is not None:
        mine = {"rank": rank, "gpu": gpu, "workers": [first, first + count], "batch": [b_first, b_first + b_count],
                "ms_per_step": round(local_s * 1e3 / args.steps, 6), "dominant_ms": rf["mean_ms"],
                "achieved": rf["achieved"], "frac": rf["frac"]}

        def _gather_rows():
            rows = [None] * world
            dist.all_gather_object(rows, mine)
            return rows
        cfg["per_rank"] = guarded(cfg, "per_rank_error", _gather_rows)

    # the optional exchange and the split's self-check (exchange_and_verify:
    # every failure an *_error field, all ranks on the same branch)
    if dist is not None and (args.shard == "batch" or count < P or world == 1):
        exchange_and_verify(pifft, torch, dist, job, rank, world, barrier, red_dev, cfg,
                            verify=args.shard == "workers" and (count < P or world == 1), gather=args.allgather)
    job.free()

    if not args.no_secondary and not emulated:
        if dist is None and args.log_n == 28 and args.prec == 64 and args.batch == 1:
            cfg["secondary"] = secondary_configs(pifft, torch, gpu, args.steps, args.warmup, args.seed,
                                                 args.cpu_threads, not args.no_cpu_baseline)
        elif dist is not None and args.shard == "workers":
            sec = guarded(cfg, "secondary_error", multi_secondary, pifft, torch, dist, gpu, rank, world,
                          args.steps, args.warmup, args.seed, barrier, red_dev)
            if sec is not None and world == 8:  # (config5 refuses cleanly when the HBM cannot hold it)
                try:
                    sec["C5"] = config5(pifft, torch, dist, gpu, rank, world, min(args.steps, 5),
                                        min(args.warmup, 2), args.seed, barrier, red_dev, args.c5_log_n,
                                        same_device=args.same_device)
                except Exception as e:  # reported, never silently replaced
                    sec["C5"] = {"error": repr(e)[:400]}
            cfg["secondary"] = sec

    if rank == 0:
        # rank 0 of every job (also N > 1, so the driver's scaling lines carry
        # it), after the GPU work: the other ranks do not wait for it
        if not emulated and not args.no_cpu_baseline:
            try:
                full["cpu_baseline"] = headline_cpu_baseline(args.cpu_log_n or args.log_n, args.prec,
                                                             batch=args.batch, threads=args.cpu_threads or None)
            except Exception as e:  # reported, never silently replaced
                full["cpu_baseline"] = {"value": None, "error": repr(e)}
        emit(full, args.detail)
    if dist is not None:
        guarded({}, "destroy", dist.destroy_process_group)
    return 0


if __name__ == "__main__":
    sys.exit(main())
