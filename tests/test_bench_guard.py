"""bench.py's line survives the optional stages (round-4 verdict: the first
8-GPU run executes the RCCL exchange for the first time, and a failure there
must not cost the headline), and the printed line stays short enough for the
driver's ~8 KB stdout tail with every config's numbers in it.  CPU only: the
multi-rank part runs bench.exchange_and_verify on world-size-2 gloo ranks
with stand-in stages (the GPU leg: test_bench.py's injected-fault run)."""
import json
import os
import socket
import sys

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

KNAME = "void pifft::k_pass<double, 1024, 8, 2, 1, 0, 16>(pifft::PassArgs)"


def _rf(nl=3):
    return {"bound": "hbm", "kernel": "pass kernel of launches [2] (mean launch 1.65750 ms: a clean loop of ...)",
            "kernel_name": KNAME, "launches": [nl - 1], "mean_ms": 1.657502, "loop_reps": 10,
            "trace_loop_dispatches": 10, "sampled_mean_ms": 1.66, "achieved": 5182.5, "peak": 8000.0,
            "unit": "GB/s", "frac": 0.6478, "algorithmic_bytes": 8589934592, "kernel_ms_per_step": 1.6575,
            "all_launches_ms_per_step": 4.52, "step_ms": 4.53, "event_ms_per_step": 4.6,
            "event_overhead_subtracted_ms": 0.01, "step_achieved": 5678.1, "step_frac": 0.7098,
            "loops_ms_per_step": 4.5, "traffic": 8592565621.03,
            "traffic_source": "profiles/r05_traffic_n2^28_f64_b1_P1_q1.json",
            "checks": {"tol": 0.03, "dominant_fits_step": True, "dominant_fits_step_tol": True,
                       "all_loops_fit_step_tol": True, "sampled_events_fit_step": False}}


def _cpu():
    return {"value": 12.29, "unit": "GFLOP/s", "cores": 16, "kind": "reference", "ms": 3057.573,
            "sample": "reference fourier-parallel-pi-cpu-pthreads built -O2 -Dfloat=double (oracle/_ref, from "
                      "the reference source), f64 N=2^28, p=16 pthreads; worker 0's tree+cylinder time 3057.6 ms "
                      "(the reference's own timer); process wall 31.0 s" + " x" * 200,
            "host_bytes_touched": 107374182400, "child_peak_rss_GiB": 99.99, "cpu_model": "AMD EPYC 9575F",
            "host_cpus": 256, "physical_cores": 128, "cpu_affinity": 256, "cgroup_cpu_quota": 16.0,
            "mem_available_GiB": 2920.8, "cgroup_mem_limit_GiB": 300.1, "cpu_share": 16, "selection": "x" * 120,
            "alternative": {"value": 7.1, "cores": 32, "ms": 5300.0, "sample": "y" * 300},
            "O0": {"value": 5.3, "cores": 16, "ms": 7100.0, "wall_s": 40.2}}


def _launches(nl):
    return [{"kind": "pass", "bytes": 8589934592, "ms": 1.4, "event_ms": 1.41, "GB/s": 6100.0}] * nl


def _sec_rec(n, nl=2):
    return {"workload": "config x: " + "w" * 120, "value": 4700.12, "unit": "GFLOP/s", "ms_per_step": 0.022301,
            "steps": 1000, "dtype": "f64", "n": n, "workers": 8, "workers_in_plan": 1, "batch": 1, "passes": nl,
            "radix": [1024] * nl, "launches": _launches(nl), "roofline": _rf(nl),
            "cpu_baseline": {k: v for k, v in _cpu().items() if k != "alternative"}}


def _full(world=1):
    nl = 3
    cfg = {"workload": "config 4: one fp64 complex N=2^28 pi-FFT, P=1 workers, 1 per GPU (no data-path collective)",
           "n": 1 << 28, "workers": world, "workers_per_gpu": 1, "batch": 1, "batch_per_gpu": 1, "shard": "workers",
           "local_n": (1 << 28) // world, "passes": nl, "radix": [512, 512, 1024], "lines_per_workgroup": [16, 16, 8],
           "kernel_names": [KNAME] * nl, "hbm_bytes_per_step_algorithmic": 25769803776,
           "hbm_GBps_per_step_algorithmic": 5678.1, "launches": _launches(nl), "parallelism": "pi-split p1",
           "allgather_ms": None, "verify": None, "per_rank": None, "emulated_rank": None, "secondary": None,
           "detail": "gpurun_out/bench_detail.json"}
    if world == 1:
        cfg["secondary"] = {k: _sec_rec(n) for k, n in (("C1", 1 << 20), ("C2", 1 << 20), ("C2_slice", 1 << 20),
                                                         ("C3", 1 << 12), ("C4_f32", 1 << 28))}
    else:
        cfg["per_rank"] = [{"rank": r, "gpu": r, "workers": [r, r + 1], "batch": [0, 1], "ms_per_step": 1.26,
                            "dominant_ms": 0.88, "achieved": 5500.0, "frac": 0.69} for r in range(world)]
        cfg["allgather_ms"] = 420.5
        ver = {"slices_bitwise": True, "slices_checked": world, "slices_differing": [], "tol": 1e-12,
               "reference": "r" * 200, "rel_l2": 5e-16, "bins_ok": True, "bins": 64, "bins_max_err": 1e-15,
               "bins_bound": 1e-9, "ok": True}
        cfg["verify"] = ver
        sec = {}
        for key in ("C2_split", "C3_batch", "C5"):
            r = _sec_rec(1 << 20)
            r.pop("roofline")
            r.pop("cpu_baseline")
            r.update({"roofline_rank0": _rf(), "n_gpus": world, "verify": dict(ver), "allgather_ms": 3.2})
            sec[key] = r
        sec["C5"].update({"hbm_need_GiB": 132.0, "hbm_free_GiB": 280.0})
        cfg["secondary"] = sec
    return {"metric": bench._baseline_metric(), "value": 8280.56, "unit": "GFLOP/s", "n_gpus": world, "steps": 20,
            "warmup": 5, "ms_per_step": 4.538455, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic: splitmix64 U[-1,1]/sqrt(N) complex input generated in HBM",
            "config": cfg, "roofline": _rf(), "cpu_baseline": _cpu()}


@pytest.mark.parametrize("world", [1, 2, 8])
def test_line_fits_the_driver_tail_with_every_config(world, tmp_path, capsys):
    full = _full(world)
    side = tmp_path / "detail.json"
    s = bench.emit(full, str(side))
    out = capsys.readouterr().out.strip().splitlines()
    assert out == [s] and len(s) <= bench.LINE_MAX_CHARS, len(s)
    line = json.loads(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in line
    rf = line["roofline"]
    assert rf["frac"] == 0.6478 and rf["traffic"] and rf["kernel_name"] == KNAME and rf["checks"]["tol"] == 0.03
    # the counters name their source: the committed PMC summary, not this run
    assert rf["traffic_source"].startswith("profiles/") and "traffic" in rf["traffic_source"]
    assert line["cpu_baseline"]["value"] == 12.29 and line["cpu_baseline"]["cores"] == 16
    assert line["cpu_baseline"]["alternative"]["cores"] == 32
    # the reference Makefile's own -O0 build beside the -O2 one
    assert line["cpu_baseline"]["O0"] == {"value": 5.3, "cores": 16, "ms": 7100.0}
    sec = line["config"]["secondary"]
    want = {"C1", "C2", "C2_slice", "C3", "C4_f32"} if world == 1 else {"C2_split", "C3_batch", "C5"}
    assert set(sec) == want
    for rec in sec.values():
        r = rec.get("roofline") or rec.get("roofline_rank0")
        assert rec["value"] and rec["ms_per_step"] and r["frac"] and r["traffic"] and r["mean_ms"]
        assert r["traffic_source"].startswith("profiles/")
        if world == 1:
            assert rec["cpu_baseline"]["value"] and rec["cpu_baseline"]["cores"] and rec["cpu_baseline"]["ms"]
    if world > 1:
        assert len(line["config"]["per_rank"]) == world and line["config"]["verify"]["ok"]
    # the sidecar holds the full record
    d = json.loads(side.read_text())
    assert d["config"]["launches"] and d["config"]["kernel_names"] and d == json.loads(json.dumps(full))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _FakeJob:
    pass


def _guard_rank(rank, world, port, fault, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if fault:
        os.environ["BENCH_FAULT"] = fault
        os.environ["PIFFT_TUNING"] = "1"  # (BENCH_FAULT is read only under it)
    sys.path.insert(0, ROOT)
    import bench as b
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def fake_prepare(pifft, torch_, dist_, job, rank_, world_):
            rows = [None] * world_
            dist_.all_gather_object(rows, rank_)
            if rank_ != 0:
                return {}
            b._fault("verify", rank_)
            return {"slices_bitwise": True, "slices_checked": world_, "slices_differing": [], "tol": 1e-12}

        def fake_allgather(pifft, torch_, dist_, job, barrier, red_dev, keep=False):
            parts = [torch.zeros(4) for _ in range(world)]
            dist_.all_gather(parts, torch.full((4,), float(rank)))
            return 1.5, None

        b.verify_prepare = fake_prepare
        b.allgather = fake_allgather
        rec = {}
        b.exchange_and_verify(None, torch, dist, _FakeJob(), rank, world, lambda: None, None, rec)
        # every rank still reaches the same next collective (no rank left waiting)
        t = None
        dist.barrier()
        full = _full(world)
        full["config"].update({k: rec.get(k) for k in ("allgather_ms", "verify")})
        full["config"].update({k: v for k, v in rec.items() if k.endswith("_error")})
        line = None
        if rank == 0:
            import io
            import contextlib
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                b.emit(full, None)
            line = json.loads(buf.getvalue().strip().splitlines()[-1])
        q.put((rank, rec, line, t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fault", ["", "allgather:0", "allgather:1", "verify:0"])
def test_exchange_failure_keeps_the_line(fault):
    """An injected failure in the all-gather (on rank 0 or 1) or in rank 0's
    self-check: both ranks finish (the others skip, no collective left
    waiting), the failing stage is reported as *_error and rank 0's line
    still parses with value and ms_per_step."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_guard_rank, args=(r, world, port, fault, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, rec, line, _ = q.get(timeout=120)
        res[rank] = (rec, line)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    rec0, line = res[0]
    assert line["value"] == 8280.56 and line["ms_per_step"] == 4.538455
    if not fault:
        assert rec0["allgather_ms"] == 1.5 and rec0["verify"]["ok"] and not any(k.endswith("_error") for k in rec0)
        return
    stage, _, r = fault.partition(":")
    key = "allgather_error" if stage == "allgather" else "verify_error"
    for rank, (rec, _) in res.items():
        assert key in rec, (rank, rec)
        assert ("injected" in rec[key]) == (rank == int(r)), (rank, rec[key])
    assert key in line["config"]
    if stage == "verify":  # the self-check is dropped on every rank; the exchange still runs
        assert rec0["allgather_ms"] == 1.5 and "verify" not in rec0
    else:
        assert "allgather_ms" not in rec0 and "verify" not in rec0


def test_bench_fault_needs_the_tuning_switch(monkeypatch):
    """BENCH_FAULT is a test-only switch: without PIFFT_TUNING=1 a stray one in
    the driver's environment injects nothing."""
    monkeypatch.setenv("BENCH_FAULT", "allgather:0")
    monkeypatch.delenv("PIFFT_TUNING")
    bench._fault("allgather", 0)  # no exception
    monkeypatch.setenv("PIFFT_TUNING", "1")
    with pytest.raises(RuntimeError, match="injected"):
        bench._fault("allgather", 0)
