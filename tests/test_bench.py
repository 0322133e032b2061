"""bench.py's output contract (the driver parses its one JSON line): keys,
types, the BASELINE.json metric, the roofline and cpu_baseline objects, and
the batch-shard mode.  Small sizes; the timing itself is not judged here."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


LINE_MAX_CHARS = 7000  # bench.LINE_MAX_CHARS: the driver keeps the last ~8 KB of stdout


def _bench(*args, env_extra=None, tmp=None):
    """Runs bench.py; checks the printed line (one at N = 1; at N > 1 the
    headline first, printed before the optional exchange, then the final
    line) and returns the full record from its sidecar (--detail), with the
    printed line under "_line"."""
    import tempfile
    side = os.path.join(tmp or tempfile.mkdtemp(), "detail.json")
    env = dict(os.environ)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args, "--detail", side],
                       capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    multi = ("--gpus" in args and args[args.index("--gpus") + 1] != "1") or "--pg" in args
    assert len(lines) == (2 if multi else 1), r.stdout
    for ln in lines:
        assert len(ln) <= LINE_MAX_CHARS, len(ln)
    line = json.loads(lines[-1])
    if multi:
        first = json.loads(lines[0])
        assert first["config"]["stage"].startswith("headline") and line["config"].get("stage") is None
        assert first["value"] == line["value"] and first["ms_per_step"] == line["ms_per_step"]
    with open(side) as f:
        d = json.load(f)
    assert d["value"] == line["value"] and d["ms_per_step"] == line["ms_per_step"]
    assert line["roofline"].get("frac") == d["roofline"].get("frac")
    for key, rec in (d["config"].get("secondary") or {}).items():  # every config's numbers are in the line
        lrec = line["config"]["secondary"][key]
        assert lrec.get("value") == rec.get("value") and lrec.get("ms_per_step") == rec.get("ms_per_step")
    d["_line"] = line
    return d


def _common(d, steps, warmup, n_gpus=1):
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        assert d["metric"] == json.load(f)["metric"]
    assert d["unit"] == "GFLOP/s" and d["higher_is_better"] is True
    assert d["n_gpus"] == n_gpus and d["steps"] == steps and d["warmup"] == warmup
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert d["scaling"] in ("strong", "weak") and d["vs_baseline"] is None
    n = d["config"]["n"]
    # value = 5 N log2 N (x batch) / t
    flops = 5.0 * n * (n.bit_length() - 1) * d["config"]["batch"]
    # (ms_per_step is printed to 1e-6 ms)
    tol = d["value"] * (1e-3 + 1e-6 / d["ms_per_step"]) + 0.01
    assert abs(d["value"] - flops / (d["ms_per_step"] * 1e-3) / 1e9) <= tol
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert set(rf["checks"]) >= {"tol", "dominant_fits_step_tol", "all_loops_fit_step_tol"}
    _roofline_ok(rf, d["ms_per_step"] if n_gpus == 1 else None, contended=n_gpus > 1)
    assert len(d["config"]["launches"]) >= 1


def _roofline_ok(rf, ms_per_step=None, contended=False):
    """A roofline object is self-consistent: frac = achieved / peak, the
    dominant kernel's launches (a clean back-to-back loop) fit in the step
    (bench.py refuses beyond REFUSE_TOL) and all launches' sampled times fit
    in it too (their event overhead is scaled out).
    contended: a --same-device rehearsal rank, timed while 7 other ranks share
    its GPU -- bench.py may refuse that frac (the kernel's loop time beyond the
    step); the refusal is then all the object says."""
    if contended and rf.get("frac") is None:
        assert rf["error"].startswith("refused:") and rf["achieved"] is None, rf
        return
    assert "error" not in rf, rf
    assert 0 < rf["achieved"] and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert rf["algorithmic_bytes"] > 0
    assert 0 < rf["kernel_ms_per_step"] <= rf["step_ms"] * 1.03
    if not contended:
        assert rf["all_launches_ms_per_step"] <= rf["step_ms"] * (1 + 1e-6) + 1e-6
    assert rf["loop_reps"] >= 10 and rf["trace_loop_dispatches"] == rf["loop_reps"] * len(rf["launches"])
    if ms_per_step is not None:
        assert abs(rf["step_ms"] - ms_per_step) <= 1e-5 * ms_per_step + 1e-6


def test_bench_default_contract_small():
    d = _bench("--log-n", "20", "--steps", "3", "--warmup", "1", "--cpu-log-n", "16", "--cpu-threads", "2")
    _common(d, 3, 1)
    assert d["dtype"] == "f64" and d["config"]["workers"] == 1 and d["config"]["shard"] == "workers"
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] == 2 and cb["kind"] in ("reference", "port") and cb["sample"]


def test_bench_batch_shard_rank_share():
    d = _bench("--log-n", "12", "--prec", "32", "--batch", "64", "--shard", "batch", "--as-rank", "1/4",
               "--steps", "3", "--warmup", "1")
    _common(d, 3, 1)
    assert d["dtype"] == "f32" and d["config"]["batch_per_gpu"] == 16 and d["config"]["shard"] == "batch"
    assert d["cpu_baseline"] is None  # emulated rank: never a job-level CPU comparison


def test_bench_gpus_2_spawns_two_ranks():
    """--gpus 2 without torchrun launches two rank processes (rehearsed on one
    GPU with gloo): n_gpus 2, one record per rank, the all-gather timed."""
    d = _bench("--gpus", "2", "--same-device", "--dist-backend", "gloo", "--log-n", "20", "--steps", "3",
               "--warmup", "1", "--cpu-log-n", "16", "--cpu-threads", "2")
    _common(d, 3, 1, n_gpus=2)
    pr = d["config"]["per_rank"]
    assert [r["rank"] for r in pr] == [0, 1] and [r["workers"] for r in pr] == [[0, 1], [1, 2]]
    assert all(r["ms_per_step"] > 0 and (r["frac"] is None or 0 < r["frac"]) for r in pr)  # (None: refused, contended)
    # the job time is the slowest rank's
    assert d["ms_per_step"] >= max(r["ms_per_step"] for r in pr) * 0.999
    assert d["config"]["allgather_ms"] > 0
    # rank 0 carries the reference CPU baseline at N > 1 too (the driver's scaling lines)
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] == 2 and cb["kind"] == "reference"
    # configs 2 (one worker per GPU) and 3 (batch-sharded) as multi-GPU loops
    sec = d["config"]["secondary"]
    assert set(sec) == {"C2_split", "C3_batch"}
    for key, rec in sec.items():
        assert "error" not in rec, (key, rec)
        assert rec["value"] > 0 and rec["n_gpus"] == 2
    assert sec["C3_batch"]["batch_per_gpu"] == 2048
    # the split checks itself: slices bitwise vs rank 0's replay, the gathered result vs one GPU
    v = d["config"]["verify"]
    assert v["ok"] and v["slices_bitwise"] and v["slices_checked"] == 2 and v["rel_l2"] <= 1e-12, v
    assert sec["C2_split"]["verify"]["ok"], sec["C2_split"]["verify"]


def test_bench_gpus_8_rehearsal_config5():
    """The 8-GPU line's code path (the driver's scaling run), rehearsed with 8
    gloo ranks on one GPU and a small config 5: the headline, configs 2/3 split
    over the ranks, config 5 and its all-gather all report without error."""
    d = _bench("--gpus", "8", "--same-device", "--dist-backend", "gloo", "--log-n", "20", "--steps", "2",
               "--warmup", "1", "--c5-log-n", "22", "--no-cpu-baseline")
    _common(d, 2, 1, n_gpus=8)
    assert len(d["config"]["per_rank"]) == 8 and d["config"]["allgather_ms"] > 0
    sec = d["config"]["secondary"]
    assert set(sec) == {"C2_split", "C3_batch", "C5"}
    for key, rec in sec.items():
        assert "error" not in rec, (key, rec)
        assert rec["value"] > 0
    assert sec["C5"]["allgather_ms"] > 0 and sec["C3_batch"]["batch_per_gpu"] == 512
    assert sec["C5"]["hbm_free_GiB"] >= sec["C5"]["hbm_need_GiB"]
    for key in ("C2_split", "C3_batch"):
        _roofline_ok(sec[key]["roofline_rank0"], contended=True)
    _roofline_ok(sec["C5"]["roofline_rank0"], contended=True)
    # self-verification of every worker split (round-3 verdict: the first 8-GPU run proves itself)
    v = d["config"]["verify"]
    assert v["ok"] and v["slices_bitwise"] and v["slices_checked"] == 8 and v["rel_l2"] <= 1e-12, v
    assert sec["C2_split"]["verify"]["ok"] and sec["C5"]["verify"]["ok"], (sec["C2_split"]["verify"], sec["C5"]["verify"])
    assert sec["C5"]["verify"]["slices_bitwise"] and sec["C5"]["verify"]["rel_l2"] <= 1e-12
    assert v["bins_ok"] and sec["C5"]["verify"]["bins_ok"] and sec["C5"]["verify"]["bins"] == 64


def test_bench_config5_hbm_check_refuses_cleanly():
    """Config 5 checks every rank's free HBM against its peak before allocating:
    a size that cannot fit (2^34 fp64, 8 ranks on one GPU) is reported as an
    error by all ranks -- no out-of-memory mid-collective, no hang."""
    d = _bench("--gpus", "8", "--same-device", "--dist-backend", "gloo", "--log-n", "16", "--steps", "2",
               "--warmup", "1", "--c5-log-n", "34", "--no-cpu-baseline")
    c5 = d["config"]["secondary"]["C5"]
    assert "error" in c5 and "not run" in c5["error"] and c5["hbm_need_GiB"] > c5["hbm_free_GiB"]


def test_bench_secondary_configs():
    """The headline run also times configs 1, 2 (whole + one slice) and 3, each
    with its own dominant-kernel roofline (CPU baselines skipped here)."""
    d = _bench("--steps", "2", "--warmup", "1", "--no-cpu-baseline")
    _common(d, 2, 1)
    sec = d["config"]["secondary"]
    assert set(sec) == {"C1", "C2", "C2_slice", "C3", "C4_f32"}
    for key, rec in sec.items():
        assert "error" not in rec, (key, rec)
        flops = 5.0 * rec["n"] * (rec["n"].bit_length() - 1) * rec["batch"]
        assert abs(rec["value"] - flops / (rec["ms_per_step"] * 1e-3) / 1e9) <= rec["value"] * 1e-3 + 0.01
        _roofline_ok(rec["roofline"], rec["ms_per_step"])
        assert 0 < rec["roofline"]["frac"] < 1.0
    assert sec["C4_f32"]["dtype"] == "f32" and sec["C4_f32"]["n"] == 1 << 28
    assert sec["C3"]["dtype"] == "f32" and sec["C3"]["batch"] == 4096
    assert sec["C2"]["workers"] == 8 and sec["C2_slice"]["workers_in_plan"] == 1


def test_bench_exchange_failure_keeps_the_line():
    """An injected failure in the exchange (BENCH_FAULT, rank 0 after the
    collective) on a 2-rank rehearsal: both lines print, the final one with
    allgather_error, value and ms_per_step, and no rank hangs."""
    d = _bench("--gpus", "2", "--same-device", "--dist-backend", "gloo", "--log-n", "18", "--steps", "2",
               "--warmup", "1", "--no-cpu-baseline", "--no-secondary", env_extra={"BENCH_FAULT": "allgather:0"})
    line = d["_line"]
    assert line["value"] > 0 and line["ms_per_step"] > 0
    assert "injected" in line["config"]["allgather_error"] and line["config"]["allgather_ms"] is None
    assert line["config"].get("verify") is None


def test_bench_rccl_world_size_one():
    """The multi-GPU code path under RCCL, executed on one GPU (round-5 verdict:
    the driver's first 8-GPU run must not be its first execution): bench.py
    --pg opens a 1-rank nccl group through torchrun -- init_process_group with
    device_id, barrier(device_ids), the device-tensor all-reduce of
    max_over_ranks, all_gather_object, all_gather_into_tensor of the complex
    result, the self-check -- and configs 2 (8 workers on the one GPU) and 3
    (the 4096 transforms on one rank) as multi_secondary runs them."""
    d = _bench("--pg", "--dist-backend", "nccl", "--log-n", "20", "--steps", "3", "--warmup", "1",
               "--no-cpu-baseline")
    _common(d, 3, 1, n_gpus=1)
    cfg = d["config"]
    assert "per_rank_error" not in cfg and "allgather_error" not in cfg and "verify_error" not in cfg, cfg
    assert [r["rank"] for r in cfg["per_rank"]] == [0] and cfg["per_rank"][0]["gpu"] == 0
    assert cfg["allgather_ms"] > 0
    v = cfg["verify"]
    assert v["ok"] and v["slices_bitwise"] and v["slices_checked"] == 1 and v["rel_l2"] == 0.0 and v["bins_ok"], v
    sec = cfg["secondary"]
    assert set(sec) == {"C2_split", "C3_batch"}
    for key, rec in sec.items():
        assert "error" not in rec and "allgather_error" not in rec, (key, rec)
        assert rec["value"] > 0 and rec["n_gpus"] == 1
        _roofline_ok(rec["roofline_rank0"])
    assert sec["C3_batch"]["batch_per_gpu"] == 4096
    assert sec["C2_split"]["allgather_ms"] > 0 and sec["C2_split"]["verify"]["ok"], sec["C2_split"]
    assert "8 workers" in sec["C2_split"]["workload"]


_NCCL_ONE_RANK = r"""
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.path.join(sys.argv[1], "cs87project-msolano2_amd"))
import pifft_dist
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
try:
    assert dist.get_backend() == "nccl"
    g = torch.Generator(device="cpu").manual_seed(7)
    for dt in (torch.complex128, torch.complex64):
        x = torch.randn(3 * 4096, dtype=dt, generator=g).to(dev).view(3, 4096)
        y = pifft_dist.allgather_slices(x)
        assert y.is_cuda and y.dtype == dt and tuple(y.shape) == (3, 4096), (y.dtype, y.shape)
        assert torch.equal(torch.view_as_real(y).view(torch.int32), torch.view_as_real(x).view(torch.int32))
        assert pifft_dist.tensor_digest(y) == pifft_dist.tensor_digest(x)
    r = pifft_dist.allgather_slices(torch.arange(10, dtype=torch.float64, device=dev))
    assert torch.equal(r.cpu(), torch.arange(10, dtype=torch.float64))
    assert pifft_dist.max_over_ranks(1.25, dev) == 1.25
    rows = [None]
    dist.all_gather_object(rows, {"rank": 0, "ms": 1.5})
    assert rows == [{"rank": 0, "ms": 1.5}]
    dist.barrier(device_ids=[0])
    print("NCCL-ONE-RANK-OK", flush=True)
finally:
    dist.destroy_process_group()
"""


def test_pifft_dist_under_a_one_rank_rccl_group():
    """pifft_dist's collectives on device tensors under RCCL (a 1-rank nccl
    group on one GPU, in a child process): allgather_slices' complex view
    through all_gather_into_tensor returns the input's bytes (complex128 and
    complex64), max_over_ranks all-reduces a device tensor, all_gather_object
    and barrier(device_ids) complete."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", _NCCL_ONE_RANK, ROOT], capture_output=True, text=True, timeout=180,
                       env=env)
    assert r.returncode == 0 and "NCCL-ONE-RANK-OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])
