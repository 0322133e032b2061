"""bench.py's host-side logic (no GPU): the --gpus / WORLD_SIZE contract and
the CPU-baseline sizing rule (the reference needs (2 + 2P) S bytes of host
memory, CPU.c:225-239, 396-407)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _run(args, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=60, env=env)


def test_gpus_must_match_world_size():
    r = _run(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "does not match the 2 rank(s)" in r.stderr
    r = _run(["--gpus", "8"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "--gpus 8 does not match" in r.stderr


def test_as_rank_is_single_process():
    r = _run(["--gpus", "2", "--as-rank", "0/2"], {})
    assert r.returncode != 0 and "--as-rank" in r.stderr


def test_reference_touched_memory_model():
    """The reference's touched host memory (in + per worker tmp_in + the tmp_out
    pages its levels write, CPU.c:220-247, 396-478): 3 S at p = 1, and 49 S
    (196 GiB at fp64 2^28) at the reference's p_to = 32."""
    n = 1 << 28
    assert bench.ref_touched_elems(n, 1) == 3 * n
    assert bench.ref_touched_elems(n, 32) == 49 * n
    vals = [bench.ref_touched_elems(1 << 12, 1 << k) for k in range(6)]
    assert vals == sorted(vals)


@pytest.mark.parametrize("avail_gib,cpus,share,threads,log_n,esz,want", [
    (2900, 256, 16, None, 28, 16, 16),  # the GPU box: 256 online CPUs, a 16-CPU cgroup quota -> p = 16
    (2900, 256, 256, None, 28, 16, 32),  # no quota: the reference's p_to = 32 (196 GiB) under the per-command cap
    (2900, 256, 16, 32, 28, 16, 32),    # --cpu-threads 32
    (100, 256, 256, None, 28, 16, 8),   # 72 GiB budget: p = 8 touches 52 GiB, p = 16 100 GiB
    (2900, 8, 8, None, 28, 16, 8),      # 8 online CPUs: how_many_cores caps p (CPU.c:200)
    (64, 8, 8, 8, 20, 16, 8),           # small N: the thread count decides
    (1024, 256, 256, 1, 20, 16, 1),
])
def test_reference_worker_count(monkeypatch, avail_gib, cpus, share, threads, log_n, esz, want):
    monkeypatch.setattr(bench, "_mem_available", lambda: avail_gib << 30)
    monkeypatch.setattr(bench, "_cgroup_mem_limit", lambda: None)
    monkeypatch.setattr(bench.os, "cpu_count", lambda: cpus)
    monkeypatch.setattr(bench, "_cpu_share", lambda: share)
    assert bench.ref_workers(log_n, esz, threads) == want
    # the reference's own rule (online CPUs only) for the line's "alternative"
    if threads is None and cpus >= 32 and avail_gib > 1000:
        assert bench.ref_workers(log_n, esz, share=False) == 32


def test_cpu_share_follows_the_cgroup_quota(monkeypatch):
    monkeypatch.setattr(bench.os, "cpu_count", lambda: 256)
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setattr(bench, "_cgroup_cpu_quota", lambda: 16.0)
    assert bench._cpu_share() == 16
    monkeypatch.setattr(bench, "_cgroup_cpu_quota", lambda: None)
    assert bench._cpu_share() == 256
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(12)))
    assert bench._cpu_share() == 12


def test_reference_worker_count_follows_cgroup_limit(monkeypatch):
    monkeypatch.setattr(bench, "_mem_available", lambda: 2900 << 30)
    monkeypatch.setattr(bench, "_cgroup_mem_limit", lambda: 110 << 30)  # 91 GiB budget: p = 16 touches 100
    monkeypatch.setattr(bench.os, "cpu_count", lambda: 256)
    monkeypatch.setattr(bench, "_cpu_share", lambda: 256)
    assert bench.ref_workers(28, 16) == 8


def test_reference_worker_count_refuses_oversize(monkeypatch):
    monkeypatch.setattr(bench, "_mem_available", lambda: 16 << 30)
    monkeypatch.setattr(bench, "_cgroup_mem_limit", lambda: None)
    with pytest.raises(RuntimeError, match="host memory"):
        bench.ref_workers(28, 16, 16)  # even P=1 touches 12 GiB > 4.8 GiB


def test_headline_cpu_baseline_runs_the_reference():
    """The cpu_baseline object a bench line carries (every N, rank 0): the
    reference binary built from its source, its own timer, the threads used
    and the host's CPU/memory description."""
    import pifft_oracle
    if pifft_oracle.reference_binary(64) is None:
        pytest.skip("oracle/_ref not built (make -C oracle ref)")
    rec = bench.headline_cpu_baseline(14, 64, threads=2)
    assert rec["kind"] == "reference" and rec["cores"] == 2 and rec["value"] > 0 and rec["unit"] == "GFLOP/s"
    for k in ("host_cpus", "physical_cores", "cpu_affinity", "mem_available_GiB", "host_bytes_touched",
              "child_peak_rss_GiB"):
        assert k in rec, k
    assert "p=2 pthreads" in rec["sample"]


def test_pg_is_a_process_group_option():
    """--pg opens a process group at one rank (bench.py's multi-GPU branch on
    one GPU); it cannot be combined with --as-rank, the single-process
    emulation of another rank's plan."""
    r = _run(["--pg", "--as-rank", "0/2"], {})
    assert r.returncode != 0 and "--as-rank" in r.stderr
    r = _run(["--pg", "--as-rank", "0/2"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "--as-rank" in r.stderr
