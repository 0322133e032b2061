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


@pytest.mark.parametrize("avail_gib,threads,log_n,esz,want", [
    (1024, 16, 28, 16, 16),   # (2 + 32) * 4 GiB = 136 GiB <= the 160 GiB cap
    (1024, 64, 28, 16, 16),   # 32 workers would need 264 GiB: capped
    (100, 16, 28, 16, 4),     # 70 GiB budget: (2 + 8) * 4 = 40 GiB fits, P=8 needs 72
    (64, 8, 20, 16, 8),       # small N: the thread count decides
    (1024, 1, 20, 16, 1),
])
def test_reference_worker_count_fits_memory(monkeypatch, avail_gib, threads, log_n, esz, want):
    monkeypatch.setattr(bench, "_mem_available", lambda: avail_gib << 30)
    assert bench.ref_workers(log_n, esz, threads) == want


def test_reference_worker_count_refuses_oversize(monkeypatch):
    monkeypatch.setattr(bench, "_mem_available", lambda: 16 << 30)
    with pytest.raises(RuntimeError, match="host memory"):
        bench.ref_workers(28, 16, 16)  # even P=1 needs 16 GiB
