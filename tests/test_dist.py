"""The N>1 path on CPU: world_size-2 gloo ranks, each owning a worker range of
the pi split (no data-path collective), then the optional all-gather + stride-P
interleave.  The per-worker compute here is the oracle (the GPU leg is
covered by test_gpu_parity.py's single-worker plans); what is under test is
the sharding, gather and reorder logic bench.py uses (pifft_dist)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, n, P, q_out, batch=1):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "oracle"), os.path.join(root, "cs87project-msolano2_amd")):
        sys.path.insert(0, p)
    import pifft_dist
    import pifft_oracle as oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        xs = oracle.generate(n, np.complex128, count=batch * n).reshape(batch, n)
        first, count = pifft_dist.worker_range(rank, world, P)
        # this rank's result as a slice-major plan writes it: (transform, its workers, bins)
        mine = np.stack([np.stack([pifft_dist.slice_of_natural(oracle.worker_bins(xs[b], P, q), P, q)
                                   for q in range(first, first + count)]) for b in range(batch)])
        local = torch.from_numpy(mine.reshape(-1).view(np.float64).copy())
        gathered = pifft_dist.allgather_slices(local)
        gathered = pifft_dist.slices_transform_major(gathered, world, batch).numpy().view(np.complex128)
        natural = np.stack([pifft_dist.interleave_slices(s.reshape(P, n // P))
                            for s in gathered.reshape(batch, n)])
        t = pifft_dist.max_over_ranks(float(rank + 1))
        if rank == 0:
            want = np.stack([oracle.fft(xs[b], P=1) for b in range(batch)])
            q_out.put((natural.tobytes() == want.tobytes(), t))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,P,batch", [(4096, 4, 1), (1 << 14, 8, 1), (256, 2, 1), (1024, 4, 3), (512, 2, 2)])
def test_two_rank_split_gather_equals_transform(n, P, batch):
    """batch > 1: the gathered buffer is rank-major and is reordered to the
    transform-major slice layout before the interleave (bench.py allgather)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, n, P, q, batch)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    ok, tmax = q.get()
    assert ok, "gathered + interleaved slices differ from the oracle transform"
    assert tmax == 2.0


def test_worker_range():
    import pifft_dist
    assert [pifft_dist.worker_range(r, 4, 8) for r in range(4)] == [(0, 2), (2, 2), (4, 2), (6, 2)]
    assert pifft_dist.worker_range(0, 1, 8) == (0, 8)
    with pytest.raises(ValueError):
        pifft_dist.worker_range(0, 3, 8)


def test_interleave_matches_reference_ownership():
    import pifft_dist
    import pifft_oracle as oracle
    n, P = 512, 8
    x = oracle.generate(n, np.complex64)
    X = oracle.fft(x)
    sl = np.stack([pifft_dist.slice_of_natural(X, P, q) for q in range(P)])
    assert pifft_dist.interleave_slices(sl).tobytes() == X.tobytes()


def _batch_rank_main(rank, world, port, n, batch, q_out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    for p in (os.path.join(root, "oracle"), os.path.join(root, "cs87project-msolano2_amd")):
        sys.path.insert(0, p)
    import pifft_dist
    import pifft_oracle as oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        first, count = pifft_dist.batch_range(rank, world, batch)
        # this rank's transforms of the global batch, exactly as bench.py --shard batch generates them
        x = oracle.generate(n, np.complex64, count=count * n, first=first * n).reshape(count, n)
        mine = np.stack([oracle.fft(x[b]) for b in range(count)])
        local = torch.from_numpy(mine.reshape(-1).view(np.float32).copy())
        gathered = pifft_dist.allgather_slices(local).numpy().view(np.complex64).reshape(batch, n)
        if rank == 0:
            xa = oracle.generate(n, np.complex64, count=batch * n).reshape(batch, n)
            want = np.stack([oracle.fft(xa[b]) for b in range(batch)])
            q_out.put(gathered.tobytes() == want.tobytes())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n,batch", [(4096, 8), (256, 6)])
def test_two_rank_batch_shard_gather_equals_batch(n, batch):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_batch_rank_main, args=(r, world, port, n, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get(), "gathered batch shards differ from the per-transform oracle"


def test_batch_range():
    import pifft_dist
    assert [pifft_dist.batch_range(r, 8, 4096) for r in (0, 7)] == [(0, 512), (3584, 512)]
    assert pifft_dist.batch_range(0, 1, 5) == (0, 5)
    with pytest.raises(ValueError):
        pifft_dist.batch_range(0, 3, 4096)
    with pytest.raises(ValueError):
        pifft_dist.batch_range(0, 2, 0)


# ------------------------------------------------ multi-GPU self-verification ---
def _digest_rank_main(rank, world, port, q_out):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "cs87project-msolano2_amd"))
    import pifft_dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(5)
        t = torch.randn(3000, dtype=torch.complex128, generator=g)
        if rank == 1:
            t = t.clone()
        digests = [None] * world
        dist.all_gather_object(digests, pifft_dist.tensor_digest(t, chunk=512))
        if rank == 0:
            q_out.put(all(tuple(d) == pifft_dist.tensor_digest(t) for d in digests))
    finally:
        dist.destroy_process_group()


def test_two_rank_slice_digests_agree():
    """bench.py's slices_bitwise check: each rank's integer digest, gathered
    with all_gather_object (gloo), equals rank 0's for the same bits, and the
    digest does not depend on the chunking."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_digest_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    assert q.get()


def test_tensor_digest_sees_every_bit():
    import pifft_dist
    x = torch.randn(1 << 12, dtype=torch.complex128)
    d0 = pifft_dist.tensor_digest(x)
    assert pifft_dist.tensor_digest(x.clone(), chunk=100) == d0
    for pos in (0, 777, (1 << 12) - 1):
        y = torch.view_as_real(x.clone()).reshape(-1).view(torch.int64)
        y[2 * pos + 1] ^= 1  # the lowest mantissa bit of one imaginary part
        assert pifft_dist.tensor_digest(torch.view_as_complex(y.view(torch.float64).view(-1, 2))) != d0
    a = x.clone()
    a[[3, 4]] = a[[4, 3]]  # two values swapped: same multiset, different positions
    assert pifft_dist.tensor_digest(a) != d0
    f = torch.randn(1000, dtype=torch.complex64)
    assert pifft_dist.tensor_digest(f) == pifft_dist.tensor_digest(f.clone())


def test_direct_bins_match_fft_and_sample_ownership():
    import pifft_dist
    n, P = 1 << 12, 8
    x = torch.randn(n, dtype=torch.complex128)
    ks = pifft_dist.sample_bins(n, P)
    assert len(ks) == 8 * P and len(set(ks)) == len(ks)
    # each worker's bins are its own residue class bitrev(q) + P k
    for q in range(P):
        r = pifft_dist.bitrev(q, 3)
        assert all(k % P == r for k in ks[8 * q:8 * (q + 1)])
    want = np.fft.fft(x.numpy())[ks]
    got = pifft_dist.dft_bins(x, ks).numpy()
    assert np.max(np.abs(got - want)) <= 1e-12 * np.linalg.norm(want)


def test_verify_finish_accepts_and_rejects():
    """bench.py verify_finish (rank 0): rel-L2 against the one-GPU reference,
    direct bins against a misplaced bin, and the slice check's verdict."""
    import bench
    import pifft_dist
    n, P = 1 << 12, 4
    x = torch.randn(n, dtype=torch.complex128) / 64
    X = torch.fft.fft(x)
    ks = pifft_dist.sample_bins(n, P)
    good = {"slices_bitwise": True, "slices_checked": P, "slices_differing": [], "tol": 1e-12,
            "reference": "test", "ref": X.clone()}
    v = bench.verify_finish(torch, good, X * (1 + 1e-15))
    assert v["ok"] and v["rel_l2"] <= 1e-12 and v["bins_ok"] is None
    bad = X.clone()
    bad[[5, 9]] = bad[[9, 5]]  # two bins swapped: a permutation fault
    assert not bench.verify_finish(torch, good, bad)["ok"]
    assert not bench.verify_finish(torch, dict(good, slices_bitwise=False), X)["ok"]
    binsprep = {"slices_bitwise": True, "tol": 1e-12, "ks": ks, "bins": pifft_dist.dft_bins(x, ks),
                "x_norm": float(torch.linalg.vector_norm(x)), "reference": "bins"}
    v = bench.verify_finish(torch, binsprep, X)
    assert v["ok"] and v["bins_ok"] and v["bins"] == len(ks) and v["rel_l2"] is None
    moved = X.clone()
    moved[ks[3]] = X[ks[3] + P]  # a neighbouring bin of the same worker in its place
    assert not bench.verify_finish(torch, binsprep, moved)["bins_ok"]
    v = bench.verify_finish(torch, good, None)
    assert v["ok"] and v["rel_l2"] is None and "slices only" in v["note"]
    assert bench.verify_finish(torch, {}, X) is None  # ranks other than 0


def test_one_rank_group_runs_the_collectives(monkeypatch):
    """A world-size-1 group (bench.py --pg) executes pifft_dist's collectives
    instead of short-cutting them: max_over_ranks all-reduces, and
    allgather_slices returns the rank's own bytes (gloo here; the RCCL leg is
    tests/test_bench.py::test_pifft_dist_under_a_one_rank_rccl_group)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "cs87project-msolano2_amd"))
    import pifft_dist
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        calls = []
        orig = dist.all_reduce
        monkeypatch.setattr(dist, "all_reduce", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
        assert pifft_dist.max_over_ranks(1.25) == 1.25 and calls == [1]
        g = torch.Generator().manual_seed(3)
        x = torch.randn(2, 512, dtype=torch.complex128, generator=g)
        y = pifft_dist.allgather_slices(x)
        assert y.shape == x.shape and torch.equal(torch.view_as_real(y), torch.view_as_real(x))
    finally:
        dist.destroy_process_group()
