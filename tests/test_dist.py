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
