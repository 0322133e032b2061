"""pifft_dist.py -- the multi-GPU (one process per GPU) side of the pi-FFT.

The reference splits the transform over P workers that never exchange data
(CPU.c:336-360: P pinned pthreads, each writing its own output bins).  Here one
worker range lives on each GPU/rank:

  * worker_range(rank, world, P): rank r computes workers [r P/W, (r+1) P/W)
    (the reference's Pi, CPU.c:336) -- no collective on the data path;
  * batch_range(rank, world, B): for a batch of independent transforms
    (config 3) rank r runs transforms [r B/W, (r+1) B/W) whole instead;
  * the only optional exchange is the final all-gather of the slices
    (torch.distributed all_gather over RCCL/xGMI, or gloo on CPU) followed by
    the stride-P interleave (interleave_slices / pifft_interleave_device);
  * max_over_ranks: the job's time is the slowest rank's.
"""
from __future__ import annotations

import numpy as np


def worker_range(rank: int, world: int, workers: int) -> tuple[int, int]:
    if world < 1 or workers % world:
        raise ValueError(f"{workers} workers cannot be split over {world} ranks")
    per = workers // world
    return rank * per, per


def batch_range(rank: int, world: int, batch: int) -> tuple[int, int]:
    """Batched transforms (config 3) shard by transform: rank r runs transforms
    [r B/W, (r+1) B/W) whole, with its own P workers -- independent objects,
    no exchange.  The reference has no batch; a batch is its
    run() applied to each vector (CPU.c:312-380)."""
    if world < 1 or batch < 1 or batch % world:
        raise ValueError(f"a batch of {batch} transforms cannot be split over {world} ranks")
    per = batch // world
    return rank * per, per


def bitrev(x: int, bits: int) -> int:
    r = 0
    for _ in range(bits):
        r = (r << 1) | (x & 1)
        x >>= 1
    return r


def interleave_slices(slices: np.ndarray) -> np.ndarray:
    """(P, M) slice-major worker outputs -> natural order: out[bitrev(q) + P k] = slices[q, k]."""
    P, M = slices.shape
    bits = P.bit_length() - 1
    out = np.empty(P * M, dtype=slices.dtype)
    for q in range(P):
        out[bitrev(q, bits)::P] = slices[q]
    return out


def slice_of_natural(X: np.ndarray, P: int, q: int) -> np.ndarray:
    """Worker q's bins of a natural-order result: X[bitrev(q) + P k], k < N/P."""
    return X[bitrev(q, P.bit_length() - 1)::P]


def allgather_slices(local, group=None):
    """All-gather equal-size per-rank slice tensors (rank order) into one
    tensor.  RCCL: a single all_gather_into_tensor straight into the gathered
    buffer (no per-rank parts and no concatenation copy: at config 5 that is
    64 GiB per GPU saved), complex values moved as their real view."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    src = local.contiguous()
    shape = (world * src.shape[0],) + tuple(src.shape[1:]) if src.dim() else (world,)
    if dist.get_backend(group) == "nccl":
        flat = torch.view_as_real(src).reshape(-1) if src.is_complex() else src.reshape(-1)
        out = torch.empty(world * flat.numel(), dtype=flat.dtype, device=flat.device)
        dist.all_gather_into_tensor(out, flat, group=group)
        out = torch.view_as_complex(out.view(-1, 2)) if src.is_complex() else out
        return out.view(shape)  # the shape torch.cat of the per-rank parts has (the gloo path)
    staged = src.is_cuda  # gloo gathers host tensors
    if staged:
        src = src.cpu()
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    out = torch.cat(parts) if src.dim() else torch.stack(parts)
    return out.to(local.device) if staged else out


def slices_transform_major(gathered, world: int, batch: int):
    """A worker split's all-gathered result is rank-major -- (rank, transform,
    that rank's slices) -- while the stride-P interleave reads each transform's
    P slices back to back (transform, worker, bin).  Reorders the flat
    gathered buffer (a no-op view for one transform per rank)."""
    if batch == 1:
        return gathered.reshape(-1)
    return gathered.reshape(world, batch, -1).transpose(0, 1).contiguous().reshape(-1)


MASK64 = (1 << 64) - 1


def tensor_digest(t, chunk: int = 1 << 24) -> tuple[int, int]:
    """Two 64-bit digests of a tensor's BYTES (complex values as their integer
    words): a position-weighted sum and a mixed sum, both mod 2^64.  Integer
    sums are exact and order-independent, so equal bits give equal digests on
    any device (bench.py's cross-rank bitwise check of the worker slices)."""
    import torch
    v = torch.view_as_real(t).reshape(-1) if t.is_complex() else t.reshape(-1)
    v = v.view(torch.int64) if v.element_size() == 8 else v.view(torch.int32).to(torch.int64)
    dw = ds = 0
    for o in range(0, v.numel(), chunk):
        c = v[o:o + chunk]
        w = torch.arange(o, o + c.numel(), dtype=torch.int64, device=c.device) * -7046029254386353131 + 1
        dw += int((c * w).sum())
        ds += int((c ^ (c >> 29)).sum())
    return dw & MASK64, ds & MASK64


def dft_bins(x, ks):
    """Direct DFT bins X[k] = sum_n x[n] w^{nk} (w = e^{-2 pi i/N}) of a
    complex128 device vector of N = 2^L points, in float64 with exact integer
    phases mod N: n = a + 2^h b, X[k] = sum_a w^{ak} sum_b x[b, a] w^{2^h b k}
    -- one (K x 2^h) x (2^h x 2^(L-h)) GEMM over the resident input (no copy of
    it).  Independent of the FFT (bench.py's check of config 5, whose size the
    reference cannot express)."""
    import math
    import torch
    n = x.numel()
    logn = n.bit_length() - 1
    h = logn // 2
    A, B = 1 << h, n >> h
    k = torch.tensor(list(ks), dtype=torch.int64, device=x.device)[:, None]
    mask = n - 1
    b = torch.arange(B, dtype=torch.int64, device=x.device)[None, :]
    ang = (((b << h) * k) & mask).to(torch.float64) * (-2.0 * math.pi / n)
    wb = torch.polar(torch.ones_like(ang), ang)
    y = wb @ x.view(B, A)  # (K, A): sum_b x[b, a] w^{2^h b k}
    a = torch.arange(A, dtype=torch.int64, device=x.device)[None, :]
    ang = ((a * k) & mask).to(torch.float64) * (-2.0 * math.pi / n)
    wa = torch.polar(torch.ones_like(ang), ang)
    return (y * wa).sum(dim=1)


def sample_bins(n: int, workers: int, per_worker: int = 8) -> list[int]:
    """Natural-order bins to check directly: per_worker of each worker's bins
    bitrev(q) + P k (its first, second, middle and last k, and spread ones)."""
    m = n // workers
    bits = workers.bit_length() - 1
    ks = sorted({0, 1, m // 2, m - 1} | {(j * 0x9E3779B1 + 7) % m for j in range(max(0, per_worker - 4))})[:per_worker]
    return [bitrev(q, bits) + workers * k for q in range(workers) for k in ks]


def max_over_ranks(value: float, device=None) -> float:
    """The job's time: the largest value over the ranks (one all-reduce, on
    `device` -- the GPU under RCCL, the CPU under gloo).  A world-size-1 group
    runs the collective too (bench.py --pg: the RCCL path executed on one GPU)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
