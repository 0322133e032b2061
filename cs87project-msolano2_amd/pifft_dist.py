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


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
