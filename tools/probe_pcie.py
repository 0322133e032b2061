#!/usr/bin/env python3
"""tools/probe_pcie.py -- where the host boundary's 300 ms go (fp64 2^28 =
4 GiB each way): host<->device copy rates from pageable and from pinned host
memory, and the host's own memcpy rate with 1..16 threads (a pinned bounce
buffer needs one).  A probe, not product."""
import concurrent.futures as cf
import time

import numpy as np
import torch

GiB = 1 << 30


def rate(fn, nbytes, reps=3):
    best = 1e9
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return nbytes / best / 1e9, best * 1e3


def main():
    nb = 4 * GiB
    host = np.ones(nb // 8, dtype=np.float64)           # pageable
    pinned = torch.empty(nb // 8, dtype=torch.float64).pin_memory()
    dev = torch.empty(nb // 8, dtype=torch.float64, device="cuda")
    th = torch.from_numpy(host)
    print("H2D pageable %.1f GB/s (%.0f ms)" % rate(lambda: dev.copy_(th), nb), flush=True)
    print("D2H pageable %.1f GB/s (%.0f ms)" % rate(lambda: th.copy_(dev), nb), flush=True)
    print("H2D pinned   %.1f GB/s (%.0f ms)" % rate(lambda: dev.copy_(pinned, non_blocking=True), nb), flush=True)
    print("D2H pinned   %.1f GB/s (%.0f ms)" % rate(lambda: pinned.copy_(dev, non_blocking=True), nb), flush=True)
    pin_np = pinned.numpy()
    for nt in (1, 4, 8, 16):
        chunks = np.array_split(np.arange(host.size), nt)
        bounds = [(c[0], c[-1] + 1) for c in chunks]

        def copy(b):
            pin_np[b[0]:b[1]] = host[b[0]:b[1]]

        with cf.ThreadPoolExecutor(nt) as ex:
            print(f"host memcpy pageable->pinned, {nt:2d} threads: %.1f GB/s (%.0f ms)" %
                  rate(lambda: list(ex.map(copy, bounds)), nb), flush=True)


if __name__ == "__main__":
    main()
