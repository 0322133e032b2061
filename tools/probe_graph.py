#!/usr/bin/env python3
"""tools/probe_graph.py -- do hipGraphs help the launch-bound configs?

For C1 (fp64 2^20, P=1), C2 (fp64 2^20, P=8, natural), C2 slice (worker 0 of
8) and C3 (fp32 4096 x 4096) plus the 512-transform C3 share, time:
  direct : K back-to-back pifft_execute_device calls on one stream
  graph1 : one step captured in a hipGraph (torch.cuda.CUDAGraph), replayed K times
  graphK : G steps captured in one graph, replayed K/G times
and check the graph's output is bitwise the direct one.  A probe, not product.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))

import torch  # noqa: E402

import pifft  # noqa: E402

K = 400
G = 20


def timed(fn, reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0)


def case(name, log_n, prec, P, count, batch):
    n = 1 << log_n
    cdt = torch.complex128 if prec == pifft.F64 else torch.complex64
    flags = pifft.OUT_NATURAL if count == P else pifft.OUT_SLICES
    plan = pifft.Plan(n, P, batch, prec, first=0, count=count, device=0, flags=flags)
    d = plan.describe()
    x = torch.empty(n * batch, dtype=cdt, device="cuda")
    pifft.generate_device(x.data_ptr(), n * batch, n, prec, seed=7, first=0, stream=torch.cuda.current_stream())
    y = torch.empty(d["out_elems"], dtype=cdt, device="cuda")
    s = torch.cuda.current_stream()

    def step():
        plan.execute_device(x.data_ptr(), y.data_ptr(), s)

    for _ in range(20):
        step()
    t_direct = min(timed(step, K) for _ in range(3)) / K
    ref = y.clone()
    y.zero_()

    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        plan.execute_device(x.data_ptr(), y.data_ptr(), torch.cuda.current_stream())
    g1.replay()
    torch.cuda.synchronize()
    same = bool(torch.equal(torch.view_as_real(y), torch.view_as_real(ref)))
    for _ in range(20):
        g1.replay()
    t_g1 = min(timed(g1.replay, K) for _ in range(3)) / K

    gk = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gk):
        for _ in range(G):
            plan.execute_device(x.data_ptr(), y.data_ptr(), torch.cuda.current_stream())
    for _ in range(3):
        gk.replay()
    t_gk = min(timed(gk.replay, K // G) for _ in range(3)) / (K // G * G)
    print(f"{name:10s} launches {d['num_launches']}  direct {t_direct * 1e6:7.2f} us  graph1 {t_g1 * 1e6:7.2f} us"
          f"  graph{G} {t_gk * 1e6:7.2f} us  bitwise {same}", flush=True)
    plan.close()


def main():
    torch.cuda.set_device(0)
    case("C1", 20, pifft.F64, 1, 1, 1)
    case("C2", 20, pifft.F64, 8, 8, 1)
    case("C2_slice", 20, pifft.F64, 8, 1, 1)
    case("C3", 12, pifft.F32, 1, 1, 4096)
    case("C3_share", 12, pifft.F32, 1, 1, 512)
    case("2^16f64", 16, pifft.F64, 1, 1, 1)


if __name__ == "__main__":
    main()
