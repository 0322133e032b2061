"""Seeded random plan shapes vs the oracle, through the C-ABI on an MI355X.

The other GPU tests walk the planner's paths one by one; this sweep draws 48
(N, P, worker range, batch, precision, output order) combinations from a
fixed seed -- so the cases are the same on every run -- and checks each
plan's output against the oracle (oracle/pifft_oracle.c, bitwise-pinned to the
reference's CPU.c): natural order, slice-major worker ranges (worker q's
bins X[bitrev(q) + P k], CPU.c:496-499) and the reference's bit-reversed
scratch order (tmp_in, CPU.c:463-478).  Tolerances as in test_gpu_parity.py
(north star: rel-L2 1e-12 fp64, 1e-5 log2 N fp32, every bin against the
typical bin magnitude).  Sizes stay within a few seconds of oracle time.
"""
import os
import random

import numpy as np
import pytest

import pifft
import pifft_dist
import pifft_oracle as oracle
from test_gpu_parity import DT, PREC, _bitrev_perm, assert_bins_close, dev

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _cases(count=int(os.environ.get("FUZZ_COUNT", "48")), seed=int(os.environ.get("FUZZ_SEED", "20261017"))):
    # (FUZZ_COUNT / FUZZ_SEED: a longer sweep on demand, e.g. profiles/r04zb_fuzz_seed4242.txt)
    rng = random.Random(seed)
    out = []
    while len(out) < count:
        suf = rng.choice(["f32", "f64"])
        logn = rng.randint(1, 21)
        n = 1 << logn
        P = 1 << rng.randint(0, min(logn, 10))
        if P >= 64 and logn > 16:  # the oracle's tree is Theta(N) per worker
            continue
        batch = rng.choice([1, 1, 1, 2, 3, 5])
        if n * batch > 1 << 21:
            batch = 1
        flags = rng.choice([pifft.OUT_NATURAL, pifft.OUT_SLICES, pifft.OUT_BITREV])
        if flags == pifft.OUT_NATURAL:
            first, cnt = 0, P
        else:
            cnt = 1 << rng.randint(0, P.bit_length() - 1)
            first = cnt * rng.randrange(P // cnt)
        out.append((suf, logn, P, first, cnt, batch, flags))
    return out


@pytest.mark.parametrize("suf,logn,P,first,count,batch,flags", _cases())
def test_random_plan_vs_oracle(suf, logn, P, first, count, batch, flags):
    n = 1 << logn
    m = n // P
    xs = [oracle.generate(n, DT[suf], seed=logn * 131 + P * 7 + b) for b in range(batch)]
    plan = pifft.Plan(n, P, batch, PREC[suf], first=first, count=count, device=0, flags=flags)
    d_in = dev(np.concatenate(xs))
    d_out = torch.empty(plan.info.out_elems, dtype=d_in.dtype, device="cuda")
    plan.execute_device(d_in.data_ptr(), d_out.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    per = got.size // batch
    for b in sorted({0, batch - 1}):
        X = oracle.fft(xs[b], P=P, nthreads=16)
        g = got[b * per:(b + 1) * per]
        if flags == pifft.OUT_NATURAL:
            assert_bins_close(g, X, suf, n)
        elif flags == pifft.OUT_SLICES:
            for j in range(count):
                assert_bins_close(g[j * m:(j + 1) * m], pifft_dist.slice_of_natural(X, P, first + j), suf, n)
        else:  # the reference's tmp_in segments of these workers
            want = X[_bitrev_perm(n)][first * m:(first + count) * m]
            assert_bins_close(g, want, suf, n)


@pytest.mark.parametrize("suf,logn,P,first,count,batch,flags", _cases(count=24, seed=1017))
def test_random_plan_padded_workspace_bitwise(suf, logn, P, first, count, batch, flags, monkeypatch):
    """The same random shapes with padded workspace rows forced on
    (PIFFT_W_PAD_MIN_MIB=0, an odd pad): bitwise equal to the unpadded plan."""
    n = 1 << logn
    x = np.concatenate([oracle.generate(n, DT[suf], seed=logn * 17 + b) for b in range(batch)])
    outs = []
    for pad in ("0", "37"):
        monkeypatch.setenv("PIFFT_W_PAD_MIN_MIB", "0")
        monkeypatch.setenv("PIFFT_W_PAD", pad)
        plan = pifft.Plan(n, P, batch, PREC[suf], first=first, count=count, device=0, flags=flags)
        d_in = dev(x)
        d_out = torch.empty(plan.info.out_elems, dtype=d_in.dtype, device="cuda")
        plan.execute_device(d_in.data_ptr(), d_out.data_ptr(), torch.cuda.current_stream())
        torch.cuda.synchronize()
        outs.append(d_out.cpu().numpy().tobytes())
    assert outs[0] == outs[1]


def _large_cases(count=int(os.environ.get("FUZZ_LARGE_COUNT", "8")), seed=int(os.environ.get("FUZZ_LARGE_SEED", "4242"))):
    rng = random.Random(seed)
    out = []
    for _ in range(count):
        suf = rng.choice(["f32", "f64"])
        logn = rng.randint(22, 24)
        P = 1 << rng.randint(0, 4)
        flags = rng.choice([pifft.OUT_NATURAL, pifft.OUT_SLICES, pifft.OUT_BITREV])
        cnt = P if flags == pifft.OUT_NATURAL else 1 << rng.randint(0, P.bit_length() - 1)
        first = 0 if flags == pifft.OUT_NATURAL else cnt * rng.randrange(P // cnt)
        out.append((suf, logn, P, first, cnt, 1, flags))
    return out


@pytest.mark.parametrize("suf,logn,P,first,count,batch,flags", _large_cases())
def test_random_large_plan_vs_oracle(suf, logn, P, first, count, batch, flags):
    """Seeded random multi-pass shapes at N = 2^22..2^24 (three-pass local
    FFTs, the natural-store and interleave rules, fused trees), vs the oracle
    on 16 host threads."""
    test_random_plan_vs_oracle(suf, logn, P, first, count, batch, flags)


def _wil_cases(count=int(os.environ.get("FUZZ_WIL_COUNT", "16")), seed=int(os.environ.get("FUZZ_WIL_SEED", "20261018"))):
    """Natural-order all-worker shapes with P <= 16 and a multi-pass local FFT
    (M = N/P >= 2^15): the worker-interleaved layout's domain."""
    rng = random.Random(seed)
    out = []
    while len(out) < count:
        suf = rng.choice(["f32", "f64"])
        lp = rng.randint(1, 4)
        logn = rng.randint(15 + lp, 22)
        batch = rng.choice([1, 1, 2, 3])
        if (1 << logn) * batch > 1 << 22:
            batch = 1
        out.append((suf, logn, 1 << lp, batch))
    return out


@pytest.mark.parametrize("suf,logn,P,batch", _wil_cases())
def test_random_worker_interleaved_plan_vs_oracle(suf, logn, P, batch):
    """Seeded random shapes on the worker-interleaved layout (tree writing
    z_q[i] at i P + q, MODE 10 passes, natural-order last pass) vs the oracle."""
    n = 1 << logn
    xs = [oracle.generate(n, DT[suf], seed=logn * 17 + P + b) for b in range(batch)]
    plan = pifft.Plan(n, P, batch, PREC[suf])
    assert plan.describe()["worker_interleaved"], plan.describe()
    d_in = dev(np.concatenate(xs))
    d_out = torch.empty(plan.info.out_elems, dtype=d_in.dtype, device="cuda")
    plan.execute_device(d_in.data_ptr(), d_out.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().reshape(batch, n)
    for b in range(batch):
        assert_bins_close(got[b], oracle.fft(xs[b], P=1, nthreads=8), suf, n)
