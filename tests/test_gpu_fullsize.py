"""The headline configs at FULL size, on an MI355X through the C-ABI.

  * config 4 (fp64 N=2^28, one GPU): the whole natural-order spectrum of the
    1-worker plan, of the all-8-workers plan and of the 8-GPU split (eight
    one-worker plans on this GPU, gathered by pifft_allgather) against the
    oracle itself -- the C restatement of the reference (oracle/, bitwise-pinned
    to the reference's own outputs and, like the reference, bitwise invariant
    in P, so it runs as 16 workers on 16 host threads here);
  * config 5 (fp64 N=2^32, 8 GPUs): all eight workers of the split, run in
    turn on this one GPU into one slice-major union (64-bit indexing, fused
    tree), checked by Parseval over the union, 64 direct float64 DFT bins per
    worker, and after the device interleave (pifft_interleave_device) the same
    bins at their natural-order positions.  The reference cannot express N=2^32
    (uint32_t N, CPU.c:41,139), so properties are the pin there.

Bars (BASELINE.json north_star): rel-L2 <= 1e-12 (fp64); every bin within
1e-12 * rms(X) * 50 of its reference value (a misplaced bin is off by ~rms).
"""
import math
import os

import numpy as np
import pytest

import pifft
import pifft_dist
import pifft_oracle as oracle
from golden_io import rel_l2

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL64 = 1e-12


def _check_bins(got, want, tol=TOL64):
    err = rel_l2(got, want)
    assert err <= tol, f"rel-L2 {err:.3e} > {tol:.1e}"
    rms = np.linalg.norm(want) / math.sqrt(len(want))
    worst = float(np.max(np.abs(got - want)))
    assert worst <= 50 * tol * rms, f"max bin error {worst:.3e} > {50 * tol * rms:.3e}"
    return err


def _threads():
    return 16 if (os.cpu_count() or 1) >= 16 else max(1, os.cpu_count() or 1)


@pytest.mark.timeout(600)
def test_config4_full_size_vs_oracle():
    n, logn = 1 << 28, 28
    st = torch.cuda.current_stream()
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, stream=st)
    results = {}
    for P in (1, 8):
        plan = pifft.Plan(n, P, 1, pifft.F64)
        y = torch.empty_like(x)
        plan.execute_device(x.data_ptr(), y.data_ptr(), st)
        torch.cuda.synchronize()
        results[f"P={P}"] = y.cpu().numpy()
        plan.close()
        del y
    # the 8-GPU split, one GPU at a time: 8 one-worker plans + the device gather
    plans = [pifft.Plan(n, 8, 1, pifft.F64, first=q, count=1, device=0) for q in range(8)]
    assert all("tree+pass" in p.describe()["launch_kind"] for p in plans)  # the fused tree
    slices = [torch.empty(n // 8, dtype=torch.complex128, device="cuda") for _ in range(8)]
    for p, s in zip(plans, slices):
        p.execute_device(x.data_ptr(), s.data_ptr(), st)
    torch.cuda.synchronize()
    nat = torch.empty_like(x)
    pifft.allgather(plans, [s.data_ptr() for s in slices], [nat.data_ptr()] + [None] * 7)
    results["split 8"] = nat.cpu().numpy()
    for p in plans:
        p.close()
    del slices, nat
    xh = x.cpu().numpy()
    assert xh.tobytes()[:1 << 20] == oracle.generate(n, np.complex128, count=1 << 16).tobytes()
    del x
    torch.cuda.empty_cache()
    want = oracle.fft(xh, P=16, nthreads=_threads())
    for key, got in results.items():
        _check_bins(got, want)


def _dft_bins_gemm(x, ks):
    """Direct DFT bins X[k] = sum_n x[n] w^{nk} of a 2^(2h)-point vector in
    float64 on the GPU, n = a + 2^h b: X[k] = sum_a w^{ak} sum_b x[b, a]
    w^{2^h b k} -- one (K x 2^h) x (2^h x 2^h) complex128 GEMM over the
    resident input (no copy of it), with exact integer phases mod N."""
    n = x.numel()
    logn = n.bit_length() - 1
    h = logn // 2
    A, B = 1 << h, n >> h
    k = torch.tensor(ks, dtype=torch.int64, device=x.device)[:, None]
    mask = n - 1
    b = torch.arange(B, dtype=torch.int64, device=x.device)[None, :]
    ang = (((b << h) * k) & mask).to(torch.float64) * (-2.0 * math.pi / n)
    wb = torch.polar(torch.ones_like(ang), ang)
    y = wb @ x.view(B, A)  # (K, A): sum_b x[b, a] w^{2^h b k}
    a = torch.arange(A, dtype=torch.int64, device=x.device)[None, :]
    ang = ((a * k) & mask).to(torch.float64) * (-2.0 * math.pi / n)
    wa = torch.polar(torch.ones_like(ang), ang)
    return (y * wa).sum(dim=1).cpu().numpy()


def test_dft_bins_gemm_matches_fft():
    n = 1 << 20
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, stream=torch.cuda.current_stream())
    ks = [0, 1, 5, 777, n // 2, n - 1]
    want = np.fft.fft(x.cpu().numpy())[ks]
    got = _dft_bins_gemm(x, ks)
    assert np.max(np.abs(got - want)) <= 1e-12 * np.linalg.norm(want)


@pytest.mark.timeout(600)
def test_config5_all_workers_n2e32():
    free, _ = torch.cuda.mem_get_info()
    assert free >= 150 * (1 << 30), f"config 5 needs ~150 GiB of HBM, {free / 2**30:.0f} GiB free"
    n, P = 1 << 32, 8
    M = n // P
    st = torch.cuda.current_stream()
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, stream=st)
    union = torch.empty(n, dtype=torch.complex128, device="cuda")  # slice-major: worker q at [q M, (q+1) M)
    for q in range(P):
        plan = pifft.Plan(n, P, 1, pifft.F64, first=q, count=1, device=0)
        d = plan.describe()
        assert d["local_n"] == M and "tree+pass" in d["launch_kind"]
        plan.execute_device(x.data_ptr(), union[q * M:(q + 1) * M].data_ptr(), st)
        torch.cuda.synchronize()
        plan.close()
    torch.cuda.empty_cache()
    xn2 = torch.linalg.vector_norm(x).item() ** 2
    # Parseval over the union of the 8 workers' bins: sum |X|^2 = N ||x||^2
    un2 = torch.linalg.vector_norm(union).item() ** 2
    assert abs(un2 / n - xn2) <= 1e-12 * xn2 * 100, (un2 / n, xn2)
    # 64 direct DFT bins per worker, at X[bitrev(q) + 8 k]
    rng = np.random.default_rng(32)
    kk = np.unique(np.concatenate([[0, 1, M - 1], rng.integers(0, M, 61)]))
    bins, got = [], []
    for q in range(P):
        r = pifft_dist.bitrev(q, 3)
        bins += [int(r + P * k) for k in kk]
        got.append(union[q * M + torch.as_tensor(kk, device="cuda")].cpu().numpy())
    got = np.concatenate(got)
    want = _dft_bins_gemm(x, bins)
    scale = math.sqrt(xn2)  # |X[k]| ~ ||x||
    assert np.max(np.abs(got - want)) <= 1e-12 * scale * 50, np.max(np.abs(got - want)) / scale
    del x
    torch.cuda.empty_cache()
    # the gathered layout into natural order on the device: the same bins at
    # their natural positions, bit for bit
    natural = torch.empty_like(union)
    pifft.interleave_device(union.data_ptr(), natural.data_ptr(), n, P, 1, pifft.F64, st)
    torch.cuda.synchronize()
    nat_bins = natural[torch.as_tensor(bins, device="cuda")].cpu().numpy()
    assert nat_bins.tobytes() == got.tobytes()
    nn2 = torch.linalg.vector_norm(natural).item() ** 2
    assert nn2 == pytest.approx(un2, rel=1e-13)


@pytest.mark.timeout(600)
def test_config4_fp32_full_size_vs_oracle():
    """The reference's own precision (data_t = float, CPU.c:33-36) at N = 2^28:
    the default fp32 plan (three packed 32-value passes 512 x 512 x 1024) and
    the 8-worker plan against the oracle (fp32 restatement, 16 workers).
    Bar: rel-L2 <= 1e-5 log2 N."""
    n, logn = 1 << 28, 28
    st = torch.cuda.current_stream()
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F32, stream=st)
    got = {}
    for P in (1, 8):
        plan = pifft.Plan(n, P, 1, pifft.F32)
        if P == 1:
            assert plan.describe()["vpt"] == [32, 32, 32]
        y = torch.empty_like(x)
        plan.execute_device(x.data_ptr(), y.data_ptr(), st)
        torch.cuda.synchronize()
        got[P] = y.cpu().numpy()
        plan.close()
        del y
    xh = x.cpu().numpy()
    del x
    torch.cuda.empty_cache()
    want = oracle.fft(xh, P=16, nthreads=_threads())
    for P, g in got.items():
        _check_bins(g, want, tol=1e-5 * logn)


@pytest.mark.timeout(600)
def test_reference_max_size_n2e30_fp64():
    """N = 2^30, the largest size the reference can express (uint32_t N and
    atoi, CPU.c:41,139): the 1-worker and 8-worker plans agree bin for bin,
    FFT(conj(FFT(x))) = N conj(x), Parseval, and 16 direct DFT bins."""
    free, _ = torch.cuda.mem_get_info()
    assert free >= 80 * (1 << 30), f"needs ~80 GiB of HBM, {free / 2**30:.0f} GiB free"
    n = 1 << 30
    st = torch.cuda.current_stream()
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, stream=st)
    X = torch.empty_like(x)
    p1 = pifft.Plan(n, 1, 1, pifft.F64)
    p1.execute_device(x.data_ptr(), X.data_ptr(), st)
    Y = torch.empty_like(x)
    p8 = pifft.Plan(n, 8, 1, pifft.F64)
    p8.execute_device(x.data_ptr(), Y.data_ptr(), st)
    torch.cuda.synchronize()
    p8.close()
    err = (torch.linalg.vector_norm(Y - X) / torch.linalg.vector_norm(X)).item()
    assert err <= TOL64, err
    xn = torch.linalg.vector_norm(x).item()
    assert abs(torch.linalg.vector_norm(X).item() ** 2 / n - xn ** 2) <= 1e-12 * xn ** 2
    ks = [0, 1, 3, 12345, n // 2, n // 2 + 7, n - 1] + [int(k) for k in np.random.default_rng(30).integers(0, n, 9)]
    want = _dft_bins_gemm(x, ks)
    got = X[torch.as_tensor(ks, device="cuda")].cpu().numpy()
    assert np.max(np.abs(got - want)) <= 1e-12 * xn * 50
    # double transform
    Xc = X.conj().resolve_conj()
    del Y
    Z = torch.empty_like(x)
    p1.execute_device(Xc.data_ptr(), Z.data_ptr(), st)
    torch.cuda.synchronize()
    err2 = (torch.linalg.vector_norm(Z.conj() / n - x) / xn).item()
    assert err2 <= TOL64, err2


ORDERS = {"0": [1024, 512, 512], "1": [512, 512, 1024]}  # PIFFT_POS_MODEL: the radix order at 2^28


@pytest.mark.parametrize("pos", ["0", "1"])
def test_packed_vpt32_fp32_three_pass_bitwise(pos, monkeypatch):
    """fp32 2^28 in three passes on the 16384-value tile: the packed VPT-32
    passes (512 threads, two butterflies per register pair, PIFFT_VPT32=1)
    equal the 16-values-per-thread passes (1024 threads) bit for bit -- the
    same radices, twiddles and operation order. (The packed plan is fp32
    2^28's default, so test_config4_fp32_full_size_vs_oracle checks it
    against the oracle.)  Both radix orders."""
    n = 1 << 28
    monkeypatch.setenv("PIFFT_POS_MODEL", pos)
    st = torch.cuda.current_stream()
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F32, seed=33, stream=st)
    monkeypatch.setenv("PIFFT_TILE32", "16384")
    monkeypatch.setenv("PIFFT_PASSES", "3")
    monkeypatch.setenv("PIFFT_VPT32", "0")
    v16 = pifft.Plan(n, 1, 1, pifft.F32)
    monkeypatch.setenv("PIFFT_VPT32", "1")
    v32 = pifft.Plan(n, 1, 1, pifft.F32)
    assert v16.describe()["radix"] == v32.describe()["radix"] == ORDERS[pos]
    assert v16.describe()["vpt"] == [16, 16, 16] and v32.describe()["vpt"] == [32, 32, 32]
    ya = torch.empty_like(x)
    v16.execute_device(x.data_ptr(), ya.data_ptr(), st)
    v16.close()
    yb = torch.empty_like(x)
    v32.execute_device(x.data_ptr(), yb.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(torch.view_as_real(ya), torch.view_as_real(yb))


# shapes whose radix order the position-aware planner changed (round 3,
# profiles/r03_pos_model_shapes.log): (log2 N, precision, workers)
POS_SHAPES = [(25, pifft.F32, 1), (26, pifft.F32, 1), (25, pifft.F64, 64), (29, pifft.F64, 1)]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("logn,prec,P", POS_SHAPES)
def test_position_model_orders_vs_oracle(logn, prec, P, monkeypatch):
    """Every plan shape whose radix order the position model changed, in both
    orders (PIFFT_POS_MODEL 1 / 0): the orders differ, and each result matches
    the oracle (2^25-2^26) or, at 2^29, the other order's result, per bin.
    Bars: rel-L2 <= 1e-12 fp64, <= 1e-5 log2 N fp32."""
    n = 1 << logn
    f64 = prec == pifft.F64
    cdt = torch.complex128 if f64 else torch.complex64
    tol = TOL64 if f64 else 1e-5 * logn
    st = torch.cuda.current_stream()
    x = torch.empty(n, dtype=cdt, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, prec, seed=91, stream=st)
    got, radix = {}, {}
    for pos in ("1", "0"):
        monkeypatch.setenv("PIFFT_POS_MODEL", pos)
        plan = pifft.Plan(n, P, 1, prec)
        radix[pos] = plan.describe()["radix"]
        y = torch.empty_like(x)
        plan.execute_device(x.data_ptr(), y.data_ptr(), st)
        torch.cuda.synchronize()
        got[pos] = y.cpu().numpy()
        plan.close()
        del y
    assert radix["1"] != radix["0"], radix
    if logn <= 26:
        want = oracle.fft(x.cpu().numpy(), P=16, nthreads=_threads())
        for g in got.values():
            _check_bins(g, want, tol=tol)
    else:
        _check_bins(got["1"], got["0"], tol=tol)
