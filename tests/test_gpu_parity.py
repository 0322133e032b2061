"""HIP path vs the reference, through the C-ABI (libpifft.so) on an MI355X.

Oracle: the reference's own outputs (tests/golden/, bitwise-pinned) and the C
restatement (oracle/) on the same seeded inputs.  Bars (BASELINE.json
north_star): relative L2 error <= 1e-12 (fp64) and <= 1e-5*log2(N) (fp32);
index permutation exact (every bin within 50 x the tolerance of the typical
bin magnitude of its own reference value, as well as in L2); the tree stage
and the input generator bit-exact.  Sizes beyond the oracle's reach are checked
through size-independent properties (double-transform identity, Parseval,
linearity, direct DFT bins, P-split consistency).
"""
import hashlib
import math
import os

import numpy as np
import pytest

import pifft
import pifft_dist
import pifft_oracle as oracle
from golden_io import load_fft, load_tree, manifest, rel_l2

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DT = {"f32": np.complex64, "f64": np.complex128}
PREC = {"f32": pifft.F32, "f64": pifft.F64}
TDT = {np.complex64: torch.complex64, np.complex128: torch.complex128}


def tol(suf, n):
    return 1e-12 if suf == "f64" else 1e-5 * math.log2(n)


def dev(x):
    return torch.from_numpy(np.ascontiguousarray(x)).to("cuda")


def run(plan, x, slices=False):
    """Execute a plan on a host array through device buffers; returns host result."""
    d_in = dev(x)
    info = plan.info
    d_out = torch.empty(info.out_elems, dtype=d_in.dtype, device="cuda")
    plan.execute_device(d_in.data_ptr(), d_out.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    return d_out.cpu().numpy()


def assert_bins_close(got, want, suf, n):
    err = rel_l2(got, want)
    assert err <= tol(suf, n), f"rel-L2 {err:.3e} > {tol(suf, n):.1e}"
    # permutation, per bin: every bin within 50 tol of the TYPICAL bin
    # magnitude rms(X) = ||X|| / sqrt(N) of its own reference value (a
    # misplaced bin is off by ~rms; at fp32 2^26 the bound is 1.3 % of rms)
    rms = np.linalg.norm(want) / math.sqrt(len(want))
    worst = float(np.max(np.abs(got - want)))
    assert worst <= max(50 * tol(suf, n), 1e-9) * rms, f"bin error {worst:.3e} vs rms {rms:.3e}"


def test_device_visible():
    assert torch.cuda.is_available()
    assert pifft.gpu_count() >= 1


# ------------------------------------------------------------------ golden ---
@pytest.mark.parametrize("suf", list(DT))
@pytest.mark.parametrize("n", [2, 4, 8, 16, 64, 1024, 4096])
def test_golden_all_workers_natural(suf, n):
    x, X = load_fft(suf, n)
    for P in (1, 2, 4, 8, n):
        if P > n:
            continue
        plan = pifft.Plan(n, P, 1, PREC[suf])
        got = run(plan, x)
        assert_bins_close(got, X, suf, n)


@pytest.mark.parametrize("suf", list(DT))
def test_reference_known_answer_exact(suf):
    # CPU.c:251-260,689-705: exact float equality
    x = np.array([0, 1, 0, 1, 0, 1, 0, 1], dtype=DT[suf])
    for P in (1, 2, 4, 8):
        got = run(pifft.Plan(8, P, 1, PREC[suf]), x)
        assert np.array_equal(got, np.array([4, 0, 0, 0, -4, 0, 0, 0], dtype=DT[suf]))


@pytest.mark.parametrize("suf", list(DT))
@pytest.mark.parametrize("n,P", [(64, 8), (64, 2), (1024, 4), (4096, 16), (256, 256)])
def test_tree_stage_bitwise_vs_reference(suf, n, P):
    """k_tree / k_tree_stage == the reference's post-tree segments, bit for bit."""
    x, segs = load_tree(suf, n, P)
    plan = pifft.Plan(n, P, 1, PREC[suf], first=0, count=P, device=0, flags=pifft.OUT_SLICES)
    d_in = dev(x)
    d_seg = torch.empty(n, dtype=d_in.dtype, device="cuda")
    plan.tree_device(d_in.data_ptr(), d_seg.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = d_seg.cpu().numpy().reshape(P, n // P)
    assert got.tobytes() == segs.tobytes()
    # and for single-worker plans (one GPU of a P-GPU job)
    for q in (0, P - 1, P // 2):
        p1 = pifft.Plan(n, P, 1, PREC[suf], first=q, count=1, device=0)
        d1 = torch.empty(n // P, dtype=d_in.dtype, device="cuda")
        p1.tree_device(d_in.data_ptr(), d1.data_ptr(), torch.cuda.current_stream())
        torch.cuda.synchronize()
        assert d1.cpu().numpy().tobytes() == segs[q].tobytes(), f"q={q}"


@pytest.mark.parametrize("suf", list(DT))
@pytest.mark.parametrize("logn,P", [(12, 2), (16, 8), (18, 16), (20, 4), (22, 32)])
def test_tree_stage_bitwise_every_worker(suf, logn, P):
    """Every worker's tree output == the oracle's, bit for bit, at sizes where
    glibc's sincos and cos/sin disagree on hundreds of fp64 twiddles (the
    pinned -O2 reference build uses sincos; see oracle/pifft_oracle_impl.h).
    P = 32 takes two tree launches."""
    n = 1 << logn
    x = oracle.generate(n, DT[suf])
    d_in = dev(x)
    want = np.concatenate([oracle.tree_segment(x, P, q) for q in range(P)])
    plan = pifft.Plan(n, P, 1, PREC[suf], first=0, count=P, device=0, flags=pifft.OUT_SLICES)
    d_all = torch.empty(n, dtype=d_in.dtype, device="cuda")
    plan.tree_device(d_in.data_ptr(), d_all.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert d_all.cpu().numpy().tobytes() == want.tobytes()
    m = n // P
    for q in range(P):
        p1 = pifft.Plan(n, P, 1, PREC[suf], first=q, count=1, device=0)
        d1 = torch.empty(m, dtype=d_in.dtype, device="cuda")
        p1.tree_device(d_in.data_ptr(), d1.data_ptr(), torch.cuda.current_stream())
        torch.cuda.synchronize()
        assert d1.cpu().numpy().tobytes() == want[q * m:(q + 1) * m].tobytes(), f"q={q}"
    ref = manifest()["tree_big"].get(f"{suf}_n{n}_p{P}")
    if ref:  # the reference's own per-worker digests
        got = d_all.cpu().numpy().reshape(P, m)
        assert [hashlib.sha256(got[q].tobytes()).hexdigest() for q in range(P)] == ref["sha256_seg_q"]


@pytest.mark.parametrize("suf", list(DT))
@pytest.mark.parametrize("logn,P", [(20, 512), (18, 4096)])
def test_multi_launch_tree_in_place_large_p(suf, logn, P):
    """log2 P > 4: the tree runs as ceil(log2 P / 4) launches, all but the
    first in place over the plan's tree buffer (k_tree without __restrict__).
    A sample of workers, bit for bit against the oracle's post-tree segments,
    and the whole transform against the oracle."""
    n = 1 << logn
    m = n // P
    x = oracle.generate(n, DT[suf], seed=P)
    d_in = dev(x)
    plan = pifft.Plan(n, P, 1, PREC[suf], first=0, count=P, device=0, flags=pifft.OUT_SLICES)
    assert plan.describe()["tree_launches"] == (P.bit_length() - 1 + 3) // 4
    d_all = torch.empty(n, dtype=d_in.dtype, device="cuda")
    plan.tree_device(d_in.data_ptr(), d_all.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = d_all.cpu().numpy()
    for q in sorted({0, 1, P // 3, P // 2 + 1, P - 2, P - 1}):
        assert got[q * m:(q + 1) * m].tobytes() == oracle.tree_segment(x, P, q).tobytes(), f"q={q}"
    assert_bins_close(run(pifft.Plan(n, P, 1, PREC[suf]), x), oracle.fft(x, P=1, nthreads=8), suf, n)


@pytest.mark.parametrize("suf", list(DT))
def test_generator_bitwise(suf):
    n = 1 << 16
    d = torch.empty(n, dtype=TDT[DT[suf]], device="cuda")
    pifft.generate_device(d.data_ptr(), n, n, PREC[suf], seed=0x5EED, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert d.cpu().numpy().tobytes() == oracle.generate(n, DT[suf], 0x5EED).tobytes()
    # the N=2^20 fixture digest
    big = manifest()["big"][suf]
    n = big["n"]
    d = torch.empty(n, dtype=TDT[DT[suf]], device="cuda")
    pifft.generate_device(d.data_ptr(), n, n, PREC[suf], stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert hashlib.sha256(d.cpu().numpy().tobytes()).hexdigest() == big["sha256_x"]


# ------------------------------------------------ the BASELINE configs (1-3) ---
@pytest.mark.parametrize("P", [1, 8])
def test_config1_2_n2e20_fp64(P):
    """C1 (P=1) and C2 (P=8 on one GPU), against the oracle on identical input."""
    n = 1 << 20
    x = oracle.generate(n, np.complex128)
    want = oracle.fft(x, P=P, nthreads=8)
    got = run(pifft.Plan(n, P, 1, pifft.F64), x)
    assert_bins_close(got, want, "f64", n)


def test_config2_slices_per_gpu_fp64():
    """C2 as 8 single-worker plans (one per GPU in the 8-GPU job): each owns
    bins bitrev(q) + 8k, and their all-gather + interleave is the transform."""
    n, P = 1 << 20, 8
    x = oracle.generate(n, np.complex128)
    want = oracle.fft(x, P=1, nthreads=1)
    slices = []
    for q in range(P):
        plan = pifft.Plan(n, P, 1, pifft.F64, first=q, count=1, device=0)
        s = run(plan, x)
        assert_bins_close(s, pifft_dist.slice_of_natural(want, P, q), "f64", n)
        slices.append(s)
    assert_bins_close(pifft_dist.interleave_slices(np.stack(slices)), want, "f64", n)
    # device interleave of the gathered slices
    d_sl = dev(np.concatenate(slices))
    d_out = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.interleave_device(d_sl.data_ptr(), d_out.data_ptr(), n, P, 1, pifft.F64, torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert d_out.cpu().numpy().tobytes() == pifft_dist.interleave_slices(np.stack(slices)).tobytes()


def test_config3_batched_fp32_4096x4096():
    n, b = 4096, 4096
    x = oracle.generate(n, np.complex64, count=n * b)
    plan = pifft.Plan(n, 1, b, pifft.F32)
    assert plan.describe()["num_passes"] == 1
    got = run(plan, x).reshape(b, n)
    xs = x.reshape(b, n)
    # all 4096 transforms against the oracle (the reference's arithmetic, fp32),
    # each with the per-transform rel-L2 and per-bin checks of assert_bins_close
    want = np.stack([oracle.fft(xs[i]) for i in range(b)])
    err = np.linalg.norm(got - want, axis=1) / np.linalg.norm(want, axis=1)
    assert float(err.max()) <= tol("f32", n), f"worst transform rel-L2 {err.max():.3e}"
    rms = np.linalg.norm(want, axis=1) / math.sqrt(n)
    worst = np.max(np.abs(got - want), axis=1)
    assert np.all(worst <= 50 * tol("f32", n) * rms), int(np.argmax(worst / rms))
    # and the whole batch against a float64 numpy FFT (same tolerance)
    assert rel_l2(got, np.fft.fft(xs.astype(np.complex128), axis=1)) <= tol("f32", n)
    # config 3 on 8 GPUs (bench.py --shard batch): rank r generates and runs
    # transforms [512 r, 512 (r+1)) of the same batch; its results are those
    # rows of the 1-GPU batch, bit for bit (same single-pass kernel)
    for r in (0, 5, 7):
        first, count = pifft_dist.batch_range(r, 8, b)
        d_x = torch.empty(count * n, dtype=torch.complex64, device="cuda")
        pifft.generate_device(d_x.data_ptr(), count * n, n, pifft.F32, first=first * n,
                              stream=torch.cuda.current_stream())
        d_y = torch.empty_like(d_x)
        pifft.Plan(n, 1, count, pifft.F32).execute_device(d_x.data_ptr(), d_y.data_ptr(),
                                                          torch.cuda.current_stream())
        torch.cuda.synchronize()
        assert d_x.cpu().numpy().tobytes() == x[first * n:(first + count) * n].tobytes(), f"rank {r} input"
        assert d_y.cpu().numpy().reshape(count, n).tobytes() == got[first:first + count].tobytes(), f"rank {r}"


# ------------------------------------------------------------- sweeps/edges ---
@pytest.mark.parametrize("suf", list(DT))
@pytest.mark.parametrize("logn", list(range(1, 23)))
def test_size_sweep_vs_oracle(suf, logn):
    n = 1 << logn
    x = oracle.generate(n, DT[suf], seed=1234 + logn)
    want = oracle.fft(x, P=1)
    for P in sorted({1, 2, min(n, 8), min(n, 32)}):
        got = run(pifft.Plan(n, P, 1, PREC[suf]), x)
        assert_bins_close(got, want, suf, n)


@pytest.mark.parametrize("suf", list(DT))
@pytest.mark.parametrize("n,P,b", [(2, 2, 3), (16, 16, 5), (1024, 4, 7), (1 << 15, 8, 3), (1 << 16, 64, 2),
                                   (64, 64, 2), (8192, 1, 33), (1 << 14, 2, 4)])
def test_batched_and_many_workers(suf, n, P, b):
    x = oracle.generate(n, DT[suf], seed=99, count=n * b)
    got = run(pifft.Plan(n, P, b, PREC[suf]), x).reshape(b, n)
    for i in range(b):
        assert_bins_close(got[i], oracle.fft(x[i * n:(i + 1) * n]), suf, n)


@pytest.mark.parametrize("suf", list(DT))
def test_worker_ranges_slices_layout(suf):
    n, P = 1 << 12, 16
    x = oracle.generate(n, DT[suf])
    want = oracle.fft(x)
    for first, count in [(0, 16), (0, 8), (8, 8), (4, 4), (12, 2), (5, 1)]:
        plan = pifft.Plan(n, P, 1, PREC[suf], first=first, count=count, device=0, flags=pifft.OUT_SLICES)
        got = run(plan, x).reshape(count, n // P)
        for j in range(count):
            assert_bins_close(got[j], pifft_dist.slice_of_natural(want, P, first + j), suf, n)


def test_host_boundary_and_group():
    """pifft_execute (the reference run() shape) and pifft_execute_group (the
    multi-GPU job from one host thread; here 4 plans share device 0)."""
    n, P = 1 << 14, 4
    x = oracle.generate(n, np.complex128)
    want = oracle.fft(x)
    out = np.zeros_like(x)
    t1, t2 = pifft.Plan(n, P, 1, pifft.F64).execute(x, out)
    assert t1 >= 0 and t2 > 0
    assert_bins_close(out, want, "f64", n)
    plans = [pifft.Plan(n, P, 1, pifft.F64, first=q, count=1, device=0) for q in range(P)]
    out2 = np.zeros_like(x)
    pifft.execute_group(plans, x, out2)
    assert_bins_close(out2, want, "f64", n)


def test_timed_execution_reports_every_launch(monkeypatch):
    n = 1 << 20
    monkeypatch.setenv("PIFFT_WIL_FUSE", "0")  # (the three-launch form: tree + two passes)
    plan = pifft.Plan(n, 8, 1, pifft.F64)
    d = plan.describe()
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, stream=torch.cuda.current_stream())
    y = torch.empty(n, dtype=torch.complex128, device="cuda")
    ms = plan.execute_device_timed(x.data_ptr(), y.data_ptr(), torch.cuda.current_stream())
    assert len(ms) == d["num_launches"] and all(m > 0 for m in ms)
    # (the last pass stores natural order itself at this size: no interleave launch)
    assert d["launch_kind"] == ["tree", "pass", "pass"]
    # asynchronous profiling: events for 3 back-to-back executions, one read
    plan.profile_start(3, pifft.PROFILE_ALL)
    for _ in range(5):  # only the first 3 are recorded
        plan.execute_device(x.data_ptr(), y.data_ptr(), torch.cuda.current_stream())
    used, sums, cnt = plan.profile_read()
    assert used == 3 and len(sums) == d["num_launches"] and all(m > 0 for m in sums) and cnt == [3, 3, 3]
    assert plan.profile_read()[0] == 0
    # in-context sampling: odd executions time launch (k/2) mod 3 -> 2 samples each in 12
    plan.profile_start(12, pifft.PROFILE_SAMPLED)
    for _ in range(12):
        plan.execute_device(x.data_ptr(), y.data_ptr(), torch.cuda.current_stream())
    used, sums, cnt = plan.profile_read()
    assert used == 12 and cnt == [2, 2, 2] and all(m > 0 for m in sums)
    with pytest.raises(pifft.PifftError, match="profile mode"):
        plan.profile_start(3, 7)
    torch.cuda.synchronize()
    # the profiled executions compute the same transform
    want = y.clone()
    plan.execute_device(x.data_ptr(), y.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert torch.equal(y, want)


def test_launch_loop_times_and_restores_the_result():
    """pifft_launch_loop (bench.py's dominant-kernel timing): a clean loop of
    some launches alone, then one full execution -- the output is bitwise the
    plan's result again (the loop re-runs launches on whatever their buffers
    hold); out-of-range launches, reps < 1 and an empty list are refused."""
    n = 1 << 20
    plan = pifft.Plan(n, 8, 1, pifft.F64)
    st = torch.cuda.current_stream()
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, stream=st)
    want = torch.empty(n, dtype=torch.complex128, device="cuda")
    plan.execute_device(x.data_ptr(), want.data_ptr(), st)
    y = torch.zeros_like(want)
    nl = plan.info.num_launches
    for ls in ([nl - 1], list(range(nl))):
        ms = plan.launch_loop(ls, 50, x.data_ptr(), y.data_ptr(), st)
        assert 0 < ms < 1.0, ms
        torch.cuda.synchronize()
        assert torch.equal(y, want)
    for ls, reps in (([nl], 5), ([-1], 5), ([0], 0), ([], 5)):
        with pytest.raises(pifft.PifftError):
            plan.launch_loop(ls, reps, x.data_ptr(), y.data_ptr(), st)


@pytest.mark.parametrize("suf,logn,P", [("f64", 22, 1), ("f32", 24, 1), ("f64", 21, 8)])
def test_tune_workspace_keeps_results(suf, logn, P):
    """pifft_plan_tune_workspace only re-places the plan's workspace: the
    output is bitwise the untuned plan's; a plan without a workspace (single
    pass) returns at once; tries < 1 is refused."""
    n = 1 << logn
    x = dev(oracle.generate(n, DT[suf], seed=logn))
    st = torch.cuda.current_stream()
    kw = dict(first=0, count=1, device=0) if P > 1 else {}
    plan = pifft.Plan(n, P, 1, PREC[suf], **kw)
    a = torch.empty(plan.info.out_elems, dtype=x.dtype, device="cuda")
    plan.execute_device(x.data_ptr(), a.data_ptr(), st)
    ms = plan.tune_workspace(x.data_ptr(), a.data_ptr(), st, 3)
    assert ms > 0
    b = torch.empty_like(a)
    plan.execute_device(x.data_ptr(), b.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    single = pifft.Plan(4096, 1, 4, PREC[suf])
    y = torch.empty(4 * 4096, dtype=x.dtype, device="cuda")
    assert single.tune_workspace(x.data_ptr(), y.data_ptr(), st, 4) == 0.0
    with pytest.raises(pifft.PifftError, match="tries"):
        plan.tune_workspace(x.data_ptr(), a.data_ptr(), st, 0)


def test_device_errors():
    plan = pifft.Plan(64, 2, 1, pifft.F64)
    x = torch.zeros(64, dtype=torch.complex128, device="cuda")
    with pytest.raises(pifft.PifftError, match="in-place"):
        plan.execute_device(x.data_ptr(), x.data_ptr())
    with pytest.raises(pifft.PifftError, match="device"):
        pifft.Plan(64, 2, 1, pifft.F64, first=0, count=2, device=pifft.gpu_count())


# ------------------------------------------------------ full-size properties ---
def _dft_bins(x, ks):
    """Direct DFT bins in float64 (chunked; exact integer phase)."""
    n = len(x)
    out = []
    for k in ks:
        acc = 0j
        for s in range(0, n, 1 << 22):
            idx = np.arange(s, min(n, s + (1 << 22)), dtype=np.int64)
            ph = (idx * k) % n
            acc += np.sum(x[s:s + len(idx)].astype(np.complex128) * np.exp(-2j * np.pi * ph / n))
        out.append(acc)
    return np.array(out)


@pytest.mark.parametrize("logn,P", [(24, 1), (24, 8), (26, 4), (28, 1), (28, 8)])
def test_large_fp64_properties(logn, P):
    n = 1 << logn
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, stream=torch.cuda.current_stream())
    plan = pifft.Plan(n, P, 1, pifft.F64)
    X = torch.empty_like(x)
    plan.execute_device(x.data_ptr(), X.data_ptr(), torch.cuda.current_stream())
    # double transform: FFT(conj(FFT(x))) = N conj(x)
    Y = torch.empty_like(x)
    Xc = X.conj().resolve_conj().contiguous()
    plan.execute_device(Xc.data_ptr(), Y.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    err = (torch.linalg.vector_norm(Y.conj() / n - x) / torch.linalg.vector_norm(x)).item()
    assert err <= 1e-12, err
    # Parseval
    pe = abs(torch.linalg.vector_norm(X).item() ** 2 / n - torch.linalg.vector_norm(x).item() ** 2)
    assert pe <= 1e-12 * torch.linalg.vector_norm(x).item() ** 2
    # direct DFT bins
    xh = x.cpu().numpy()
    ks = [0, 1, n // 2 + 3, n - 1, 12345 % n]
    want = _dft_bins(xh, ks)
    got = X.cpu().numpy()[ks]
    scale = np.linalg.norm(xh)  # |X[k]| ~ ||x||
    assert np.max(np.abs(got - want)) <= 1e-12 * scale * math.sqrt(n) * 10
    del Y, Xc
    if logn <= 24:  # the oracle itself (8 threads) at 2^24
        want_full = oracle.fft(xh, P=8, nthreads=8)
        assert_bins_close(X.cpu().numpy(), want_full, "f64", n)


def test_large_split_consistency_fp64():
    """2^28 split over 8 single-worker plans (the 8-GPU job, one GPU at a time)
    equals the 1-worker transform bin for bin."""
    n, P = 1 << 28, 8
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, stream=torch.cuda.current_stream())
    full = torch.empty_like(x)
    pifft.Plan(n, 1, 1, pifft.F64).execute_device(x.data_ptr(), full.data_ptr(), torch.cuda.current_stream())
    for q in (0, 3, 7):
        plan = pifft.Plan(n, P, 1, pifft.F64, first=q, count=1, device=0)
        s = torch.empty(n // P, dtype=torch.complex128, device="cuda")
        plan.execute_device(x.data_ptr(), s.data_ptr(), torch.cuda.current_stream())
        r = pifft_dist.bitrev(q, 3)
        ref = full[r::P]
        torch.cuda.synchronize()
        err = (torch.linalg.vector_norm(s - ref) / torch.linalg.vector_norm(ref)).item()
        assert err <= 1e-12, (q, err)


def test_large_fp64_linearity():
    n = 1 << 26
    a = torch.empty(n, dtype=torch.complex128, device="cuda")
    b = torch.empty_like(a)
    pifft.generate_device(a.data_ptr(), n, n, pifft.F64, seed=1, stream=torch.cuda.current_stream())
    pifft.generate_device(b.data_ptr(), n, n, pifft.F64, seed=2, stream=torch.cuda.current_stream())
    plan = pifft.Plan(n, 1, 1, pifft.F64)
    outs = []
    for v in (a, b, (2.0 * a - 3.0 * b).contiguous()):
        o = torch.empty_like(v)
        plan.execute_device(v.data_ptr(), o.data_ptr(), torch.cuda.current_stream())
        outs.append(o)
    torch.cuda.synchronize()
    lhs, rhs = outs[2], 2.0 * outs[0] - 3.0 * outs[1]
    assert (torch.linalg.vector_norm(lhs - rhs) / torch.linalg.vector_norm(rhs)).item() <= 1e-13


# -------------------------------------------------------------------- CLI ---
def _cli(args, env=None):
    import subprocess
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([pifft.CLI_PATH] + args, capture_output=True, text=True, timeout=300, env=e)


@pytest.mark.parametrize("prec", ["32", "64"])
@pytest.mark.parametrize("P", ["1", "2", "4", "8"])
def test_cli_known_answer(prec, P):
    r = _cli(["-t", "-p", P, "-f", prec])
    assert r.returncode == 0, r.stderr
    assert "Output is correct. Test passed." in r.stdout
    assert "4.0+0.0i, 0.0+0.0i, 0.0+0.0i, 0.0+0.0i, -4.0+0.0i" in r.stdout


def test_cli_tsv_and_dump(tmp_path):
    r = _cli(["-n", "65536", "-p", "8", "-o"])
    assert r.returncode == 0, r.stderr
    cols = r.stdout.strip().split("\t")
    assert len(cols) == 5 and cols[0] == "65536" and cols[1] == "8"
    assert abs(float(cols[2]) - float(cols[3]) - float(cols[4])) < 1e-3
    r = _cli(["-n", "1024", "-p", "4"])
    assert r.stdout.splitlines()[0] == "n\tp\ttime (total)\ttime (stage 1)\ttime (stage 2)"
    out = tmp_path / "x.bin"
    r = _cli(["-n", "4096", "-p", "4", "-f", "64", "-s", "7", "-w", str(out), "-o"])
    assert r.returncode == 0, r.stderr
    got = np.fromfile(out, dtype=np.complex128)
    x = oracle.generate(4096, np.complex128, seed=7)
    assert_bins_close(got, oracle.fft(x, P=4), "f64", 4096)
    # -r: the reference's scratch order, on one GPU and split over two plans
    for g in ("1", "2"):
        r = _cli(["-n", "4096", "-p", "4", "-f", "64", "-s", "7", "-w", str(out), "-o", "-r", "-g", g])
        if g == "2" and pifft.gpu_count() < 2:
            continue
        assert r.returncode == 0, r.stderr
        got = np.fromfile(out, dtype=np.complex128)
        assert_bins_close(got, oracle.fft(x, P=4)[_bitrev_perm(4096)], "f64", 4096)


def test_cli_extra_columns_kernel_and_wall_stages():
    """-x: GFLOP/s, GB/s and the kernel-only stage sums beside the wall-clock
    stage timers (markers around each stage, the reference's tm_funnel /
    tm_tube, CPU.c:414-481): the kernels fit inside the wall stage times."""
    for args in (["-n", "1048576", "-p", "8", "-f", "64"], ["-n", "1048576", "-p", "8", "-f", "64", "-u"],
                 ["-n", "1048576", "-p", "1", "-f", "64"]):
        r = _cli(args + ["-x", "-W", "3"])
        assert r.returncode == 0, r.stderr
        head, vals = r.stdout.strip().splitlines()[-2:]
        assert head.split("\t")[-2:] == ["kernels (stage 1)", "kernels (stage 2)"]
        c = [float(v) for v in vals.split("\t")]
        assert len(c) == 9 and abs(c[2] - c[3] - c[4]) < 1e-3
        assert c[7] >= 0 and c[8] > 0 and c[7] + c[8] <= 1.2 * c[2] + 0.005, c
        if args[3] == "1":
            assert c[3] == 0 and c[7] == 0  # P = 1: no tree stage


@pytest.mark.parametrize("args", [["-f", "64", "-p", "8", "-g", "4"], ["-f", "32", "-p", "8", "-g", "8"],
                                  ["-f", "64", "-p", "4", "-g", "2", "-r"], ["-f", "64", "-p", "16", "-g", "4", "-b", "3"]])
def test_cli_split_checks_itself(args):
    """-t with -g G > 1 (rehearsed on GPU 0, -R): the split's result against a
    one-GPU all-worker plan (rel-L2) and each plan's worker range replayed on
    GPU 0 bit for bit.  -n after -t transforms 4096 points (the reference's
    quirk: its N = 8 known answer then fails, the split check still runs)."""
    r = _cli(["-t", "-n", "4096"] + args + ["-R"])
    assert r.returncode == 0, r.stderr
    assert "Split check passed." in r.stdout, r.stdout[-400:]
    assert "replayed bit for bit: yes" in r.stdout
    # a failing check is a failing run (round-4 advice): one output bit flipped
    # (test-only PIFFT_FAULT=split_check) -> "FAILED" and a non-zero exit status
    r = _cli(["-t", "-n", "4096"] + args + ["-R"], env={"PIFFT_TUNING": "1", "PIFFT_FAULT": "split_check"})
    assert "Split check FAILED." in r.stdout, r.stdout[-400:]
    assert r.returncode == 1 and "Could not run" not in r.stderr, (r.returncode, r.stderr)


@pytest.mark.parametrize("P", ["1", "2", "8"])
def test_cli_known_answer_scratch_order(P):
    r = _cli(["-t", "-p", P, "-r"])
    assert r.returncode == 0, r.stderr
    assert "Output is correct. Test passed." in r.stdout


# ------------------------------------------------- fused tree + first pass ---
@pytest.mark.parametrize("suf", list(DT))
@pytest.mark.parametrize("logn,P", [(16, 2), (18, 4), (19, 8), (20, 16), (22, 2), (23, 8), (24, 2), (24, 8), (25, 4), (26, 8)])
def test_fused_tree_first_pass(suf, logn, P, monkeypatch):
    """Single-worker plans with a multi-pass local FFT evaluate the tree inside
    the first pass (MODE 3); results must match the oracle and the unfused plan."""
    n = 1 << logn
    x = oracle.generate(n, DT[suf], seed=logn * 7 + P)
    want = oracle.fft(x, P=1, nthreads=8)
    for q in sorted({0, (P // 2 + 1) % P, P - 1}):
        fused = pifft.Plan(n, P, 1, PREC[suf], first=q, count=1, device=0)
        kinds = fused.describe()["launch_kind"]
        assert "tree" not in kinds, kinds  # fused: no separate tree launch
        got = run(fused, x)
        assert_bins_close(got, pifft_dist.slice_of_natural(want, P, q), suf, n)
        plain = pifft.Plan(n, P, 1, PREC[suf], first=q, count=1, device=0,
                           flags=pifft.OUT_SLICES | pifft.SEPARATE_TREE)
        assert plain.describe()["launch_kind"][0] == "tree"
        assert rel_l2(run(plain, x), got) <= tol(suf, n)


@pytest.mark.parametrize("env,last_vpt", [({}, 8), ({"PIFFT_LAST_VPT": "16"}, 16),
                                          ({"PIFFT_LAST_VPT": "8", "PIFFT_LAST_C": "8"}, 8)])
@pytest.mark.parametrize("logn,P", [(20, 8), (18, 4), (21, 16)])
def test_slice_last_pass_forms_vs_oracle(logn, P, env, last_vpt, monkeypatch):
    """One-worker fp64 slices (config 2's shape and neighbours): the last
    strided pass runs at 8 values per thread by default (round 4), at 16 or
    at C = 8 under the tuning variables -- every form matches the oracle."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    n = 1 << logn
    x = oracle.generate(n, DT["f64"], seed=logn * 5 + P)
    want = oracle.fft(x, P=1, nthreads=8)
    for q in sorted({0, P - 1}):
        plan = pifft.Plan(n, P, 1, pifft.F64, first=q, count=1, device=0)
        d = plan.describe()
        assert d["launch_kind"] == ["tree+pass", "pass"] and d["vpt"][-1] == last_vpt, d
        assert_bins_close(run(plan, x), pifft_dist.slice_of_natural(want, P, q), "f64", n)


def test_cli_separate_tree_stage_columns(tmp_path):
    """CLI -u (PIFFT_SEPARATE_TREE): the tree stays its own launch, so the TSV's
    stage-1 column is the funnel alone (the column analyze-results.R:56 fits
    on n(p-1)/p); without it a one-worker-per-GPU plan fuses the tree into the
    first pass (stage 1 = tree + first pass), and an all-worker plan too
    (MODE 11, whose first radix then differs).  The same transform either
    way."""
    import subprocess
    cli = pifft.CLI_PATH
    n, P = 1 << 20, 8
    outs = {}
    for flag in ([], ["-u"]):
        # (one GPU holds all 8 workers here; the stage split of a one-worker
        # plan is checked through the ABI below)
        dump = str(tmp_path / f"out{len(flag)}.bin")
        r = subprocess.run([cli, "-n", str(n), "-p", str(P), "-o", "-f", "64", "-s", "3", "-w", dump] + flag,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        cols = r.stdout.strip().splitlines()[-1].split("\t")
        assert len(cols) == 5 and float(cols[3]) > 0 and float(cols[4]) > 0
        outs[bool(flag)] = open(dump, "rb").read()
    a, b = (np.frombuffer(outs[k], dtype=np.complex128) for k in (False, True))
    assert rel_l2(a, b) <= 1e-12
    x = oracle.generate(n, np.complex128, seed=3)
    fused = pifft.Plan(n, P, 1, pifft.F64, first=0, count=1, device=0)
    sep = pifft.Plan(n, P, 1, pifft.F64, first=0, count=1, device=0, flags=pifft.OUT_SLICES | pifft.SEPARATE_TREE)
    assert fused.describe()["launch_kind"][0] == "tree+pass"
    assert sep.describe()["launch_kind"][:2] == ["tree", "pass"]
    out = np.zeros(n, np.complex128)
    t1, t2 = sep.execute(x, out)
    assert t1 > 0 and t2 > 0
    assert_bins_close(pifft_dist.slice_of_natural(out, P, 0), pifft_dist.slice_of_natural(oracle.fft(x, P=1), P, 0),
                      "f64", n)


# ------------------------------------------------------------- config 5 ---
def _dft_bins_gpu(x, ks):
    """Direct DFT bins on the GPU in float64 (exact integer phase mod N)."""
    n = x.numel()
    mask = n - 1
    out = []
    for k in ks:
        acc = torch.zeros((), dtype=torch.complex128, device=x.device)
        for s in range(0, n, 1 << 26):
            idx = torch.arange(s, min(n, s + (1 << 26)), dtype=torch.int64, device=x.device)
            ph = (idx * k) & mask  # wraps mod 2^64, exact mod N = 2^m
            ang = ph.to(torch.float64) * (-2.0 * math.pi / n)
            acc = acc + torch.sum(x[s:s + idx.numel()] * torch.polar(torch.ones_like(ang), ang))
        out.append(acc.item())
    return np.array(out)


def test_config5_one_worker_of_8_n2e32():
    """Config 5 on one GPU: worker q of the 8-GPU split of an fp64 N=2^32
    transform (64 GiB input replica, 64-bit indexing, fused tree).  Checked
    against direct DFT bins X[bitrev(q) + 8k] computed on the GPU."""
    free, total = torch.cuda.mem_get_info()
    if free < 110 * (1 << 30):
        pytest.skip("needs ~110 GiB of HBM")
    n, P, q = 1 << 32, 8, 5
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, stream=torch.cuda.current_stream())
    plan = pifft.Plan(n, P, 1, pifft.F64, first=q, count=1, device=0)
    d = plan.describe()
    assert d["local_n"] == n // P and "tree+pass" in d["launch_kind"]
    y = torch.empty(n // P, dtype=torch.complex128, device="cuda")
    plan.execute_device(x.data_ptr(), y.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    r = pifft_dist.bitrev(q, 3)
    kk = [0, 1, 12345, n // P - 1]
    want = _dft_bins_gpu(x, [r + P * k for k in kk])
    got = y[kk].cpu().numpy()
    scale = torch.linalg.vector_norm(x).item()
    assert np.max(np.abs(got - want)) <= 1e-10 * scale, (got, want)


# ------------------------------------------- the reference's run(), patched ---
def _ref_gpu(prec):
    p = os.path.join(oracle.REF_DIR, "fourier-parallel-pi-cpu-pthreads-gpu" + ("-f64" if prec == 64 else ""))
    # built in the build container (__graft_entry__.build) and shipped with the
    # tree: its absence on the GPU box is a failure, not a skip
    assert os.path.exists(p), "oracle/_ref integration binary not built (make -C oracle ref-gpu)"
    return p


@pytest.mark.parametrize("prec", [32, 64])
def test_reference_run_with_pifft_backend(prec):
    """INTEGRATION.md section 2 applied to the reference source itself: its own
    main / setup_from_args / initialize_data / verify_results, with the worker
    fan-out of run() replaced by pifft_plan_create + pifft_execute."""
    import subprocess
    exe = _ref_gpu(prec)
    for P in ("1", "2", "4", "8"):
        r = subprocess.run([exe, "-t", "-p", P], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        assert "Output is correct. Test passed." in r.stdout
    r = subprocess.run([exe, "-n", "1048576", "-p", "8", "-o"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    cols = r.stdout.strip().split("\t")
    assert len(cols) == 5 and cols[:2] == ["1048576", "8"]
    r = subprocess.run([exe, "-n", "1048576"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "Missing option: -p" in r.stderr


# ------------------------------------- bit-reversed (reference scratch) order ---
def _bitrev_perm(n):
    bits = n.bit_length() - 1
    i = np.arange(n, dtype=np.uint64)
    r = np.zeros(n, dtype=np.uint64)
    for b in range(bits):
        r |= ((i >> np.uint64(b)) & np.uint64(1)) << np.uint64(bits - 1 - b)
    return r.astype(np.int64)


@pytest.mark.parametrize("suf", list(DT))
@pytest.mark.parametrize("n", [8, 64, 1024, 4096])
def test_bitrev_output_is_reference_scratch(suf, n):
    """PIFFT_OUT_BITREV == the reference's tmp_in after the cylinder stage
    (CPU.c:463-478): its scatter out[bitrev(i)] = tmp_in[i] (CPU.c:496-499)
    is a pure permutation, so tmp_in = golden X[bitrev_N(i)] exactly."""
    x, X = load_fft(suf, n)
    want = X[_bitrev_perm(n)]
    for P in (1, 2, 8):
        if P > n:
            continue
        got = run(pifft.Plan(n, P, 1, PREC[suf], first=0, count=P, device=0, flags=pifft.OUT_BITREV), x)
        assert_bins_close(got, want, suf, n)


@pytest.mark.parametrize("suf", list(DT))
@pytest.mark.parametrize("logn,P,batch", [(16, 1, 3), (20, 8, 1), (22, 4, 2), (24, 1, 1)])
def test_bitrev_output_vs_oracle(suf, logn, P, batch):
    """Multi-pass local FFTs (the last Stockham pass stores bit-reversed), all
    workers and single-worker plans, batched; vs the oracle permuted."""
    n = 1 << logn
    m = n // P
    xs = [oracle.generate(n, DT[suf], seed=0x5EED + b) for b in range(batch)]
    Xs = [oracle.fft(x, P=P, nthreads=8) for x in xs]
    perm = _bitrev_perm(n)
    d_in = dev(np.concatenate(xs))
    plan = pifft.Plan(n, P, batch, PREC[suf], first=0, count=P, device=0, flags=pifft.OUT_BITREV)
    d_out = torch.empty(batch * n, dtype=d_in.dtype, device="cuda")
    plan.execute_device(d_in.data_ptr(), d_out.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    got = d_out.cpu().numpy().reshape(batch, n)
    for b in range(batch):
        assert_bins_close(got[b], Xs[b][perm], suf, n)
    if P > 1:
        q = P - 2
        p1 = pifft.Plan(n, P, batch, PREC[suf], first=q, count=1, device=0, flags=pifft.OUT_BITREV)
        d1 = torch.empty(batch * m, dtype=d_in.dtype, device="cuda")
        p1.execute_device(d_in.data_ptr(), d1.data_ptr(), torch.cuda.current_stream())
        torch.cuda.synchronize()
        g1 = d1.cpu().numpy().reshape(batch, m)
        for b in range(batch):
            assert_bins_close(g1[b], Xs[b][perm][q * m:(q + 1) * m], suf, n)


def test_bitrev_host_boundary_segments():
    """pifft_execute on a PIFFT_OUT_BITREV plan writes the reference's tmp_in
    segments of its workers at q*M (other positions untouched)."""
    n, P = 1 << 12, 4
    x = oracle.generate(n, np.complex128)
    want = oracle.fft(x, P=P)[_bitrev_perm(n)]
    out = np.full(n, np.nan + 0j, dtype=np.complex128)
    plan = pifft.Plan(n, P, 1, pifft.F64, first=2, count=2, device=0, flags=pifft.OUT_BITREV)
    plan.execute(x, out)
    m = n // P
    assert np.all(np.isnan(out[:2 * m]))
    assert_bins_close(out[2 * m:], want[2 * m:], "f64", n)


# ---------------------------------------- worker-interleaved layout (wil) ---
@pytest.mark.parametrize("suf,logn,P,batch", [("f64", 20, 8, 1), ("f64", 21, 2, 2), ("f32", 20, 8, 3),
                                              ("f64", 19, 16, 1), ("f32", 22, 4, 1), ("f64", 18, 8, 2),
                                              ("f64", 24, 8, 1), ("f32", 16, 2, 5), ("f32", 23, 16, 1)])
def test_worker_interleaved_layout_vs_slice_major(suf, logn, P, batch, monkeypatch):
    """All-worker natural-order plans on the worker-interleaved layout (tree
    writing z_q[i] at i P + q, MODE 10 passes, the last one storing worker q
    at slot bitrev(q)) equal the slice-major plans (PIFFT_WORKER_IL=0: the
    same per-line arithmetic, then the interleave or the natural-order store)
    value for value, and the oracle within tolerance."""
    n = 1 << logn
    x = oracle.generate(n * batch, DT[suf], seed=logn * 3 + P)
    d_in = dev(x)
    st = torch.cuda.current_stream()
    # (the default plan, whose passes run at 8 values per thread at config-2
    # sizes, against the oracle; then at 16, the slice-major plan's radices,
    # value for value)
    dflt = pifft.Plan(n, P, batch, PREC[suf])
    a = torch.empty_like(d_in)
    dflt.execute_device(d_in.data_ptr(), a.data_ptr(), st)
    torch.cuda.synchronize()
    got = a.cpu().numpy().reshape(batch, n)
    for bt in range(batch):
        assert_bins_close(got[bt], oracle.fft(x[bt * n:(bt + 1) * n], P=1, nthreads=8), suf, n)
    monkeypatch.setenv("PIFFT_WIL_VPT", "16")
    # (the default plan's tree reads the factored two-level twiddles; with the
    # reference-formula table -- the slice-major plan's -- the arithmetic is the
    # slice-major plan's, bit for bit)
    monkeypatch.setenv("PIFFT_WIL_TREE_DIRECT", "1")
    monkeypatch.setenv("PIFFT_WIL_FUSE", "0")  # (the tree as its own launch, as the slice-major plan's)
    wil = pifft.Plan(n, P, batch, PREC[suf])
    assert wil.describe()["worker_interleaved"] and "interleave" not in wil.describe()["launch_kind"]
    assert set(wil.describe()["vpt"]) == {16}
    monkeypatch.setenv("PIFFT_WORKER_IL", "0")
    sm = pifft.Plan(n, P, batch, PREC[suf])
    assert not sm.describe()["worker_interleaved"]
    a = torch.empty_like(d_in)
    b = torch.empty_like(d_in)
    wil.execute_device(d_in.data_ptr(), a.data_ptr(), st)
    sm.execute_device(d_in.data_ptr(), b.data_ptr(), st)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    got = a.cpu().numpy().reshape(batch, n)
    for bt in range(batch):
        assert_bins_close(got[bt], oracle.fft(x[bt * n:(bt + 1) * n], P=1, nthreads=8), suf, n)



@pytest.mark.parametrize("suf,logn,P,batch,j", [("f64", 20, 8, 1, 0), ("f64", 20, 8, 1, 16), ("f32", 20, 8, 1, 0),
                                                ("f64", 18, 4, 2, 0), ("f64", 16, 2, 3, 0), ("f64", 22, 16, 1, 4),
                                                ("f32", 22, 16, 2, 0), ("f64", 21, 8, 1, 4), ("f32", 17, 2, 1, 32),
                                                ("f64", 24, 8, 1, 0), ("f32", 23, 4, 1, 0), ("f64", 19, 16, 1, 8),
                                                ("f32", 20, 8, 1, 16), ("f64", 20, 2, 1, 0), ("f64", 22, 4, 1, 0),
                                                ("f64", 22, 8, 1, 0), ("f32", 21, 8, 1, 0), ("f32", 22, 8, 1, 0),
                                                ("f64", 17, 4, 1, 0), ("f32", 18, 8, 2, 0), ("f64", 17, 8, 1, 0),
                                                ("f64", 14, 2, 1, 0), ("f64", 15, 4, 1, 0), ("f32", 16, 16, 1, 0),
                                                ("f32", 16, 8, 1, 0), ("f32", 12, 4, 3, 0), ("f64", 11, 8, 5, 0),
                                                ("f64", 12, 32, 2, 0), ("f32", 10, 2, 7, 0), ("f64", 13, 2, 64, 0),
                                                ("f64", 15, 4, 3, 0),
                                                ("f32", 14, 8, 5, 0), ("f32", 21, 16, 1, 0), ("f64", 21, 16, 1, 0)])
def test_fused_all_worker_tree_pass(suf, logn, P, batch, j, monkeypatch):
    """All-worker natural-order plans with every worker's tree fused into the
    first worker-interleaved pass (MODE 11: each position's P leaves loaded
    once, the full radix-2 tree, an LDS transpose into the pass): against the
    oracle (tolerance + per bin) and against the same plan with the tree as
    its own launch (PIFFT_WIL_FUSE=0).  j: the tile's adjacent line indices
    (PIFFT_WIL_FUSE_J; 0 = the planner's: the 4096-value tile at J = 4 up to
    2^20 values, J = 4 where J = 8 would split the remainder, else J = 8)."""
    n = 1 << logn
    x = oracle.generate(n * batch, DT[suf], seed=logn * 5 + P + j)
    if j:
        monkeypatch.setenv("PIFFT_WIL_FUSE_J", str(j))
    fused = pifft.Plan(n, P, batch, PREC[suf])
    d = fused.describe()
    assert d["worker_interleaved"] and d["launch_kind"][0] == "tree+pass" and d["launch_mode"][0] == 11, d
    assert "tree" not in d["launch_kind"] and "interleave" not in d["launch_kind"]
    got = run(fused, x).reshape(batch, n)
    for bt in range(batch):
        assert_bins_close(got[bt], oracle.fft(x[bt * n:(bt + 1) * n], P=1, nthreads=8), suf, n)
    monkeypatch.setenv("PIFFT_WIL_FUSE", "0")
    sep = pifft.Plan(n, P, batch, PREC[suf])
    assert sep.describe()["launch_kind"][0] == "tree"
    assert rel_l2(run(sep, x), got.reshape(-1)) <= tol(suf, n)


ONE = ["tree+pass"]
TWO = ["tree+pass", "pass"]
THREE = ["tree", "pass", "interleave"]


@pytest.mark.parametrize("suf,logn,P,kinds", [("f64", 17, 16, ["tree", "pass", "pass"]), ("f64", 18, 16, ["tree", "pass", "pass"]),
                                             ("f64", 16, 16, ["tree", "pass", "pass"]), ("f64", 15, 4, TWO),
                                             ("f32", 17, 8, TWO), ("f32", 14, 2, TWO), ("f64", 14, 8, TWO),
                                             ("f64", 14, 16, THREE), ("f32", 15, 16, TWO),
                                             ("f64", 13, 2, THREE), ("f64", 12, 2, ONE)])
def test_single_pass_all_worker_plans_two_pass(suf, logn, P, kinds, monkeypatch):
    """A single transform whose local FFT is one pass (N / P <= 2^14) runs the
    two-pass worker-interleaved plan from 2^11 points per worker up (the fused
    tree pass, or at fp64 P = 16 the tree launch and two passes), and a
    transform of P M <= 8192 values (M < 4096) one fused launch: against the
    oracle and against the three-launch plan (PIFFT_WIL_SINGLE=0), within
    tolerance (the radices differ)."""
    n = 1 << logn
    x = oracle.generate(n, DT[suf], seed=logn * 7 + P)
    plan = pifft.Plan(n, P, 1, PREC[suf])
    d = plan.describe()
    assert d["launch_kind"] == kinds and d["worker_interleaved"] == (kinds != THREE), d
    got = run(plan, x)
    assert_bins_close(got, oracle.fft(x, P=1, nthreads=8), suf, n)
    monkeypatch.setenv("PIFFT_WIL_SINGLE", "0")
    single = pifft.Plan(n, P, 1, PREC[suf])
    assert single.describe()["launch_kind"] == THREE
    assert rel_l2(run(single, x), got) <= tol(suf, n)


@pytest.mark.parametrize("suf", ["f64", "f32"])
@pytest.mark.parametrize("logn", [10, 11, 12, 13])
@pytest.mark.parametrize("P", [2, 4, 8, 16, 32])
def test_tiny_all_worker_plans_one_launch(suf, logn, P, monkeypatch):
    """The reference's own GPU sweep grid (cuda/run-experiments:16-17: n =
    1024-8192, p up to 32): one fused launch -- every worker's tree, then its
    whole N/P-point FFT, natural-order store -- where N/P < 4096 (P = 32: two
    threads per position, each with half the workers' tree; fp64 up to 4096),
    against the oracle and the three-launch (P = 32: four-launch) plan."""
    n = 1 << logn
    x = oracle.generate(n, DT[suf], seed=logn * 3 + P)
    plan = pifft.Plan(n, P, 1, PREC[suf])
    kinds = plan.describe()["launch_kind"]
    many = ["tree", "tree", "pass", "interleave"] if P == 32 else THREE
    one = (n // P < 4096 or (suf == "f32" and P == 2)) and not (P == 32 and suf == "f64" and n == 8192)
    assert kinds == (ONE if one else many), kinds
    got = run(plan, x)
    assert_bins_close(got, oracle.fft(x, P=1, nthreads=8), suf, n)
    monkeypatch.setenv("PIFFT_WIL_ONE_LAUNCH", "0")
    three = pifft.Plan(n, P, 1, PREC[suf])
    assert three.describe()["launch_kind"] == many
    assert rel_l2(run(three, x), got) <= tol(suf, n)


# ------------------------------------------------ the final exchange (8e) ---
@pytest.mark.parametrize("suf,logn,P,per,batch", [("f64", 20, 8, 1, 1), ("f32", 18, 8, 2, 3), ("f64", 16, 4, 1, 2),
                                                  ("f64", 12, 64, 16, 1)])
def test_allgather_bitwise_vs_host_scatter(suf, logn, P, per, batch):
    """pifft_allgather over the plans of a P-worker split (all on this GPU;
    hipMemcpyPeerAsync degenerates to a device copy) equals the host-side
    interleave of the same slices bit for bit, and the natural-order transform
    within tolerance."""
    n = 1 << logn
    x = oracle.generate(n * batch, DT[suf], seed=logn)
    d_in = dev(x)
    st = torch.cuda.current_stream()
    plans = [pifft.Plan(n, P, batch, PREC[suf], first=f, count=per, device=0) for f in range(0, P, per)]
    slices = [torch.empty(p.info.out_elems, dtype=d_in.dtype, device="cuda") for p in plans]
    for p, s in zip(plans, slices):
        p.execute_device(d_in.data_ptr(), s.data_ptr(), st)
    torch.cuda.synchronize()
    nat = torch.empty(n * batch, dtype=d_in.dtype, device="cuda")
    ms = pifft.allgather(plans, [s.data_ptr() for s in slices], [nat.data_ptr()] + [None] * (len(plans) - 1))
    assert ms > 0
    got = nat.cpu().numpy().reshape(batch, n)
    host = [s.cpu().numpy().reshape(batch, per, n // P) for s in slices]
    for bt in range(batch):
        sl = np.concatenate([h[bt] for h in host])  # (P, M), worker order
        assert got[bt].tobytes() == pifft_dist.interleave_slices(sl).tobytes()
        want = oracle.fft(x[bt * n:(bt + 1) * n], P=1, nthreads=8)
        assert_bins_close(got[bt], want, suf, n)
    # every destination gets the same result
    if len(plans) > 1:
        nat2 = torch.empty_like(nat)
        dests = [None] * len(plans)
        dests[-1] = nat2.data_ptr()
        pifft.allgather(plans, [s.data_ptr() for s in slices], dests)
        torch.cuda.synchronize()
        assert torch.equal(nat2, nat)


def test_allgather_every_destination_at_once():
    """Every plan a destination in ONE call (the 8-GPU line's pattern: each
    destination runs its own copy streams and interleave while the others
    still read the sources): all destinations bitwise equal to the
    one-destination result."""
    n, P = 1 << 16, 8
    x = oracle.generate(n, np.complex128, seed=7)
    d_in = dev(x)
    st = torch.cuda.current_stream()
    plans = [pifft.Plan(n, P, 1, pifft.F64, first=q, count=1, device=0) for q in range(P)]
    slices = [torch.empty(p.info.out_elems, dtype=d_in.dtype, device="cuda") for p in plans]
    for p, sl in zip(plans, slices):
        p.execute_device(d_in.data_ptr(), sl.data_ptr(), st)
    torch.cuda.synchronize()
    one = torch.empty(n, dtype=d_in.dtype, device="cuda")
    pifft.allgather(plans, [sl.data_ptr() for sl in slices], [one.data_ptr()] + [None] * (P - 1))
    nats = [torch.empty(n, dtype=d_in.dtype, device="cuda") for _ in range(P)]
    pifft.allgather(plans, [sl.data_ptr() for sl in slices], [t.data_ptr() for t in nats])
    torch.cuda.synchronize()
    for t in nats:
        assert torch.equal(t, one)


def test_allgather_rejects_aliased_destinations():
    """A destination overlapping a source (or another destination) is refused
    before any copy is queued."""
    n, P = 1 << 12, 4
    plans = [pifft.Plan(n, P, 1, pifft.F64, first=q, count=1, device=0) for q in range(P)]
    big = torch.zeros(2 * n, dtype=torch.complex128, device="cuda")
    bufs = [big[q * (n // P):(q + 1) * (n // P)] for q in range(P)]  # the slices: the first n of big
    nat = torch.empty(n, dtype=torch.complex128, device="cuda")
    with pytest.raises(pifft.PifftError, match="overlaps d_slices"):
        pifft.allgather(plans, [b.data_ptr() for b in bufs], [big[n // 2:].data_ptr(), None, None, None])
    with pytest.raises(pifft.PifftError, match="overlaps d_natural"):
        pifft.allgather(plans, [b.data_ptr() for b in bufs], [nat.data_ptr(), nat.data_ptr(), None, None])
    pifft.allgather(plans, [b.data_ptr() for b in bufs], [big[n:].data_ptr(), None, None, None])  # adjacent: fine


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="needs 2+ GPUs (multi-device placement)")
@pytest.mark.parametrize("suf", list(DT))
def test_allgather_plans_on_distinct_devices(suf):
    """Plan q on GPU q % device_count: the cross-device peer copies (xGMI) and
    the execute_group input broadcast give the single-device result bit for
    bit."""
    ndev = torch.cuda.device_count()
    n, P, batch = 1 << 16, 8, 2
    x = oracle.generate(n * batch, DT[suf], seed=5)
    multi = [pifft.Plan(n, P, batch, PREC[suf], first=q, count=1, device=q % ndev) for q in range(P)]
    single = [pifft.Plan(n, P, batch, PREC[suf], first=q, count=1, device=0) for q in range(P)]
    a = np.zeros(n * batch, dtype=DT[suf])
    b = np.zeros(n * batch, dtype=DT[suf])
    pifft.execute_group(multi, x, a)
    pifft.execute_group(single, x, b)
    assert a.tobytes() == b.tobytes()


def test_allgather_errors():
    n, P = 1 << 12, 4
    plans = [pifft.Plan(n, P, 1, pifft.F64, first=q, count=1, device=0) for q in range(P)]
    bufs = [torch.empty(n // P, dtype=torch.complex128, device="cuda") for _ in range(P)]
    nat = torch.empty(n, dtype=torch.complex128, device="cuda")
    with pytest.raises(pifft.PifftError, match="cover workers"):
        pifft.allgather(plans[:3], [b.data_ptr() for b in bufs[:3]], [nat.data_ptr(), None, None])
    with pytest.raises(pifft.PifftError, match="cover workers"):
        dup = [plans[0], plans[0], plans[2], plans[3]]
        pifft.allgather(dup, [b.data_ptr() for b in bufs], [nat.data_ptr(), None, None, None])
    whole = pifft.Plan(n, P, 1, pifft.F64)
    with pytest.raises(pifft.PifftError, match="slice-major"):
        pifft.allgather([whole], [bufs[0].data_ptr()], [nat.data_ptr()])
    other = pifft.Plan(n * 2, P, 1, pifft.F64, first=3, count=1, device=0)
    with pytest.raises(pifft.PifftError, match="share"):
        pifft.allgather(plans[:3] + [other], [b.data_ptr() for b in bufs], [nat.data_ptr(), None, None, None])


@pytest.mark.parametrize("site", ["enable_peer", "broadcast", "peer_copy", "peer_copy:3"])
def test_multi_gpu_error_paths_fail_cleanly(site, monkeypatch):
    """The multi-GPU error branches (peer access, the xGMI input broadcast of
    pifft_execute_group, the peer copies of pifft_allgather), reached on one
    GPU through the test-only fault switch (PIFFT_TUNING=1 PIFFT_FAULT=<site>):
    each call returns -1 with the message (CPU.c:102-109's -1 + message), holds
    no more device memory afterwards than before, and the next call on the
    same plans succeeds with the same bytes.  peer_copy:3 fails the third copy
    of the all-gather, after two copies were enqueued: the part-way cleanup
    (waiting for the copies in flight before returning) runs."""
    n, P, batch = 1 << 16, 8, 2
    x = oracle.generate(n * batch, np.complex128, seed=31)
    plans = [pifft.Plan(n, P, batch, pifft.F64, first=q, count=1, device=0) for q in range(P)]
    want = np.zeros(n * batch, np.complex128)
    pifft.execute_group(plans, x, want)  # allocates the staging and gather buffers and the copy streams
    st = torch.cuda.current_stream()
    d_in = dev(x)
    slices = [torch.empty(p.info.out_elems, dtype=d_in.dtype, device="cuda") for p in plans]
    for p, sl in zip(plans, slices):
        p.execute_device(d_in.data_ptr(), sl.data_ptr(), st)
    nat = torch.empty(n * batch, dtype=d_in.dtype, device="cuda")
    torch.cuda.synchronize()  # (pifft_allgather: once the executions that produced the slices have completed)
    pifft.allgather(plans, [sl.data_ptr() for sl in slices], [nat.data_ptr()] + [None] * (P - 1))
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(0)[0]
    monkeypatch.setenv("PIFFT_TUNING", "1")
    monkeypatch.setenv("PIFFT_FAULT", site)
    got = np.zeros(n * batch, np.complex128)
    with pytest.raises(pifft.PifftError, match="injected fault"):
        if site.startswith("peer_copy"):
            pifft.allgather(plans, [sl.data_ptr() for sl in slices], [nat.data_ptr()] + [None] * (P - 1))
        else:
            pifft.execute_group(plans, x, got)
    assert "injected fault" in pifft.last_error()
    if site == "peer_copy":  # the device gather inside execute_group fails the same way
        with pytest.raises(pifft.PifftError, match="injected fault"):
            pifft.execute_group(plans, x, got)
    torch.cuda.synchronize()
    assert torch.cuda.mem_get_info(0)[0] == free0
    monkeypatch.delenv("PIFFT_FAULT")
    pifft.execute_group(plans, x, got)
    assert got.tobytes() == want.tobytes()
    nat2 = torch.empty_like(nat)
    pifft.allgather(plans, [sl.data_ptr() for sl in slices], [nat2.data_ptr()] + [None] * (P - 1))
    torch.cuda.synchronize()
    assert torch.equal(nat2, nat) and nat.cpu().numpy().tobytes() == want.tobytes()


@pytest.mark.parametrize("suf", list(DT))
def test_execute_group_device_gather_equals_host_scatter(suf):
    """pifft_execute_group: a group holding all workers returns host_out via
    the device gather; the same plans run as partial groups scatter on the
    host.  Both paths give the same bytes (and the transform)."""
    n, P, batch = 1 << 16, 8, 2
    x = oracle.generate(n * batch, DT[suf], seed=99)
    plans = [pifft.Plan(n, P, batch, PREC[suf], first=q, count=1, device=0) for q in range(P)]
    a = np.zeros(n * batch, dtype=DT[suf])
    pifft.execute_group(plans, x, a)
    b = np.zeros(n * batch, dtype=DT[suf])
    pifft.execute_group(plans[:3], x, b)  # partial groups: host scatter
    pifft.execute_group(plans[3:], x, b)
    assert a.tobytes() == b.tobytes()
    for bt in range(batch):
        assert_bins_close(a[bt * n:(bt + 1) * n], oracle.fft(x[bt * n:(bt + 1) * n], P=1), suf, n)


def test_host_boundary_rejects_mismatched_buffers():
    """Plan.execute checks dtype, size, contiguity and writeability before any
    pointer crosses the ABI (a wrong buffer would be read/written out of
    bounds by the C side)."""
    n = 1024
    plan = pifft.Plan(n, 2, 1, pifft.F64)
    x = oracle.generate(n, np.complex128)
    with pytest.raises(pifft.PifftError, match="dtype"):
        plan.execute(x.astype(np.complex64), np.zeros(n, np.complex128))
    with pytest.raises(pifft.PifftError, match="dtype"):
        plan.execute(x, np.zeros(n, np.complex64))
    with pytest.raises(pifft.PifftError, match="holds"):
        plan.execute(x[: n // 2], np.zeros(n, np.complex128))
    with pytest.raises(pifft.PifftError, match="holds"):
        plan.execute(x, np.zeros(n // 2, np.complex128))
    with pytest.raises(pifft.PifftError, match="contiguous"):
        plan.execute(x, np.zeros(2 * n, np.complex128)[::2])
    ro = np.zeros(n, np.complex128)
    ro.setflags(write=False)
    with pytest.raises(pifft.PifftError, match="writeable"):
        plan.execute(x, ro)
    out = np.zeros(n, np.complex128)
    plan.execute(x, out)
    assert_bins_close(out, oracle.fft(x, P=2), "f64", n)


# -------------------------------------------------------------- 8(f) rows ---
def test_cli_lists_devices():
    """-l: the device query (the reference's how-many-concurrent-blocks /
    how_many_cores, gpu/cuda/how-many-concurrent-blocks.cu:65, CPU.c:835-837)."""
    r = _cli(["-l"])
    assert r.returncode == 0, r.stderr
    assert int(r.stdout.strip()) == pifft.gpu_count() >= 1


@pytest.mark.timeout(300)
def test_sweep_drives_the_mi355x_cli(tmp_path):
    """8(f) row 1 on the GPU: the reference's experiment loop (T x n x p ->
    5-column TSV, gpu/cuda/run-experiments:58-66) over the MI355X CLI, fed to
    both of the reference's analyses (analyze-results.R:35-71 regressions and
    the R-less analyze-results.awk)."""
    import pifft_sweep
    out = tmp_path / "mi355x.tsv"
    k = pifft_sweep.run_sweep(pifft.CLI_PATH, 2, 1 << 16, 1 << 20, 1, 8, str(out), extra=["-f", "64", "-s", "5"])
    d = pifft_sweep.load(str(out))
    assert k == len(d) == 2 * 5 * 4
    assert set(d[:, 0]) == {1 << e for e in range(16, 21)} and set(d[:, 1]) == {1, 2, 4, 8}
    assert np.all(d[:, 2] > 0) and np.allclose(d[:, 2], d[:, 3] + d[:, 4], atol=2e-3)
    assert np.all(d[d[:, 1] == 1][:, 3] == 0)  # P = 1: no tree stage
    res = pifft_sweep.analyze(d)
    assert np.all(np.isfinite(res["coef_time"])) and set(res["speedup"]) == set(int(v) for v in d[:, 0])
    txt = pifft_sweep.analyze_awk(out.read_text().splitlines(keepends=True))
    lines = txt.splitlines()
    assert lines[0].startswith("Empirical time complexity of pi-DFT on NVIDIA GPU (p=8, 2 replications)")
    assert [int(ln.split()[0]) for ln in lines[3:]] == [1 << e for e in range(16, 21)]


def test_concurrent_plans_from_host_threads():
    """The shim's threading contract (include/pifft.h; SURVEY.md 8(b)
    Threading, the reference's P pthreads, CPU.c:336-351): plans are
    independent objects.  Six host threads each create their own plan and
    stream and execute it 20 times concurrently (ctypes releases the GIL inside
    the calls); every result is bitwise the one-thread result.  A seventh
    thread keeps failing calls: pifft_last_error is per thread, so the workers
    never see its message."""
    import threading
    cases = [(16, 1, "f64", 1), (18, 8, "f64", 1), (17, 4, "f32", 2), (20, 2, "f64", 1), (15, 16, "f32", 3),
             (19, 1, "f32", 1)]
    xs, ref = [], []
    for logn, P, suf, b in cases:
        x = dev(oracle.generate((1 << logn) * b, DT[suf], seed=logn * 7 + P))
        p = pifft.Plan(1 << logn, P, b, PREC[suf])
        y = torch.empty(p.info.out_elems, dtype=x.dtype, device="cuda")
        p.execute_device(x.data_ptr(), y.data_ptr(), torch.cuda.current_stream())
        torch.cuda.synchronize()
        xs.append(x)
        ref.append(y.cpu())
        p.close()
    out = [None] * len(cases)
    errs = []
    stop = threading.Event()

    def worker(i):
        try:
            logn, P, suf, b = cases[i]
            p = pifft.Plan(1 << logn, P, b, PREC[suf])
            s = torch.cuda.Stream()
            y = torch.empty(p.info.out_elems, dtype=xs[i].dtype, device="cuda")
            with torch.cuda.stream(s):
                for _ in range(20):
                    p.execute_device(xs[i].data_ptr(), y.data_ptr(), s)
            s.synchronize()
            out[i] = (y.cpu(), pifft.last_error())
            p.close()
        except Exception as e:  # surfaced below
            errs.append(repr(e))

    def failer():
        p = pifft.Plan(1 << 10, 1, 1, pifft.F64)
        msgs = set()
        while not stop.is_set():
            assert pifft.lib().pifft_execute_device(p.handle, None, None, None) == -1
            msgs.add(pifft.last_error())
        out.append(msgs)
        p.close()

    tf = threading.Thread(target=failer)
    tf.start()
    ts = [threading.Thread(target=worker, args=(i,)) for i in range(len(cases))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    stop.set()
    tf.join()
    assert not errs, errs
    for i, (y, msg) in enumerate(out[:len(cases)]):
        assert torch.equal(y, ref[i]), f"case {cases[i]}: concurrent result differs"
        assert msg == "", f"case {cases[i]}: another thread's error leaked: {msg!r}"
    assert out[len(cases)] == {"NULL device buffer"}


@pytest.mark.parametrize("suf,logn,P,batch", [
    ("f64", 20, 8, 1), ("f64", 18, 2, 3), ("f64", 21, 16, 1), ("f32", 20, 8, 2), ("f64", 12, 4, 64),
    ("f32", 12, 8, 33), ("f64", 13, 8, 1), ("f32", 16, 4, 1), ("f64", 22, 8, 1), ("f64", 10, 2, 5)])
def test_natural_store_in_last_pass(suf, logn, P, batch, monkeypatch):
    """All-worker plans whose last pass stores natural order itself
    (PassArgs::ilv_log; PIFFT_ILV=1 forces it where the planner's size rule
    would not): bitwise equal to the slice-major store + interleave launch
    (PIFFT_ILV=0), and to the oracle -- multi-pass and single-pass local FFTs,
    batches, lines per transform below and above the tile's."""
    n = 1 << logn
    x = oracle.generate(n * batch, DT[suf], seed=logn * 3 + P + batch)
    monkeypatch.setenv("PIFFT_WORKER_IL", "0")  # the slice-major layout's natural store
    monkeypatch.setenv("PIFFT_ILV", "1")
    ilv = pifft.Plan(n, P, batch, PREC[suf])
    monkeypatch.setenv("PIFFT_ILV", "0")
    sep = pifft.Plan(n, P, batch, PREC[suf])
    assert "interleave" not in ilv.describe()["launch_kind"]
    assert sep.describe()["launch_kind"][-1] == "interleave"
    got = run(ilv, x)
    assert got.tobytes() == run(sep, x).tobytes()
    got = got.reshape(batch, n)
    for bt in sorted({0, batch - 1}):
        assert_bins_close(got[bt], oracle.fft(x[bt * n:(bt + 1) * n], P=P, nthreads=8), suf, n)


@pytest.mark.parametrize("suf,logn,P,first,count,batch,flags", [
    ("f64", 20, 1, 0, 1, 1, pifft.OUT_NATURAL),   # two passes: pass 1 writes W, pass 2 reads it
    ("f64", 22, 1, 0, 1, 1, pifft.OUT_NATURAL),   # three passes: W between passes 2 and 3
    ("f32", 24, 1, 0, 1, 1, pifft.OUT_NATURAL),
    ("f64", 18, 1, 0, 1, 3, pifft.OUT_NATURAL),   # batch: padded transform stride
    ("f64", 21, 8, 5, 1, 1, pifft.OUT_SLICES),    # fused tree pass writes W
    ("f64", 22, 4, 2, 2, 2, pifft.OUT_SLICES),    # worker range + batch
    ("f64", 20, 8, 0, 8, 1, pifft.OUT_NATURAL),   # tree + passes + natural store
    ("f64", 24, 16, 3, 1, 1, pifft.OUT_SLICES),   # worker of 16 (fused tree, multi-pass)
    ("f64", 20, 1, 0, 1, 1, pifft.OUT_BITREV),    # bit-reversed last pass reads W
])
@pytest.mark.parametrize("pad", [1040, 37])
def test_padded_workspace_rows(suf, logn, P, first, count, batch, flags, pad, monkeypatch):
    """Padded workspace rows forced onto small plans (PIFFT_W_PAD_MIN_MIB=0;
    by default only W beyond the Infinity Cache is padded): bitwise equal to
    the unpadded plan (PIFFT_W_PAD=0) and to the oracle, for every hand-off
    through W (first pass, later pass, fused tree pass, batches, worker
    ranges, bit-reversed output) and an odd pad."""
    n = 1 << logn
    x = oracle.generate(n * batch, DT[suf], seed=logn + 7 * P + batch)
    monkeypatch.setenv("PIFFT_WORKER_IL", "0")  # (worker-interleaved plans keep W unpadded)
    monkeypatch.setenv("PIFFT_W_PAD_MIN_MIB", "0")
    monkeypatch.setenv("PIFFT_W_PAD", str(pad))
    padded = pifft.Plan(n, P, batch, PREC[suf], first=first, count=count, flags=flags)
    monkeypatch.setenv("PIFFT_W_PAD", "0")
    plain = pifft.Plan(n, P, batch, PREC[suf], first=first, count=count, flags=flags)
    assert padded.describe()["workspace_bytes"] > plain.describe()["workspace_bytes"]
    got = run(padded, x)
    assert got.tobytes() == run(plain, x).tobytes()
    if flags == pifft.OUT_NATURAL:
        got = got.reshape(batch, n)
        assert_bins_close(got[-1], oracle.fft(x[(batch - 1) * n:], P=P, nthreads=8), suf, n)
