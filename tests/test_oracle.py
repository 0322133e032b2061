"""Pins the CPU oracle (oracle/pifft_oracle.c) against the reference itself.

The fixtures in tests/golden/ are outputs of the reference CPU path compiled
from its own source (tests/golden/gen_golden.py); the oracle must reproduce
them BITWISE, for every worker count, in fp32 and fp64.  Runs on CPU.
"""
import hashlib

import numpy as np
import pytest

import pifft_oracle as oracle
from golden_io import load_fft, load_tree, manifest, rel_l2

SUFS = {"f32": np.complex64, "f64": np.complex128}


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("P", [1, 2, 4, 8])
def test_reference_known_answer(P):
    # CPU.c:251-260 input 0,1,0,1,... -> 4,0,0,0,-4,0,0,0 with float ==
    assert oracle.kat(P)


@pytest.mark.parametrize("suf", list(SUFS))
@pytest.mark.parametrize("n", [2, 4, 8, 16, 64, 1024, 4096])
def test_oracle_bitwise_vs_reference(suf, n):
    x, X = load_fft(suf, n)
    for P in (1, 2, 4, 8, n):
        if P > n:
            continue
        got = oracle.fft(x, P=P)
        assert got.tobytes() == X.tobytes(), f"P={P}"


@pytest.mark.parametrize("suf", list(SUFS))
@pytest.mark.parametrize("n,P", [(64, 8), (64, 2), (1024, 4), (4096, 16), (256, 256)])
def test_oracle_tree_segments_bitwise(suf, n, P):
    x, segs = load_tree(suf, n, P)
    for q in range(P):
        assert oracle.tree_segment(x, P, q).tobytes() == segs[q].tobytes(), f"q={q}"


@pytest.mark.parametrize("suf", list(SUFS))
def test_generator_matches_fixtures(suf):
    m = manifest()
    for n in (8, 1024, 4096):
        x, _ = load_fft(suf, n)
        g = oracle.generate(n, SUFS[suf], m["seed"])
        assert g.tobytes() == x.tobytes()


def test_generator_numpy_restatement():
    # splitmix64 restated in numpy; the device generator follows the same formula
    n, seed = 257, 0x5EED
    d = np.arange(2 * n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (d + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    v = (2.0 * u - 1.0) / np.sqrt(float(n))
    want = (v[0::2] + 1j * v[1::2]).astype(np.complex128)
    assert oracle.generate(n, np.complex128, seed).tobytes() == want.tobytes()


@pytest.mark.parametrize("suf", list(SUFS))
def test_oracle_big_digest(suf):
    """N=2^20: oracle output digest == the reference's (P=1 and P=8)."""
    big = manifest()["big"][suf]
    x = oracle.generate(big["n"], SUFS[suf], manifest()["seed"])
    assert _sha(x) == big["sha256_x"]
    for P in (1, 8):
        assert _sha(oracle.fft(x, P=P, nthreads=8)) == big[f"sha256_X_p{P}"]


@pytest.mark.parametrize("suf,tol", [("f32", 3e-7), ("f64", 2e-15)])
def test_oracle_is_the_dft(suf, tol):
    x = oracle.generate(4096, SUFS[suf])
    X = oracle.fft(x, P=4)
    assert rel_l2(X, np.fft.fft(x.astype(np.complex128))) < tol


def test_worker_owns_stride_p_bins():
    """Worker q owns natural-order bins bitrev_log2P(q) + P*k."""
    n, P = 256, 8
    x = oracle.generate(n, np.complex128)
    full = oracle.fft(x, P=P)
    for q in range(P):
        part = oracle.worker_bins(x, P, q)
        r = oracle.bit_reverse(q, 3)
        mask = np.zeros(n, bool)
        mask[r::P] = True
        assert np.array_equal(part[mask], full[mask])
        assert not np.any(part[~mask])


@pytest.mark.parametrize("suf", list(SUFS))
def test_oracle_tree_big_digests(suf):
    """Post-tree segments at N=2^16..2^20, every worker, == the reference's
    (SHA-256 per worker, manifest["tree_big"]).  At these sizes glibc's sincos
    (what gcc -O2 makes of the reference's cos/sin pair, CPU.c:647-648) and a
    separate cos/sin differ on hundreds of fp64 twiddles, so this pins the
    oracle's omega to the -O2 reference build."""
    for key, case in manifest()["tree_big"].items():
        if not key.startswith(suf):
            continue
        x = oracle.generate(case["n"], SUFS[suf], manifest()["seed"])
        for q, want in enumerate(case["sha256_seg_q"]):
            assert _sha(oracle.tree_segment(x, case["P"], q)) == want, f"{key} q={q}"
