"""§8(f) row 1: the sweep driver and cost-law analysis (pifft_sweep.py),
pinned on the reference's own published results file: analyze-results.R on
the Xeon Phi data printed "alpha < 1.759045e-07" (total fit) and "1e-120"
for both stage fits (xeonphi/openmp/...-results-analysis.out); the fixture
tests/golden/ref_xeonphi_results.tsv is that run's data file, copied as data."""
import os

import numpy as np
import pytest

import pifft_sweep
import pifft_oracle as oracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_reference_analysis_reproduced():
    res = pifft_sweep.analyze(pifft_sweep.load(os.path.join(GOLDEN, "ref_xeonphi_results.tsv")))
    assert f"{res['alpha']:.7g}" == "1.759045e-07"
    assert res["alpha_tr"] == 1e-120 and res["alpha_cy"] == 1e-120
    txt = pifft_sweep.report(res)
    assert "(Fit significant at the alpha < 1.759045e-07 level.)" in txt
    # 21.4x speedup at p=32 for n=131072 (Xeon Phi table)
    assert abs(res["speedup"][131072][32] - 21.4) < 0.1


def test_law_fit_recovers_coefficients():
    rng = np.random.default_rng(0)
    rows = []
    for n in (1 << 12, 1 << 14, 1 << 16):
        for p in (1, 2, 4, 8, 16):
            for _ in range(3):
                tr = 2e-4 * n * (p - 1) / p
                cy = 5e-4 * (n / p) * np.log2(n / p)
                rows.append([n, p, (tr + cy) * (1 + 1e-3 * rng.standard_normal()), tr, cy])
    res = pifft_sweep.analyze(np.array(rows))
    assert np.allclose(res["coef_time"], [2e-4, 5e-4], rtol=1e-2)
    assert abs(res["coef_time_tr"] - 2e-4) < 1e-9 and abs(res["coef_time_cy"] - 5e-4) < 1e-9


def test_run_sweep_with_reference_binary(tmp_path):
    exe = oracle.reference_binary(32)
    if not exe:
        pytest.fail("oracle/_ref not built (make -C oracle ref): the sweep check needs the reference binary")
    out = tmp_path / "r.tsv"
    k = pifft_sweep.run_sweep(exe, 2, 1024, 4096, 1, 4, str(out), max_p=os.cpu_count())
    d = pifft_sweep.load(str(out))
    assert k == len(d) == 2 * 3 * 3
    assert set(d[:, 0]) == {1024, 2048, 4096} and set(d[:, 1]) == {1, 2, 4}
    assert np.allclose(d[:, 2], d[:, 3] + d[:, 4], atol=1e-3)


@pytest.mark.parametrize("name", ["ref_cuda_results", "ref_xeonphi_results", "syn_results"])
def test_awk_limited_analysis_reproduced(name):
    """The reference's R-less analysis (gpu/cuda/analyze-results.awk piped
    through `sort -n -t 1`), text-identical to its output on the reference's
    committed CUDA and Xeon Phi results and on a synthetic file exercising its
    quirks (fixtures: tests/golden/gen_awk_golden.py)."""
    with open(os.path.join(GOLDEN, name + ".tsv")) as f:
        lines = f.readlines()
    with open(os.path.join(GOLDEN, f"awk_{name}.txt")) as f:
        want = f.read()
    assert pifft_sweep.analyze_awk(lines) == want


def test_reference_cuda_results_fit():
    """The reference's CUDA results file through the R-path regressions: its
    stage-1 and stage-2 times follow the law (the stage fits are significant)."""
    d = pifft_sweep.load(os.path.join(GOLDEN, "ref_cuda_results.tsv"))
    assert d.shape == (240, 5) and set(d[:, 0]) == {1024, 2048, 4096, 8192} and set(d[:, 1]) == {1, 2, 4, 8, 16, 32}
    res = pifft_sweep.analyze(d)
    assert res["alpha_tr"] < 1e-6 and res["alpha_cy"] < 1e-6
    assert res["speedup"][8192][32] > 10  # 102.8 -> 7.7 ms


def test_ols_exact_fit_and_no_dof_without_warnings():
    """lm(y ~ X - 1) on an exact fit: standard error 0, t = Inf, p = 0 (R's
    values), with no divide-by-zero warning; and no residual degrees of
    freedom: NaN standard errors."""
    import warnings
    import numpy as np
    X = np.array([[1.0], [0.0], [0.0]])
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        beta, se, tv, pv = pifft_sweep._ols_noint(X, np.array([3.0, 0.0, 0.0]))
        assert beta[0] == 3.0 and se[0] == 0.0 and np.isinf(tv[0]) and pv[0] == 0.0
        beta, se, tv, pv = pifft_sweep._ols_noint(X[:1], np.array([5.0]))
        assert beta[0] == pytest.approx(5.0) and np.isnan(se[0]) and np.isnan(pv[0])
