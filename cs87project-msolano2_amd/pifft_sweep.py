"""pifft_sweep.py -- the reference's experiment sweep and cost-law analysis
(SURVEY.md section 8(f), row 1), for the MI355X CLI or any binary with the
reference's `-n <n> -p <p> -o` interface and 5-column TSV output.

  run     : T replications x n (doubling) x p (doubling) -> TSV lines
            "n p time time_tr time_cy" appended to a results file
            (benchmark/fourier/parallel/pi/cpu/pthreads/
             run-experiments-and-analyze-results:27-69; cuda/run-experiments:15-73)
  analyze : the regressions of analyze-results.R:31-71 -- no-intercept least
            squares of time ~ n(p-1)/p + (n/p)log2(n/p), time_tr ~ n(p-1)/p,
            time_cy ~ (n/p)log2(n/p) -- and the printout of :40-71, plus the
            empirical speedup table of :74-83.  Plots are not reproduced.
  awk     : the reference's R-less "limited analysis" (gpu/cuda/
            analyze-results.awk), text output identical (analyze_awk)

Quirk kept on purpose: for the two-regressor fit the reference reports
max(coef(summary(lm))[4], 1e-120), which in R's column-major indexing is the
STANDARD ERROR of the (n/p)log2(n/p) coefficient, not a p-value; for the
one-regressor fits [4] is the p-value.  `analyze` reports the same numbers
(pinned by tests/test_sweep.py on the reference's own Xeon Phi results file,
whose published analysis says alpha < 1.759045e-07).

usage:
  python pifft_sweep.py run --bin ./pifft --T 2 --n-from 1048576 --n-to 16777216 \
         --p-from 1 --p-to 8 --out results.tsv [-- extra args, e.g. -f 64]
  python pifft_sweep.py analyze results.tsv
"""
from __future__ import annotations

import argparse
import math
import subprocess
import sys

import numpy as np


def law_tree(n, p):
    return n * (p - 1) / p


def law_cyl(n, p):
    return (n / p) * np.log2(n / p)


def run_sweep(binary: str, T: int, n_from: int, n_to: int, p_from: int, p_to: int, out: str,
              extra: list[str] | None = None, max_p: int | None = None) -> int:
    """Append one TSV line per run (the reference's loop order: t, n, p)."""
    lines = 0
    with open(out, "a") as f:
        for _ in range(T):
            n = n_from
            while n <= n_to:
                p = p_from
                while p <= p_to:
                    if max_p is None or p <= max_p:
                        r = subprocess.run([binary, "-n", str(n), "-p", str(p), "-o"] + (extra or []),
                                           capture_output=True, text=True, check=True)
                        row = r.stdout.strip().splitlines()[-1]
                        if len(row.split("\t")) < 5:
                            raise RuntimeError(f"unexpected output: {row!r}")
                        f.write("\t".join(row.split("\t")[:5]) + "\n")
                        lines += 1
                    p *= 2
                n *= 2
    return lines


def load(path: str) -> np.ndarray:
    """The reference's read.table(sep='\\t', col.names=n,p,time,time_tr,time_cy)."""
    d = np.loadtxt(path, ndmin=2)
    if d.shape[1] < 5:
        raise ValueError("expected 5 tab-separated columns")
    return d[:, :5]


def _ols_noint(X: np.ndarray, y: np.ndarray):
    """lm(y ~ X - 1): coefficients, standard errors, t values, two-sided p-values."""
    from scipy import stats
    beta, *_ = np.linalg.lstsq(X, y, rcond=None)
    r = y - X @ beta
    dof = len(y) - X.shape[1]
    if dof <= 0:  # R: NaN standard errors (no residual degrees of freedom)
        nan = np.full_like(beta, np.nan)
        return beta, nan, nan, nan
    s2 = float(r @ r) / dof
    se = np.sqrt(np.diag(s2 * np.linalg.inv(X.T @ X)))
    # an exact fit (se == 0): R reports t = +-Inf (p = 0), or NaN for a zero
    # coefficient -- without numpy's divide-by-zero warning
    with np.errstate(divide="ignore", invalid="ignore"):
        tv = beta / se
    pv = 2.0 * stats.t.sf(np.abs(tv), dof)
    return beta, se, tv, pv


def _coef4(beta, se, tv, pv) -> float:
    """coef(summary(lm))[4] with R's column-major indexing (see module doc)."""
    m = np.column_stack([beta, se, tv, pv])  # rows: coefficients
    return float(m.flatten(order="F")[3])


def analyze(d: np.ndarray) -> dict:
    n, p, t, ttr, tcy = d.T
    x_tr, x_cy = law_tree(n, p), law_cyl(n, p)
    fit = _ols_noint(np.column_stack([x_tr, x_cy]), t)
    fit_tr = _ols_noint(x_tr[:, None], ttr)
    fit_cy = _ols_noint(x_cy[:, None], tcy)
    res = {
        "coef_time": fit[0].tolist(),
        "alpha": max(_coef4(*fit), 1e-120),
        "coef_time_tr": float(fit_tr[0][0]),
        "alpha_tr": max(_coef4(*fit_tr), 1e-120),
        "coef_time_cy": float(fit_cy[0][0]),
        "alpha_cy": max(_coef4(*fit_cy), 1e-120),
    }
    # empirical speedup vs the smallest p, averaged over replications (analyze-results.R:74-83)
    speed = {}
    for ni in sorted(set(n)):
        pmin = p[n == ni].min()
        base = t[(n == ni) & (p == pmin)].mean()
        speed[int(ni)] = {int(pi): float(base / t[(n == ni) & (p == pi)].mean()) for pi in sorted(set(p[n == ni]))}
    res["speedup"] = speed
    return res


def _awk_num(x: float) -> str:
    """awk's default number-to-string conversion of an array subscript
    (integral values print as integers, others with CONVFMT %.6g)."""
    return str(int(x)) if float(x).is_integer() else f"{x:.6g}"


def analyze_awk(lines: list[str]) -> str:
    """The reference's "limited analysis" (the path analyze-results takes when
    R is absent): `awk -f analyze-results.awk results.csv | sort -n -t 1`
    (benchmark/fourier/parallel/pi/gpu/cuda/analyze-results.awk:15-66,
    analyze-results:27-34), restated with its quirks:
      * rows are keyed by the whole input line (t[$0]), so identical lines
        count once in the regression;
      * the reported p is the largest p in STRING order (awk compares the
        array subscripts as strings: "8" > "4" > "32" > "2" > "16" > "1");
      * beta = sum(t law) / sum(law^2) for the combined law n(p-1)/p +
        (n/p)log2(n/p); SS_tot is taken about the law's mean and SS_prd about
        an uninitialised variable (0);
      * the significance is a t-density expression, printed as 1.0e<k> with an
        order-of-magnitude estimate below 1e-15 (floored at 1.0e-120);
      * `sort -n -t 1` puts the text lines (numeric value 0, byte order) before
        the table rows (ascending n)."""
    n_obs, p_obs, t_sum, t, t_law = {}, {}, {}, {}, {}
    nr = 0

    def law(n, p):
        return n * ((p - 1) / p) + (n / p) * (math.log(n / p) / math.log(2))

    for ln in lines:
        f = ln.split()
        if not f:
            continue
        nr += 1
        n, p, tm = float(f[0]), float(f[1]), float(f[2])
        kn, kp = _awk_num(n), _awk_num(p)
        n_obs[kn], p_obs[kp] = n, p
        t_sum[(kn, kp)] = t_sum.get((kn, kp), 0.0) + tm
        key = ln.rstrip("\n")
        t[key], t_law[key] = tm, law(n, p)
    K = nr / (len(n_obs) * len(p_obs))
    at_a = sum(t_law[i] * t_law[i] for i in t)
    at_b = sum(t[i] * t_law[i] for i in t)
    beta = at_b / at_a
    N = len(t)
    t_law_m = sum(t_law.values()) / N
    ss_res = sum((t[i] - beta * t_law[i]) ** 2 for i in t)
    ss_prd = sum((t_law[i] - 0.0) ** 2 for i in t)
    eta = N - 2
    t_score = beta * math.sqrt(eta) / math.sqrt(ss_res / ss_prd)
    a = 1 / math.sqrt(eta)
    if eta % 2 == 0:
        a /= 2
        e = eta - 1
        while e > 2:
            a *= e / (e - 1)
            e -= 2
    else:
        a /= math.atan2(0, -1)
        e = eta - 1
        while e > 1:
            a *= e / (e - 1)
            e -= 2
    try:
        a /= math.sqrt(1 + t_score ** 2 / eta) ** eta
    except OverflowError:  # awk's ^ overflows to inf, and a / inf = 0
        a = 0.0
    pi = max(p_obs, key=lambda k: k)  # string order
    out = [f"Empirical time complexity of pi-DFT on NVIDIA GPU (p={int(float(pi))}, {int(K)} replications):"]
    if a < 1e-15:
        a_exp = int(42.480516 - 1.216025 * t_score - 1.366767 * eta)
        out.append(f"Fit significant at the alpha < 1.0e{max(a_exp, -120)} level.")
    else:
        out.append(f"Fit significant at the alpha < {a:.2e} level.")
    out.append("Input size (n)\tAvg. time (ms)\tTheta(n(p-1)/p + (n/p)log(n/p))")
    for kn, n in n_obs.items():
        out.append("%u\t\t%.2f\t\t%.2f" % (int(n), t_sum.get((kn, pi), 0.0) / K, beta * law(n, p_obs[pi])))

    def sort_key(line):
        import re
        m = re.match(r"\s*[-+]?\d+(\.\d*)?", line)
        return (float(m.group(0)) if m else 0.0, line.encode())
    return "\n".join(sorted(out, key=sort_key)) + "\n"


def report(res: dict) -> str:
    out = []
    out.append("  Testing the hypothesis that the parallel time complexity follows the law\n"
               "  [Funnel stage] + [Tube stage] = Theta([n((p-1)/p)] + [(n/p)*log(n/p)])...")
    out.append(("    Yes: " if res["alpha"] < 0.1 else "    No: ") +
               "the time complexity of pi-DFT is Theta([n((p-1)/p)]+[(n/p)*log(n/p)])")
    out.append(f"    (Fit significant at the alpha < {res['alpha']:.7g} level.)")
    out.append("  Testing the hypothesis that the 1st (funnel) stage is Theta(n((p-1)/p))...")
    out.append(("    Yes: " if res["alpha_tr"] < 0.1 else "    No: ") +
               "the time complexity of the 1st stage of pi-DFT is Theta(n((p-1)/p)).")
    out.append(f"    (Fit significant at the alpha < {res['alpha_tr']:.7g} level.)")
    out.append("  Testing the hypothesis that the 2nd (tube) stage is Theta((n/p)*log(n/p))...")
    out.append(("    Yes: " if res["alpha_cy"] < 0.1 else "    No: ") +
               "the time complexity of the 2nd stage of pi-DFT is Theta((n/p)*log(n/p))")
    out.append(f"    (Fit significant at the alpha < {res['alpha_cy']:.7g} level.)")
    out.append("  Empirical speedup (vs smallest p):")
    for ni, row in res["speedup"].items():
        out.append(f"    n={ni}: " + "  ".join(f"p={pi}:{s:.2f}x" for pi, s in row.items()))
    return "\n".join(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("run")
    r.add_argument("--bin", required=True)
    r.add_argument("--T", type=int, default=2)
    r.add_argument("--n-from", type=int, required=True)
    r.add_argument("--n-to", type=int, required=True)
    r.add_argument("--p-from", type=int, default=1)
    r.add_argument("--p-to", type=int, default=8)
    r.add_argument("--max-p", type=int, default=None)
    r.add_argument("--out", required=True)
    r.add_argument("extra", nargs="*")
    a = sub.add_parser("analyze")
    a.add_argument("results")
    w = sub.add_parser("awk")
    w.add_argument("results")
    args = ap.parse_args(argv)
    if args.cmd == "awk":
        with open(args.results) as f:
            sys.stdout.write(analyze_awk(f.readlines()))
        return 0
    if args.cmd == "run":
        if args.T <= 0:
            print("Invalid number of replications!")
            return 1
        k = run_sweep(args.bin, args.T, args.n_from, args.n_to, args.p_from, args.p_to, args.out, args.extra,
                      args.max_p)
        print(f"Done. {k} results appended to {args.out}")
        return 0
    print(report(analyze(load(args.results))))
    return 0


if __name__ == "__main__":
    sys.exit(main())
