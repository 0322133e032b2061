"""tests/golden/gen_awk_golden.py -- fixtures for pifft_sweep.analyze_awk.

Runs in the build container only (it needs /root/reference): the reference's
own R-less analysis, `awk -f gpu/cuda/analyze-results.awk <results> | sort -n
-t 1` (the path gpu/cuda/analyze-results:27-34 takes), over
  * ref_cuda_results.tsv    the reference's committed CUDA results (data),
  * ref_xeonphi_results.tsv the reference's committed Xeon Phi results (data),
  * syn_results.tsv  a small file written here: few rows (the
    significance printed with %.2e), a repeated line (t[$0] keeps one), and
    p = 1..32 (the string-order choice of the reported p),
and stores each output as awk_<name>.txt.  The outputs are data; the awk
script itself is not copied.
Re-run:  python tests/golden/gen_awk_golden.py
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
AWK = "/root/reference/benchmark/fourier/parallel/pi/gpu/cuda/analyze-results.awk"


def synthetic() -> str:
    rows = []
    for t, noise in ((0, 1.00), (1, 1.31)):
        for n in (1024, 2048):
            for p in (1, 2, 4, 8, 16, 32):
                tr = 0.002 * n * (p - 1) / p
                cy = 0.0004 * (n / p) * max(1, (n // p).bit_length() - 1)
                f = noise if (n + p) % 3 else 1 / noise
                rows.append(f"{n}\t{p}\t{(tr + cy) * f:.6f}\t{tr:.6f}\t{cy * f:.6f}")
    rows.append(rows[3])  # an identical line: one regression row in the reference
    return "\n".join(rows) + "\n"


def main() -> None:
    syn = os.path.join(HERE, "syn_results.tsv")
    with open(syn, "w") as f:
        f.write(synthetic())
    for name in ("ref_cuda_results", "ref_xeonphi_results", "syn_results"):
        src = os.path.join(HERE, name + ".tsv")
        a = subprocess.run(["awk", "-f", AWK, src], capture_output=True, text=True, check=True).stdout
        s = subprocess.run(["sort", "-n", "-t", "1"], input=a, capture_output=True, text=True, check=True).stdout
        with open(os.path.join(HERE, f"awk_{name}.txt"), "w") as f:
            f.write(s)
        print(name, "->", f"awk_{name}.txt")


if __name__ == "__main__":
    main()
