"""tests/golden/gen_golden.py -- generates the committed golden fixtures.

Runs in the build container only (it needs /root/reference): `make -C oracle ref`
compiles the reference CPU path from its own source into oracle/_ref/, and this
script feeds it synthetic inputs (splitmix64, oracle.generate) and stores

  fft_{f32,f64}_n{N}.npz   input x and the reference output X (natural order,
                           all workers in test mode) -- verified bitwise
                           identical for every P in {1,2,4,8} (P <= N)
  tree_{f32,f64}_n{N}_p{P}.npz  every worker's segment after the tree stage
  manifest.json            sizes, seeds, SHA-256 of the reference outputs
                           (incl. N=2^20 for P=1 and P=8), rel-L2 vs a float64
                           numpy FFT, and per-worker SHA-256 of the post-tree
                           segments at N=2^16..2^20 ("tree_big": sizes where
                           glibc's sincos -- what gcc -O2 makes of the
                           reference's cos/sin pair -- and separate cos/sin
                           differ on hundreds of fp64 twiddles)

The fixtures are data (inputs and reference outputs), never reference source.
Re-run:  python tests/golden/gen_golden.py            (everything)
         python tests/golden/gen_golden.py tree-big   (only manifest["tree_big"])
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pifft_oracle as oracle  # noqa: E402

SEED = 0x5EED
FFT_SIZES = [2, 4, 8, 16, 64, 1024, 4096]
TREE_CASES = [(64, 8), (64, 2), (1024, 4), (4096, 16), (256, 256)]
BIG = 1 << 20
TREE_BIG = [(1 << 16, 8), (1 << 18, 16), (1 << 20, 4)]
DT = {"f32": np.complex64, "f64": np.complex128}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def rel_l2(a, b) -> float:
    a = a.astype(np.complex128)
    b = b.astype(np.complex128)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def tree_big() -> dict:
    out = {}
    for suf, dt in DT.items():
        for n, P in TREE_BIG:
            x = oracle.generate(n, dt, SEED)
            out[f"{suf}_n{n}_p{P}"] = {
                "n": n, "P": P,
                "sha256_seg_q": [sha(oracle.run_reference_harness("tree", x, P, q)) for q in range(P)]}
    return out


def main() -> None:
    if sys.argv[1:] == ["tree-big"]:
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "all", "ref"], check=True,
                       stdout=subprocess.DEVNULL)
        with open(os.path.join(HERE, "manifest.json")) as f:
            man = json.load(f)
        man["tree_big"] = tree_big()
        with open(os.path.join(HERE, "manifest.json"), "w") as f:
            json.dump(man, f, indent=1, sort_keys=True)
        return
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "all", "ref"], check=True,
                   stdout=subprocess.DEVNULL)
    man = {"seed": SEED, "generator": "splitmix64; re,im=(2u-1)/sqrt(N), u=(z>>11)*2^-53, draws 2e,2e+1",
           "fft": {}, "tree": {}, "big": {}}
    for suf, dt in DT.items():
        for n in FFT_SIZES:
            x = oracle.generate(n, dt, SEED)
            outs = {}
            for P in (1, 2, 4, 8):
                if P > n:
                    continue
                outs[P] = oracle.run_reference_harness("fft", x, P)
            ref = outs[1]
            for P, o in outs.items():
                assert o.tobytes() == ref.tobytes(), f"reference not P-invariant {suf} n={n} P={P}"
            np.savez(os.path.join(HERE, f"fft_{suf}_n{n}.npz"), x=x, X=ref)
            man["fft"][f"{suf}_n{n}"] = {
                "n": n, "P_checked": sorted(outs), "sha256_X": sha(ref), "sha256_x": sha(x),
                "rel_l2_vs_numpy_f64": rel_l2(ref, np.fft.fft(x.astype(np.complex128)))}
        for n, P in TREE_CASES:
            x = oracle.generate(n, dt, SEED)
            segs = np.stack([oracle.run_reference_harness("tree", x, P, q) for q in range(P)])
            np.savez(os.path.join(HERE, f"tree_{suf}_n{n}_p{P}.npz"), x=x, seg=segs)
            man["tree"][f"{suf}_n{n}_p{P}"] = {"n": n, "P": P, "sha256_seg": sha(segs)}
        # N = 2^20: digests only (16 MiB outputs are not committed)
        x = oracle.generate(BIG, dt, SEED)
        big = {"n": BIG, "sha256_x": sha(x)}
        for P in (1, 8):
            o = oracle.run_reference_harness("fft", x, P)
            big[f"sha256_X_p{P}"] = sha(o)
            if P == 1:
                big["rel_l2_vs_numpy_f64"] = rel_l2(o, np.fft.fft(x.astype(np.complex128)))
        man["big"][suf] = big
        print(suf, "done", flush=True)
    man["tree_big"] = tree_big()
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
