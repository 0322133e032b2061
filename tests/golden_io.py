"""Loaders for the committed golden fixtures (tests/golden/, made by gen_golden.py)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load_fft(suf, n):
    with np.load(os.path.join(GOLDEN, f"fft_{suf}_n{n}.npz"), allow_pickle=False) as z:
        return z["x"], z["X"]


def load_tree(suf, n, P):
    with np.load(os.path.join(GOLDEN, f"tree_{suf}_n{n}_p{P}.npz"), allow_pickle=False) as z:
        return z["x"], z["seg"]


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.complex128)
    b = np.asarray(b, dtype=np.complex128)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
