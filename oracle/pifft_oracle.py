"""oracle/pifft_oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes access to the C restatement of the reference pi-FFT
(oracle/pifft_oracle.c; reference file:line map there).  Imported only by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg -- the product
(libpifft.so) never routes through it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_pifft.so")
REF_DIR = os.path.join(HERE, "_ref")

_lib = None


def build(quiet: bool = True) -> None:
    """Compile liboracle_pifft.so (gcc, seconds)."""
    subprocess.run(["make", "-C", HERE, "liboracle_pifft.so"], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u64, u32, vp, dp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)
        for suf in ("f32", "f64"):
            f = getattr(L, f"oracle_fft_{suf}")
            f.argtypes = [vp, vp, u64, u32, u32, dp, dp, dp]
            f.restype = ctypes.c_int
            f = getattr(L, f"oracle_worker_{suf}")
            f.argtypes = [vp, vp, u64, u32, u32, dp, dp]
            f.restype = ctypes.c_int
            f = getattr(L, f"oracle_tree_segment_{suf}")
            f.argtypes = [vp, vp, u64, u32, u32]
            f.restype = ctypes.c_int
            f = getattr(L, f"oracle_generate_{suf}")
            f.argtypes = [vp, u64, u64, u64, u64]
            f.restype = None
        L.oracle_bit_reverse.argtypes = [u64, u32]
        L.oracle_bit_reverse.restype = u64
        L.oracle_splitmix64.argtypes = [u64, u64]
        L.oracle_splitmix64.restype = u64
        L.oracle_kat_f32.argtypes = [u32]
        L.oracle_kat_f32.restype = ctypes.c_int
        _lib = L
    return _lib


def _suf(dtype) -> str:
    dt = np.dtype(dtype)
    if dt == np.complex64:
        return "f32"
    if dt == np.complex128:
        return "f64"
    raise ValueError(f"unsupported dtype {dt}")


def generate(n: int, dtype, seed: int = 0x5EED, count: int | None = None, first: int = 0) -> np.ndarray:
    """Synthetic input: splitmix64(seed), re/im = (2u-1)/sqrt(n) (oracle_generate)."""
    count = n if count is None else count
    x = np.empty(count, dtype=dtype)
    getattr(lib(), f"oracle_generate_{_suf(dtype)}")(x.ctypes.data, count, n, seed, first)
    return x


def fft(x: np.ndarray, P: int = 1, nthreads: int = 0, timing: bool = False):
    """The reference transform (tree + cylinder + bit-reversed scatter), all P workers."""
    x = np.ascontiguousarray(x)
    n = x.shape[0]
    out = np.empty_like(x)
    t = [ctypes.c_double(0.0) for _ in range(3)]
    rc = getattr(lib(), f"oracle_fft_{_suf(x.dtype)}")(
        x.ctypes.data, out.ctypes.data, n, P, nthreads,
        ctypes.byref(t[0]), ctypes.byref(t[1]), ctypes.byref(t[2]))
    if rc:
        raise RuntimeError(f"oracle_fft failed rc={rc}")
    if timing:
        return out, (t[0].value, t[1].value, t[2].value)
    return out


def worker_bins(x: np.ndarray, P: int, q: int) -> np.ndarray:
    """Worker q's output written into a natural-order array (other bins zero)."""
    x = np.ascontiguousarray(x)
    out = np.zeros_like(x)
    rc = getattr(lib(), f"oracle_worker_{_suf(x.dtype)}")(x.ctypes.data, out.ctypes.data,
                                                          x.shape[0], P, q, None, None)
    if rc:
        raise RuntimeError("oracle_worker failed")
    return out


def tree_segment(x: np.ndarray, P: int, q: int) -> np.ndarray:
    """Worker q's N/P segment after the tree stage (reference tmp_in[q*N/P:...])."""
    x = np.ascontiguousarray(x)
    seg = np.empty(x.shape[0] // P, dtype=x.dtype)
    rc = getattr(lib(), f"oracle_tree_segment_{_suf(x.dtype)}")(x.ctypes.data, seg.ctypes.data,
                                                               x.shape[0], P, q)
    if rc:
        raise RuntimeError("oracle_tree_segment failed")
    return seg


def bit_reverse(x: int, m: int) -> int:
    return int(lib().oracle_bit_reverse(x, m))


def kat(P: int) -> bool:
    """The reference's N=8 known-answer test (CPU.c:251-260, 689-705)."""
    return lib().oracle_kat_f32(P) == 0


def reference_binary(prec: int) -> str | None:
    """Path of the reference CLI compiled from /root/reference (oracle/_ref), if built."""
    name = "fourier-parallel-pi-cpu-pthreads" + ("-f64" if prec == 64 else "")
    p = os.path.join(REF_DIR, name)
    return p if os.path.exists(p) else None


def run_reference_harness(mode: str, x: np.ndarray, P: int, q: int = 0) -> np.ndarray:
    """Run oracle/_ref/ref_harness_* (the reference compiled from its own source)."""
    suf = _suf(x.dtype)
    exe = os.path.join(REF_DIR, f"ref_harness_{suf}")
    if not os.path.exists(exe):
        raise FileNotFoundError(exe)
    n = x.shape[0]
    r = subprocess.run([exe, mode, str(n), str(P), str(q)], input=np.ascontiguousarray(x).tobytes(),
                       stdout=subprocess.PIPE, check=True)
    m = n if mode == "fft" else n // P
    return np.frombuffer(r.stdout, dtype=x.dtype, count=m).copy()
