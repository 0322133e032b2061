"""pifft.py -- Python (ctypes) view of libpifft.so, the MI355X pi-FFT C-ABI.

Mirrors include/pifft.h one to one; used by bench.py, tests/ and
__graft_entry__.  There is no fallback: if libpifft.so is missing or a call
fails, a PifftError is raised with the library's own message (the reference
prints its errors and exits non-zero, CPU.c:102-109).

Device buffers are plain integer addresses (e.g. torch.Tensor.data_ptr()) and
streams are raw hipStream_t handles (torch.cuda.Stream.cuda_stream) or None.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PIFFT_LIB") or os.path.join(HERE, "libpifft.so")  # PIFFT_LIB: tuning variants
CLI_PATH = os.path.join(HERE, "pifft")

F32, F64 = 32, 64
OUT_NATURAL, OUT_SLICES, OUT_BITREV = 0, 1, 2
PROFILE_ALL, PROFILE_SAMPLED = 0, 1
SEPARATE_TREE = 4  # flag bit: the tree never fused into the first pass (CLI -u)
KIND_NAMES = {1: "tree", 2: "pass", 3: "interleave", 4: "tree+pass"}
MAX_LAUNCH_INFO = 256  # PIFFT_MAX_LAUNCH_INFO (include/pifft.h)


class PifftError(RuntimeError):
    pass


class PlanInfo(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint64),
        ("workers", ctypes.c_uint32),
        ("first_worker", ctypes.c_uint32),
        ("num_workers", ctypes.c_uint32),
        ("batch", ctypes.c_uint32),
        ("prec", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("local_n", ctypes.c_uint64),
        ("in_elems", ctypes.c_uint64),
        ("out_elems", ctypes.c_uint64),
        ("workspace_bytes", ctypes.c_uint64),
        ("num_launches", ctypes.c_int32),
        ("num_passes", ctypes.c_int32),
        ("tree_launches", ctypes.c_int32),
        ("radix", ctypes.c_int32 * 8),
        ("lines", ctypes.c_int32 * 8),
        ("launch_bytes", ctypes.c_uint64 * MAX_LAUNCH_INFO),
        ("launch_kind", ctypes.c_int32 * MAX_LAUNCH_INFO),
        ("launch_fn", ctypes.c_int32 * MAX_LAUNCH_INFO),
        ("vpt", ctypes.c_int32 * 8),
        ("launch_mode", ctypes.c_int32 * MAX_LAUNCH_INFO),
        ("layout", ctypes.c_int32),
    ]


ABI_VERSION = 3  # include/pifft.h PIFFT_ABI_VERSION: the pifft_plan_info layout PlanInfo mirrors

# every symbol include/pifft.h declares, with its ctypes signature
_P = ctypes.c_void_p
_SIGS = {
    "pifft_last_error": (ctypes.c_char_p, []),
    "pifft_abi_version": (ctypes.c_int, []),
    "pifft_gpu_count": (ctypes.c_int, []),
    "pifft_plan_create": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_uint64, ctypes.c_uint32,
                                         ctypes.c_uint32, ctypes.c_int]),
    "pifft_plan_create_slices": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_uint64, ctypes.c_uint32,
                                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                ctypes.c_int, ctypes.c_int, ctypes.c_int]),
    "pifft_plan_destroy": (None, [_P]),
    "pifft_plan_dry_run": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.POINTER(PlanInfo)]),
    "pifft_plan_get_info": (ctypes.c_int, [_P, ctypes.POINTER(PlanInfo)]),
    "pifft_plan_kernel_name": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]),
    "pifft_execute_device": (ctypes.c_int, [_P, _P, _P, _P]),
    "pifft_execute_device_timed": (ctypes.c_int, [_P, _P, _P, _P, ctypes.POINTER(ctypes.c_float),
                                                  ctypes.c_int]),
    "pifft_execute": (ctypes.c_int, [_P, _P, _P, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double)]),
    "pifft_execute_group_kernel_times": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int,
                                                        ctypes.POINTER(ctypes.c_double),
                                                        ctypes.POINTER(ctypes.c_double)]),
    "pifft_execute_group": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, _P, _P,
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "pifft_generate_device": (ctypes.c_int, [_P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_int, _P]),
    "pifft_interleave_device": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.c_int, _P]),
    "pifft_tree_device": (ctypes.c_int, [_P, _P, _P, _P]),
    "pifft_profile_start": (ctypes.c_int, [_P, ctypes.c_int, ctypes.c_int]),
    "pifft_plan_tune_workspace": (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]),
    "pifft_profile_read": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int),
                                          ctypes.c_int]),
    "pifft_launch_loop": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_int, _P, _P, _P,
                                         ctypes.POINTER(ctypes.c_float)]),
    "pifft_allgather": (ctypes.c_int, [ctypes.POINTER(_P), ctypes.c_int, ctypes.POINTER(_P), ctypes.POINTER(_P),
                                       ctypes.POINTER(ctypes.c_double)]),
    "pifft_instance_count": (ctypes.c_int, []),
    "pifft_instance_desc": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_int32)]),
    "pifft_instance_found": (ctypes.c_int, [ctypes.c_int]),
    "pifft_plan_dry_run_instances": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                                    ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                                    ctypes.POINTER(ctypes.c_int32), ctypes.c_int]),
}
SYMBOLS = tuple(_SIGS)

_lib = None


def build(quiet: bool = True) -> None:
    """hipcc --offload-arch=gfx950 -> libpifft.so, gcc -> the pifft CLI (in-tree)."""
    subprocess.run(["make", "-j8", "-C", HERE, "all"], check=True,
                   stdout=subprocess.DEVNULL if quiet else None)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PifftError(f"{LIB_PATH} not built (run __graft_entry__.build() or make -C {HERE})")
        # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7;
        # loading torch first makes libpifft.so bind to that same runtime (its
        # NEEDED soname resolves to the already-loaded library).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        # PlanInfo above mirrors this layout version of pifft_plan_info
        if L.pifft_abi_version() != ABI_VERSION:
            raise PifftError(f"{LIB_PATH}: ABI version {L.pifft_abi_version()}, this binding expects {ABI_VERSION} "
                             f"(include/pifft.h PIFFT_ABI_VERSION; rebuild)")
        _lib = L
    return _lib


def last_error() -> str:
    return lib().pifft_last_error().decode()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise PifftError(f"{what}: {last_error()}")


def gpu_count() -> int:
    n = lib().pifft_gpu_count()
    if n < 0:
        raise PifftError(last_error())
    return n


def _stream(stream):
    if stream is None:
        return None
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    return int(stream)


class Plan:
    """One GPU's share of an N-point, P-worker pi-FFT (pifft_plan)."""

    def __init__(self, n: int, workers: int = 1, batch: int = 1, prec: int = F64, *,
                 first: int = 0, count: int | None = None, device: int | None = None,
                 flags: int | None = None):
        h = _P()
        if count is None and device is None and flags is None and first == 0:
            _check(lib().pifft_plan_create(ctypes.byref(h), n, workers, batch, prec), "pifft_plan_create")
        else:
            count = workers if count is None else count
            device = 0 if device is None else device
            if flags is None:
                flags = OUT_NATURAL if count == workers else OUT_SLICES
            elif flags == SEPARATE_TREE:
                flags |= OUT_NATURAL if count == workers else OUT_SLICES
            _check(lib().pifft_plan_create_slices(ctypes.byref(h), n, workers, first, count, batch, prec,
                                                  device, flags), "pifft_plan_create_slices")
        self._h = h
        self.info = self._info()

    def _info(self) -> PlanInfo:
        info = PlanInfo()
        _check(lib().pifft_plan_get_info(self._h, ctypes.byref(info)), "pifft_plan_get_info")
        return info

    @property
    def handle(self):
        return self._h

    def describe(self) -> dict:
        return describe_info(self.info)

    def kernel_name(self, launch: int) -> str:
        """Demangled kernel function of one launch (as rocprofv3 names it)."""
        buf = ctypes.create_string_buffer(512)
        _check(lib().pifft_plan_kernel_name(self._h, launch, buf, len(buf)), "pifft_plan_kernel_name")
        return buf.value.decode()

    def execute_device(self, d_in: int, d_out: int, stream=None) -> None:
        _check(lib().pifft_execute_device(self._h, d_in, d_out, _stream(stream)), "pifft_execute_device")

    def execute_device_timed(self, d_in: int, d_out: int, stream=None) -> list[float]:
        n = self.info.num_launches
        buf = (ctypes.c_float * max(n, 1))()
        _check(lib().pifft_execute_device_timed(self._h, d_in, d_out, _stream(stream), buf, n),
               "pifft_execute_device_timed")
        return list(buf[:n])

    def tune_workspace(self, d_in: int, d_out: int, stream=None, tries: int = 4) -> float:
        """pifft_plan_tune_workspace: keep the fastest of `tries` workspace
        placements for this (d_in, d_out); returns its mean execution ms."""
        ms = ctypes.c_float()
        _check(lib().pifft_plan_tune_workspace(self._h, d_in, d_out, _stream(stream), tries, ctypes.byref(ms)),
               "pifft_plan_tune_workspace")
        return ms.value

    def profile_start(self, steps: int, mode: int = 1) -> None:
        """mode PROFILE_SAMPLED (default; in-context) or PROFILE_ALL (isolated)."""
        _check(lib().pifft_profile_start(self._h, steps, mode), "pifft_profile_start")

    def profile_read(self) -> tuple[int, list[float], list[int]]:
        """(executions recorded, per-launch ms summed over its samples, samples per launch)."""
        n = self.info.num_launches
        buf = (ctypes.c_float * max(n, 1))()
        cnt = (ctypes.c_int * max(n, 1))()
        used = lib().pifft_profile_read(self._h, buf, cnt, n)
        if used < 0:
            raise PifftError(f"pifft_profile_read: {last_error()}")
        return used, list(buf[:n]), list(cnt[:n])

    def launch_loop(self, launches, reps: int, d_in: int, d_out: int, stream=None) -> float:
        """pifft_launch_loop: mean ms of the given launches run alone, back to
        back, `reps` rounds (d_out holds the plan's result afterwards)."""
        ls = (ctypes.c_int * len(launches))(*launches)
        ms = ctypes.c_float()
        _check(lib().pifft_launch_loop(self._h, ls, len(launches), reps, d_in, d_out, _stream(stream),
                                       ctypes.byref(ms)), "pifft_launch_loop")
        return ms.value

    def execute(self, host_in, host_out=None):
        """numpy in -> natural-order numpy out (only this plan's bins written)."""
        host_in, out_ptr = _host_buffers([self], host_in, host_out)
        t1, t2 = ctypes.c_double(), ctypes.c_double()
        _check(lib().pifft_execute(self._h, host_in.ctypes.data, out_ptr, ctypes.byref(t1), ctypes.byref(t2)),
               "pifft_execute")
        return t1.value, t2.value

    def tree_device(self, d_in: int, d_seg: int, stream=None) -> None:
        _check(lib().pifft_tree_device(self._h, d_in, d_seg, _stream(stream)), "pifft_tree_device")

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            lib().pifft_plan_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def describe_info(i: PlanInfo) -> dict:
    nl = i.num_launches
    return {
        "n": i.n, "workers": i.workers, "first_worker": i.first_worker, "num_workers": i.num_workers,
        "batch": i.batch, "prec": i.prec, "local_n": i.local_n, "in_elems": i.in_elems,
        "out_elems": i.out_elems, "workspace_bytes": i.workspace_bytes, "num_launches": nl,
        "num_passes": i.num_passes, "tree_launches": i.tree_launches,
        "radix": list(i.radix[: i.num_passes]), "lines": list(i.lines[: i.num_passes]),
        "launch_bytes": list(i.launch_bytes[: min(nl, MAX_LAUNCH_INFO)]),
        "launch_kind": [KIND_NAMES.get(k, "?") for k in i.launch_kind[: min(nl, MAX_LAUNCH_INFO)]],
        "launch_fn": list(i.launch_fn[: min(nl, MAX_LAUNCH_INFO)]),
        "launch_mode": list(i.launch_mode[: min(nl, MAX_LAUNCH_INFO)]),
        "vpt": list(i.vpt[: i.num_passes]),
        "worker_interleaved": bool(i.layout & 1), "natural_store": bool(i.layout & 2),
    }


INSTANCE_FIELDS = ("prec", "R", "C", "mode", "nts", "lp", "vpt")


def instances() -> list:
    """Every compiled k_pass instance as (prec, R, C, MODE, NTS, LP, VPT), in
    registry order (pifft_instance_desc)."""
    out = []
    d = (ctypes.c_int32 * 7)()
    for i in range(lib().pifft_instance_count()):
        _check(lib().pifft_instance_desc(i, d), "pifft_instance_desc")
        out.append(tuple(d))
    return out


def instances_found() -> list:
    """Registry indices of the instances the planner has found in this
    process (pifft_instance_found): every instance a plan built so far
    depends on."""
    return [i for i in range(lib().pifft_instance_count()) if lib().pifft_instance_found(i) == 1]


def dry_run_instances(n: int, workers: int = 1, batch: int = 1, prec: int = F64, *, first: int = 0,
                      count: int | None = None, flags: int | None = None) -> list:
    """The registry index of each launch's k_pass instance (-1: a tree or
    interleave launch) of the plan pifft_plan_dry_run describes (flags as
    dry_run: natural order for all workers, else slice-major)."""
    count = workers if count is None else count
    if flags is None:
        flags = OUT_NATURAL if count == workers else OUT_SLICES
    ids = (ctypes.c_int32 * MAX_LAUNCH_INFO)()
    nl = lib().pifft_plan_dry_run_instances(n, workers, first, count, batch, prec, flags, ids, MAX_LAUNCH_INFO)
    if nl < 0:
        raise PifftError(f"pifft_plan_dry_run_instances: {last_error()}")
    return list(ids[:min(nl, MAX_LAUNCH_INFO)])


def dry_run(n: int, workers: int = 1, batch: int = 1, prec: int = F64, *, first: int = 0,
            count: int | None = None, flags: int | None = None) -> dict:
    """The plan that would be built, without a device (host planning only)."""
    count = workers if count is None else count
    if flags is None:
        flags = OUT_NATURAL if count == workers else OUT_SLICES
    info = PlanInfo()
    _check(lib().pifft_plan_dry_run(n, workers, first, count, batch, prec, flags, ctypes.byref(info)),
           "pifft_plan_dry_run")
    return describe_info(info)


def _host_buffers(plans, host_in, host_out):
    """Checks the host arrays against the plans before any pointer crosses the
    ABI (pifft_execute copies batch*N values from host_in and writes up to
    batch*N values into host_out): dtype = the plans' precision (complex64 for
    F32, complex128 for F64), at least batch*N elements, host_out C-contiguous
    and writeable.  Returns (contiguous host_in, host_out pointer or None)."""
    import numpy as np
    if not plans:
        raise PifftError("no plans")
    info = plans[0].info
    want = np.dtype(np.complex128 if info.prec == F64 else np.complex64)
    need = info.batch * info.n
    host_in = np.asarray(host_in)
    if host_in.dtype != want:
        raise PifftError(f"host_in dtype {host_in.dtype} does not match the plan's precision ({want})")
    host_in = np.ascontiguousarray(host_in)
    if host_in.size < need:
        raise PifftError(f"host_in holds {host_in.size} values, the plan reads batch*N = {need}")
    if host_out is None:
        return host_in, None
    if not isinstance(host_out, np.ndarray):
        raise PifftError("host_out must be a numpy array")
    if host_out.dtype != want:
        raise PifftError(f"host_out dtype {host_out.dtype} does not match the plan's precision ({want})")
    if not host_out.flags.c_contiguous or not host_out.flags.writeable:
        raise PifftError("host_out must be C-contiguous and writeable")
    if host_out.size < need:
        raise PifftError(f"host_out holds {host_out.size} values, the plan writes up to batch*N = {need}")
    return host_in, host_out.ctypes.data


def execute_group(plans, host_in, host_out=None):
    for p in plans[1:]:
        if (p.info.n, p.info.batch, p.info.prec) != (plans[0].info.n, plans[0].info.batch, plans[0].info.prec):
            raise PifftError("plans of a group must share n, batch and precision")
    host_in, out_ptr = _host_buffers(plans, host_in, host_out)
    arr = (_P * len(plans))(*[p.handle.value for p in plans])
    t1, t2 = ctypes.c_double(), ctypes.c_double()
    _check(lib().pifft_execute_group(arr, len(plans), host_in.ctypes.data, out_ptr, ctypes.byref(t1),
                                     ctypes.byref(t2)), "pifft_execute_group")
    return t1.value, t2.value


def execute_group_kernel_times(plans):
    """pifft_execute_group_kernel_times: the kernel-only stage sums (ms) of the
    slowest plan, re-running the last execute_group's staged input."""
    arr = (_P * len(plans))(*[p.handle.value for p in plans])
    t1, t2 = ctypes.c_double(), ctypes.c_double()
    _check(lib().pifft_execute_group_kernel_times(arr, len(plans), ctypes.byref(t1), ctypes.byref(t2)),
           "pifft_execute_group_kernel_times")
    return t1.value, t2.value


def allgather(plans, d_slices, d_natural) -> float:
    """pifft_allgather: every plan's slice-major result (device addresses,
    one per plan) -> natural order on each plan's device whose d_natural entry
    is not None.  Returns the slowest destination's time (ms)."""
    n = len(plans)
    if len(d_slices) != n or len(d_natural) != n:
        raise PifftError("one slice buffer and one destination (or None) per plan")
    arr = (_P * n)(*[p.handle.value for p in plans])
    sl = (_P * n)(*[int(a) for a in d_slices])
    nat = (_P * n)(*[None if a is None else int(a) for a in d_natural])
    ms = ctypes.c_double()
    _check(lib().pifft_allgather(arr, n, sl, nat, ctypes.byref(ms)), "pifft_allgather")
    return ms.value


def generate_device(d_x: int, count: int, n: int, prec: int, seed: int = 0x5EED, first: int = 0,
                    stream=None) -> None:
    _check(lib().pifft_generate_device(d_x, count, n, seed, first, prec, _stream(stream)),
           "pifft_generate_device")


def interleave_device(d_slices: int, d_out: int, n: int, workers: int, batch: int, prec: int,
                      stream=None) -> None:
    _check(lib().pifft_interleave_device(d_slices, d_out, n, workers, batch, prec, _stream(stream)),
           "pifft_interleave_device")


def header_symbols(header_path: str | None = None) -> list[str]:
    """Function names declared in include/pifft.h (for the ABI export test)."""
    import re
    header_path = header_path or os.path.join(os.path.dirname(HERE), "include", "pifft.h")
    text = open(header_path).read()
    return sorted(set(re.findall(r"\b(pifft_[a-z_]+)\s*\(", text)))
