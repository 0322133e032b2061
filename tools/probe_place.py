#!/usr/bin/env python3
"""tools/probe_place.py -- is the C4 pass time a property of where the buffers
landed?

Pass 3 of the fp64 2^28 plan reads the plan's workspace W and writes the
caller's output at the SAME 8 MiB-strided offsets; it has measured 1.57-1.90
ms box to box and run to run.  Round 2, first probe (profiles/r02_probe_place.log):
shifting the output inside its allocation changes nothing consistently, but
a fresh allocation of the buffers does (one of five trials ran passes 2/3 at
1.41/1.57 ms for every offset, the rest at 1.48/1.65-1.85).

This probe allocates the input, output and workspace with
hipExtMallocWithFlags(flags) for flags in PROBE_FLAGS (0 = hipMalloc's
default, 4 = hipDeviceMallocContiguous), TRIALS fresh allocations each (the
earlier ones kept alive so new ones land elsewhere), and times the three
passes with HIP events.  A probe, not product.
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))

import torch  # noqa: E402

import pifft  # noqa: E402

LOG_N = int(os.environ.get("PROBE_LOG_N", "28"))
TRIALS = int(os.environ.get("PROBE_TRIALS", "4"))
FLAGS = [int(f) for f in os.environ.get("PROBE_FLAGS", "0,4").split(",")]
STEPS = 8

hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipFree.argtypes = [ctypes.c_void_p]


def dalloc(nbytes, flags):
    p = ctypes.c_void_p()
    rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, flags)
    if rc != 0:
        raise RuntimeError(f"hipExtMallocWithFlags({nbytes}, {flags}) = {rc}")
    return p.value


def main():
    torch.cuda.set_device(0)
    n = 1 << LOG_N
    s = torch.cuda.current_stream()
    keep = []
    for flags in FLAGS:
        os.environ["PIFFT_W_MALLOC_FLAGS"] = str(flags)
        for t in range(TRIALS):
            x = dalloc(n * 16, flags)
            y = dalloc(n * 16, flags)
            pifft.generate_device(x, n, n, pifft.F64, seed=11, stream=s)
            plan = pifft.Plan(n, 1, 1, pifft.F64, device=0)
            keep.append((x, y, plan))
            for rep in range(2):
                for _ in range(2):
                    plan.execute_device(x, y, s)
                torch.cuda.synchronize()
                plan.profile_start(STEPS, pifft.PROFILE_ALL)
                for _ in range(STEPS):
                    plan.execute_device(x, y, s)
                used, sums, _ = plan.profile_read()
                ms = [v / used for v in sums]
                print(f"flags {flags} trial {t} rep {rep} x={x & ((1 << 32) - 1):#010x} y={y & ((1 << 32) - 1):#010x}"
                      f"  passes " + " ".join(f"{v:.3f}" for v in ms) + f"  total {sum(ms):.3f} ms", flush=True)
    for x, y, plan in keep:
        plan.close()
        hip.hipFree(x)
        hip.hipFree(y)



def which_buffer():
    """PROBE_MODE=which: x and y fixed, six fresh plans (fresh workspace W);
    then the last plan fixed and six fresh outputs y."""
    torch.cuda.set_device(0)
    n = 1 << LOG_N
    s = torch.cuda.current_stream()
    x, y = dalloc(n * 16, 0), dalloc(n * 16, 0)
    pifft.generate_device(x, n, n, pifft.F64, seed=11, stream=s)

    def timeit(plan, yy, tag):
        for _ in range(2):
            plan.execute_device(x, yy, s)
        torch.cuda.synchronize()
        plan.profile_start(STEPS, pifft.PROFILE_ALL)
        for _ in range(STEPS):
            plan.execute_device(x, yy, s)
        used, sums, _ = plan.profile_read()
        ms = [v / used for v in sums]
        print(f"{tag} passes " + " ".join(f"{v:.3f}" for v in ms) + f"  total {sum(ms):.3f} ms", flush=True)

    plans = []
    for t in range(6):
        plans.append(pifft.Plan(n, 1, 1, pifft.F64, device=0))
        timeit(plans[-1], y, f"fresh W {t}, same x y:")
    ys = [y]
    for t in range(6):
        ys.append(dalloc(n * 16, 0))
        timeit(plans[-1], ys[-1], f"fresh y {t}, same x W:")
    for t, p in enumerate(plans):
        timeit(p, y, f"again W {t}, first y:")


if __name__ == "__main__" and os.environ.get("PROBE_MODE") == "which":
    which_buffer()
    sys.exit(0)


if __name__ == "__main__":
    main()
