#!/usr/bin/env python3
"""tools/wg_clock.py -- where a small pass's time goes, from inside the kernel.

Needs the diagnostics build (EXTRA=-DPIFFT_WG_CLOCK tools/mkvariant.sh
wgclock -> abvar/wgclock.so): every workgroup of the clocked launch records
its entry wall clock (100 MHz), the wall clock once its stores completed and
its hardware id, and thread 0 stamps each step of the load -> exchanges ->
store chain (PassArgs::wg_clock, 8 words per workgroup).  Per pass launch of
the plan this prints the kernel's event-bound duration beside the
workgroups' timeline:
  ramp   -- last workgroup entry - first entry (dispatch of the grid),
  wg     -- one workgroup's entry to stores-done (min / median / max),
  span   -- first entry to last stores-done,
so duration - span is the launch's fixed cost outside the workgroups; and the
median workgroup's chain, step by step (us): load (entry -> inputs in
registers; MODE 11: -> the tree's values handed to the first stage), s1..s3
(stage S-1's butterflies + the exchange into stage S), last (the last stage's
butterflies), store (-> stores completed).

usage: PIFFT_LIB=abvar/wgclock.so python3 tools/wg_clock.py --log-n 20 [--workers 8 --count 1] [--prec 64]
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))
os.environ.setdefault("PIFFT_LIB", os.path.join(ROOT, "abvar", "wgclock.so"))

import pifft  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log-n", type=int, default=20)
    ap.add_argument("--workers", type=int, default=1)
    ap.add_argument("--count", type=int, default=0, help="workers in the plan (default all)")
    ap.add_argument("--prec", type=int, default=64, choices=(32, 64))
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20, help="clocked launches per pass (medians reported)")
    ap.add_argument("--dump", default="", help="CSV of every workgroup of every clocked launch (launch, rep, wg, "
                                               "start_us, end_us, hw_id; times from the launch's first entry)")
    args = ap.parse_args()
    L = pifft.lib()
    f = L.pifft_debug_wg_clock
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_size_t, ctypes.POINTER(ctypes.c_ulonglong)]
    n = 1 << args.log_n
    prec = pifft.F64 if args.prec == 64 else pifft.F32
    count = args.count or args.workers
    plan = pifft.Plan(n, args.workers, args.batch, prec, first=0, count=count, device=0)
    d = plan.describe()
    cdt = torch.complex128 if prec == pifft.F64 else torch.complex64
    st = torch.cuda.current_stream()
    x = torch.empty(n * args.batch, dtype=cdt, device="cuda")
    pifft.generate_device(x.data_ptr(), n * args.batch, n, prec, stream=st)
    y = torch.empty(d["out_elems"], dtype=cdt, device="cuda")
    for _ in range(20):
        plan.execute_device(x.data_ptr(), y.data_ptr(), st)
    torch.cuda.synchronize()
    ev = [plan.execute_device_timed(x.data_ptr(), y.data_ptr(), st) for _ in range(args.reps)]
    print(f"n=2^{args.log_n} P={args.workers} count={count} fp{args.prec} batch={args.batch}: "
          f"launches {d['launch_kind']}, radix {d['radix']}")
    dump = open(args.dump, "w") if args.dump else None
    if dump:
        dump.write("launch,rep,wg,start_us,end_us,hw_id\n")
    for li in range(d["num_launches"]):
        name = plan.kernel_name(li)
        W = 8  # PIFFT_WGC_WORDS
        buf = (ctypes.c_ulonglong * (W * 65536))()
        steps = []
        hz = ctypes.c_ulonglong()
        rows = []
        for _ in range(args.reps):
            nwg = f(plan.handle, li, x.data_ptr(), y.data_ptr(), ctypes.c_void_p(st.cuda_stream), 3, buf, len(buf),
                    ctypes.byref(hz))
            if nwg < 0:
                print(f"launch {li} ({name}): {pifft.last_error()}")
                break
            us = 1e6 / hz.value
            t0 = [buf[W * w] for w in range(nwg)]
            t1 = [buf[W * w + 1] for w in range(nwg)]
            for w in range(nwg):  # the chain: entry, inputs, stages 1..3 reached, last computed, stores done
                marks = [buf[W * w]] + [buf[W * w + k] for k in (3, 4, 5, 6, 7)] + [buf[W * w + 1]]
                row, prev = [], marks[0]
                for m in marks[1:]:
                    if m == 0:  # (a stage this pass does not have)
                        row.append(None)
                        continue
                    row.append((m - prev) * us)
                    prev = m
                steps.append(row)
            durs = sorted((b - a) * us for a, b in zip(t0, t1))
            if dump:
                m0 = min(t0)
                for w in range(nwg):
                    dump.write(f"{li},{len(rows)},{w},{(t0[w] - m0) * us:.2f},{(t1[w] - m0) * us:.2f},{buf[W * w + 2]}\n")
            rows.append(((max(t0) - min(t0)) * us, durs[0], statistics.median(durs), durs[-1],
                         (max(t1) - min(t0)) * us, len({buf[W * w + 2] for w in range(nwg)})))
        if not rows:
            continue
        med = [statistics.median(r[k] for r in rows) for k in range(6)]
        dur = statistics.median(e[li] for e in ev) * 1e3
        print(f"  launch {li} {d['launch_kind'][li]:9s} {nwg:5d} WGs  event {dur:7.2f} us | ramp {med[0]:6.2f} | "
              f"wg {med[1]:6.2f} / {med[2]:6.2f} / {med[3]:6.2f} | span {med[4]:6.2f} | outside {dur - med[4]:6.2f} us"
              f"  ({int(med[5])} hw ids)  {name}")
        names = ("load", "s1", "s2", "s3", "last", "store")
        parts = []
        for k, nm in enumerate(names):
            vals = [r[k] for r in steps if r[k] is not None]
            if vals:
                parts.append(f"{nm} {statistics.median(vals):5.2f}")
        print("      chain (median workgroup, us): " + " | ".join(parts))


if __name__ == "__main__":
    main()
