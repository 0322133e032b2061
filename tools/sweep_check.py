"""Diagnostic: GPU plan vs numpy float64 FFT for a range of sizes (one process)."""
import sys, os, math
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs87project-msolano2_amd"))
import torch
import pifft
lo, hi = int(sys.argv[1]), int(sys.argv[2])
P = int(sys.argv[3]) if len(sys.argv) > 3 else 1
for logn in range(lo, hi + 1):
    n = 1 << logn
    x = torch.empty(n, dtype=torch.complex128, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, pifft.F64, stream=torch.cuda.current_stream())
    plan = pifft.Plan(n, P, 1, pifft.F64)
    X = torch.empty_like(x)
    plan.execute_device(x.data_ptr(), X.data_ptr(), torch.cuda.current_stream())
    torch.cuda.synchronize()
    xh = x.cpu().numpy(); Xh = X.cpu().numpy()
    ref = np.fft.fft(xh)
    err = np.linalg.norm(Xh - ref) / np.linalg.norm(ref)
    bad = np.nonzero(np.abs(Xh - ref) > 1e-9 * np.abs(ref).max())[0]
    print(logn, P, plan.describe()["radix"], plan.describe()["lines"], f"{err:.3e}", len(bad), bad[:8], flush=True)
