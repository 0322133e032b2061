import sys, numpy as np, torch
sys.path[:0] = ["cs87project-msolano2_amd", "oracle"]
import pifft, pifft_oracle as oracle
torch.cuda.set_device(0)
for dt, prec in ((np.complex128, pifft.F64), (np.complex64, pifft.F32)):
  for logn in (6, 10, 12, 14, 16, 18):
    n = 1 << logn
    x = oracle.generate(n, dt)
    d_in = torch.from_numpy(x).to("cuda:0")
    for P in (2, 4, 8, 16):
        bad = []
        for q in range(P):
            ref = oracle.tree_segment(x, P, q)
            p = pifft.Plan(n, P, 1, prec, first=q, count=1, device=0)
            seg = torch.empty(n // P, dtype=d_in.dtype, device="cuda:0")
            p.tree_device(d_in.data_ptr(), seg.data_ptr(), torch.cuda.current_stream())
            torch.cuda.synchronize()
            g = seg.cpu().numpy()
            if g.tobytes() != ref.tobytes():
                nb = int((g != ref).sum()); md = float(np.abs(g - ref).max())
                first = int(np.argmax(g != ref))
                bad.append((q, nb, md, first))
        # all-worker plan
        pa = pifft.Plan(n, P, 1, prec, first=0, count=P, device=0, flags=pifft.OUT_SLICES)
        sa = torch.empty(n, dtype=d_in.dtype, device="cuda:0")
        pa.tree_device(d_in.data_ptr(), sa.data_ptr(), torch.cuda.current_stream()); torch.cuda.synchronize()
        allref = np.concatenate([oracle.tree_segment(x, P, q) for q in range(P)])
        aok = sa.cpu().numpy().tobytes() == allref.tobytes()
        print(dt.__name__, logn, P, "single-bad:", bad, "all-ok:", aok, flush=True)
