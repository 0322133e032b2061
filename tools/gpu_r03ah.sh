#!/bin/bash
# tools/gpu_r03ah.sh -- round-3 session ah: a second padded workspace
# (PIFFT_W2=1: x -> W2 -> W -> y, the caller's output touched only by the last
# pass) vs the default (x -> y -> W -> y); bitwise check, then tuned A/B
set -o pipefail
out=gpurun_out/r03ah
mkdir -p "$out"
timeout -k 10 200 python - <<'PY' > "$out/bitwise.log" 2>&1 || { cat "$out/bitwise.log"; exit 1; }
import os, sys, torch
sys.path.insert(0, "cs87project-msolano2_amd")
import pifft
for prec, cdt in ((pifft.F64, torch.complex128), (pifft.F32, torch.complex64)):
    n = 1 << 28
    x = torch.empty(n, dtype=cdt, device="cuda")
    pifft.generate_device(x.data_ptr(), n, n, prec)
    ys = []
    for w2 in ("0", "1"):
        os.environ["PIFFT_W2"] = w2
        plan = pifft.Plan(n, 1, 1, prec)
        y = torch.empty_like(x)
        plan.execute_device(x.data_ptr(), y.data_ptr())
        torch.cuda.synchronize()
        ys.append(y)
        plan.close()
    print("prec", prec, "bitwise equal:", torch.equal(torch.view_as_real(ys[0]), torch.view_as_real(ys[1])))
    assert torch.equal(torch.view_as_real(ys[0]), torch.view_as_real(ys[1]))
PY
cat "$out/bitwise.log" | grep bitwise
V='[{}, {"PIFFT_W2":"1"}, {}, {"PIFFT_W2":"1"}, {}, {"PIFFT_W2":"1"}]'
{ echo "=== fp64 2^28"; timeout -k 10 400 python -u tools/tune.py --log-n 28 --prec 64 --steps 20 --warmup 3 --tune-ws 4 --variants "$V";
  echo "=== fp32 2^28"; timeout -k 10 300 python -u tools/tune.py --log-n 28 --prec 32 --steps 20 --warmup 3 --tune-ws 4 --variants "$V"; } > "$out/w2.log" 2>&1 || { tail "$out/w2.log"; exit 1; }
grep -E "===|wall" "$out/w2.log"
