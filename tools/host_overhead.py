import time, torch, sys
sys.path.insert(0, "cs87project-msolano2_amd")
import pifft
for (n, P, b, prec) in ((1 << 20, 1, 1, pifft.F64), (1 << 20, 8, 1, pifft.F64), (4096, 1, 512, pifft.F32), (64, 1, 1, pifft.F64)):
    plan = pifft.Plan(n, P, b, prec)
    dt = torch.complex128 if prec == pifft.F64 else torch.complex64
    x = torch.zeros(n * b, dtype=dt, device="cuda"); y = torch.empty_like(x)
    st = torch.cuda.current_stream()
    for _ in range(20): plan.execute_device(x.data_ptr(), y.data_ptr(), st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    K = 500
    t0 = time.perf_counter(); e0.record()
    for _ in range(K): plan.execute_device(x.data_ptr(), y.data_ptr(), st)
    t1 = time.perf_counter(); e1.record(); torch.cuda.synchronize(); t2 = time.perf_counter()
    print(f"n={n} P={P} batch={b} launches={plan.info.num_launches}: host enqueue {1e6*(t1-t0)/K:.1f} us/step, wall {1e6*(t2-t0)/K:.1f} us/step, gpu {1e3*e0.elapsed_time(e1)/K:.1f} us/step")
    # raw ctypes call cost: a failing call (NULL buffers) returns before any HIP call
    t0 = time.perf_counter()
    for _ in range(K):
        pifft.lib().pifft_execute_device(plan.handle, None, None, None)
    print(f"   ctypes round trip (error path) {1e6*(time.perf_counter()-t0)/K:.2f} us")
