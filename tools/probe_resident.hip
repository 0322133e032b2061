// tools/probe_resident.hip -- standalone probe (not part of the product).
// Is a 128-KiB-tile copy (the pass kernel's shape: 16 x 16 B per lane, 512
// threads, one tile per workgroup) bound by the CU pipeline or by the memory
// level?  The same copy over buffers from 2 MiB (L2-resident per XCD after the
// first launch) to 4 GiB (HBM), 20 launches back to back, plain loads/stores.
// If cache-resident sizes copy far above ~6 TB/s, sub-passes kept in L2 would
// be cheap; if not, the pipeline is the limit at every level.
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_resident.hip -o tools/probe_resident
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float __attribute__((ext_vector_type(4))) f4;

template <int U>
__global__ __launch_bounds__(512) void tile_k(const f4* __restrict__ in, f4* __restrict__ out) {
    const uint64_t base = (uint64_t)blockIdx.x * blockDim.x * U + threadIdx.x;
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = in[base + (uint64_t)u * blockDim.x];
#pragma unroll
    for (int u = 0; u < U; u++) out[base + (uint64_t)u * blockDim.x] = v[u];
}

int main() {
    const uint64_t maxS = 1ull << 32;
    f4 *A, *B;
    if (hipMalloc(&A, maxS) || hipMalloc(&B, maxS)) return 1;
    (void)hipMemset(A, 0, maxS);
    (void)hipMemset(B, 0, maxS);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    printf("bytes\ttile\tlaunches\tus_per_launch\tGB/s(r+w)\n");
    for (uint64_t S = 2ull << 20; S <= maxS; S <<= 1) {
        for (int which = 0; which < 2; which++) {
            const int U = which ? 16 : 1, BS = which ? 512 : 256;
            const unsigned grid = (unsigned)(S / 16 / ((uint64_t)BS * U));
            auto launch = [&] {
                if (which) hipLaunchKernelGGL((tile_k<16>), dim3(grid), dim3(BS), 0, 0, A, B);
                else hipLaunchKernelGGL((tile_k<1>), dim3(grid), dim3(BS), 0, 0, A, B);
            };
            const int reps = S <= (256ull << 20) ? 50 : 5;
            launch();
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0, 0);
            for (int r = 0; r < reps; r++) launch();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double us = 1e3 * ms / reps;
            printf("%llu\t%s\t%d\t%.2f\t%.0f\n", (unsigned long long)S, which ? "128KiB" : "4KiB", reps, us,
                   2.0 * S / (us * 1e-6) / 1e9);
        }
    }
    return 0;
}
