// tools/probe_fused.hip -- standalone probe (not part of the product).
// The copy ceiling of the fused tree + first pass of one GPU's plan in the
// 8-GPU split of fp64 N = 2^28 (k_pass<double,512,16,3,1,3>: worker q's
// segment M = 2^25, R = 512, C = 16 lines per tile): each of a tile's 8192
// inputs z[j + r 2^16] sums its P = 8 leaves x[j + r 2^16 + m 2^25] (no
// twiddles, no FFT), and the tile's 8192 results are stored contiguously.
// Loads in rounds of G*P leaves per thread (the kernel's PIFFT_TREE_LOADS),
// 512 threads, 2 workgroups per CU like the kernel.  Against the kernel's
// 0.865-0.876 ms (profiles/r02_rank_plans.log).
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_fused.hip -o tools/probe_fused
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double __attribute__((ext_vector_type(2))) d2;

__device__ __forceinline__ uint64_t xcd_tile(uint32_t b, uint32_t nblocks) {
    const uint32_t log_xg = 2;
    if (nblocks & ((8u << log_xg) - 1)) return b;
    const uint32_t xcd = b & 7, slot = b >> 3, gmask = (1u << log_xg) - 1;
    return ((uint64_t)(slot >> log_xg) << (log_xg + 3)) + ((uint64_t)xcd << log_xg) + (slot & gmask);
}

template <int LOADS>
__global__ __launch_bounds__(512, 2) void k_fused_copy(const d2* __restrict__ x, d2* __restrict__ out) {
    extern __shared__ d2 dummy[];
    constexpr int P = 8, G = LOADS / P;
    const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    d2 v[16];
#pragma unroll
    for (int k0 = 0; k0 < 16; k0 += G) {
        d2 w[G][P];
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int e = threadIdx.x + (k0 + g) * 512;  // element of the tile: line c = e % 16, row r = e / 16
            const uint64_t zi = tile * 16 + (e & 15) + ((uint64_t)(e >> 4) << 16);
#pragma unroll
            for (int m = 0; m < P; m++) w[g][m] = __builtin_nontemporal_load(x + zi + ((uint64_t)m << 25));
        }
#pragma unroll
        for (int g = 0; g < G; g++) {
            d2 s = w[g][0];
#pragma unroll
            for (int m = 1; m < P; m++) s += w[g][m];
            v[k0 + g] = s;
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (threadIdx.x == 4095) dummy[0] = v[0];  // never true: keeps the LDS allocation (2 WG/CU)
#pragma unroll
    for (int k = 0; k < 16; k++) __builtin_nontemporal_store(v[k], out + tile * 8192 + threadIdx.x + k * 512);
}

int main() {
    const uint64_t n = 1ull << 28, M = n >> 3;
    d2 *x, *y;
    if (hipMalloc(&x, n * 16) || hipMalloc(&y, M * 16)) return 1;
    (void)hipMemset(x, 0, n * 16);
    (void)hipFuncSetAttribute((const void*)k_fused_copy<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
    (void)hipFuncSetAttribute((const void*)k_fused_copy<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
    (void)hipFuncSetAttribute((const void*)k_fused_copy<32>, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto time = [&](auto launch) {
        for (int w = 0; w < 3; w++) launch();
        (void)hipEventRecord(e0);
        for (int it = 0; it < 20; it++) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / 20;
    };
    const uint32_t ntiles = (uint32_t)(M >> 13);
    const double bytes = (double)n * 16 + (double)M * 16;
    for (int round = 0; round < 3; round++) {
        const float t8 = time([&] { hipLaunchKernelGGL(k_fused_copy<8>, dim3(ntiles), dim3(512), 72 * 1024, 0, x, y); });
        const float t16 = time([&] { hipLaunchKernelGGL(k_fused_copy<16>, dim3(ntiles), dim3(512), 72 * 1024, 0, x, y); });
        const float t32 = time([&] { hipLaunchKernelGGL(k_fused_copy<32>, dim3(ntiles), dim3(512), 72 * 1024, 0, x, y); });
        printf("round %d: leaves in flight per thread 8: %.3f ms %.0f GB/s | 16: %.3f ms %.0f GB/s | 32: %.3f ms %.0f GB/s\n",
               round, t8, bytes / t8 / 1e6, t16, bytes / t16 / 1e6, t32, bytes / t32 / 1e6);
        fflush(stdout);
    }
    if (hipGetLastError() != hipSuccess) return 2;
    return 0;
}
