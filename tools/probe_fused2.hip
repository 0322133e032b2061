// tools/probe_fused2.hip -- standalone probe (not part of the product), round 5.
// The copy ceiling of one rank's fused tree + first pass in the G-GPU split of
// fp64 N = 2^28 (k_pass<double,512,16,3,1,LP>), by leaf-read segment width:
// each of a tile's 8192 inputs z[j + r M/R] (C adjacent lines j, R = 8192/C
// rows r) sums its P leaves x[zi + m M] (M = N/P; no twiddles, no FFT), the
// tile's results stored contiguously -- the kernel's data movement at C = 8,
// 16, 32, 64 (128 B .. 1 KiB row segments).  "flat": the same bytes with
// every wave instruction reading 64 consecutive elements of a leaf (1 KiB,
// the k_tree pattern) -- the best these P streams can do.  P = 1 is a plain
// first-pass copy (strided read at C*16 B, contiguous write).  512 threads,
// 16 values per thread, 2 workgroups per CU, 8 leaf loads in flight per
// thread and round, groups of 4 tiles per XCD: as the kernel.
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_fused2.hip -o tools/probe_fused2_bin
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

// C = 0: flat (consecutive elements per wave instruction)
template <int C, int P>
__global__ __launch_bounds__(512, 2) void k_copy(const d2* __restrict__ x, d2* __restrict__ out, uint32_t log_m) {
    extern __shared__ d2 dummy[];
    constexpr int G = P >= 8 ? 1 : 8 / P;  // values per round: 8 leaf loads in flight
    const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint32_t log_lines = C ? log_m - (13 - __builtin_ctz(C)) : 0;  // log2(M/R), R = 8192/C
    d2 v[16];
#pragma unroll
    for (int k0 = 0; k0 < 16; k0 += G) {
        d2 w[G][P];
#pragma unroll
        for (int g = 0; g < G; g++) {
            const int e = threadIdx.x + (k0 + g) * 512;
            const uint64_t zi = C ? tile * C + (e % (C ? C : 1)) + ((uint64_t)(e / (C ? C : 1)) << log_lines)
                                  : tile * 8192 + e;
#pragma unroll
            for (int m = 0; m < P; m++) w[g][m] = __builtin_nontemporal_load(x + zi + ((uint64_t)m << log_m));
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

static hipEvent_t e0, e1;

template <int C, int P>
static float run(const d2* x, d2* y, uint32_t log_n) {
    const uint32_t log_m = log_n - __builtin_ctz(P);
    const uint32_t ntiles = (uint32_t)((1ull << log_m) >> 13);
    auto k = k_copy<C, P>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
    auto launch = [&] { hipLaunchKernelGGL(k, dim3(ntiles), dim3(512), 72 * 1024, 0, x, y, log_m); };
    for (int w = 0; w < 3; w++) launch();
    (void)hipEventRecord(e0);
    for (int it = 0; it < 20; it++) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 20;
}

template <int P>
static void row(const d2* x, d2* y, uint32_t log_n) {
    const double bytes = (double)(1ull << log_n) * 16 * (1.0 + 1.0 / P);
    const float t8 = run<8, P>(x, y, log_n), t16 = run<16, P>(x, y, log_n), t32 = run<32, P>(x, y, log_n),
                t64 = run<64, P>(x, y, log_n), tf = run<0, P>(x, y, log_n);
    printf("P=%d (%.2f GB): C=8 (128 B) %.3f ms %.0f GB/s | C=16 (256 B) %.3f ms %.0f | C=32 (512 B) %.3f ms %.0f | "
           "C=64 (1 KiB) %.3f ms %.0f | flat %.3f ms %.0f\n",
           P, bytes / 1e9, t8, bytes / t8 / 1e6, t16, bytes / t16 / 1e6, t32, bytes / t32 / 1e6, t64,
           bytes / t64 / 1e6, tf, bytes / tf / 1e6);
    fflush(stdout);
}

int main() {
    const uint32_t log_n = 28;
    d2 *x, *y;
    if (hipMalloc(&x, (1ull << log_n) * 16) || hipMalloc(&y, (1ull << log_n) * 16)) return 1;
    (void)hipMemset(x, 0, (1ull << log_n) * 16);
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int round = 0; round < 2; round++) {
        printf("round %d\n", round);
        row<8>(x, y, log_n);
        row<4>(x, y, log_n);
        row<2>(x, y, log_n);
        row<1>(x, y, log_n);
    }
    if (hipGetLastError() != hipSuccess) return 2;
    return 0;
}
