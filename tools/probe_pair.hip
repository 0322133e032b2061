// tools/probe_pair.hip -- standalone probe (not part of the product).
// The C4 passes 2 and 3 (fp64 2^28, 512-point lines 8 MiB apart) run in one of
// two states per (workspace W, output y) pair of allocations: fast (1.41 /
// 1.58 ms) or slow (1.48 / 1.70-1.86 ms), stable for the pair and independent
// of x (tools/probe_place.py, profiles/r02_probe_place.log).  Is that an
// alignment between the two buffers' rows that a padded W layout breaks?
// Copies with the exact index maps of pass 2 (y -> W) and pass 3 (W -> y),
// element e of W at e + (e >> s) p, for several fresh W allocations against
// one y.
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_pair.hip -o tools/probe_pair
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double __attribute__((ext_vector_type(2))) d2;

__device__ __forceinline__ uint64_t padded(uint64_t e, int s, int p) { return e + (p ? (e >> s) * (uint64_t)p : 0); }

__device__ __forceinline__ uint64_t xcd_tile(uint32_t b, uint32_t nblocks) {
    const uint32_t log_xg = 2;
    if (nblocks & ((8u << log_xg) - 1)) return b;
    const uint32_t xcd = b & 7, slot = b >> 3, gmask = (1u << log_xg) - 1;
    return ((uint64_t)(slot >> log_xg) << (log_xg + 3)) + ((uint64_t)xcd << log_xg) + (slot & gmask);
}

// pass 2: line j < 2^19 reads y[j + r 2^19], writes W[(j>>10)<<19 + (j&1023) + r 1024]
// pass 3: line j < 2^19 reads W[j + r 2^19], writes y[j + r 2^19]      (r < 512, C = 16)
template <int PASS>
__global__ __launch_bounds__(512, 2) void k_copy(const d2* __restrict__ in, d2* __restrict__ out, int s, int p) {
    extern __shared__ d2 dummy[];
    const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    d2 v[16];
    uint64_t src[16], dst[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + k * 512;
        const int c = g & 15, r = g >> 4;
        const uint64_t j = tile * 16 + c;
        if (PASS == 2) {
            src[k] = j + ((uint64_t)r << 19);
            dst[k] = padded(((j >> 10) << 19) + (j & 1023) + ((uint64_t)r << 10), s, p);
        } else {
            src[k] = padded(j + ((uint64_t)r << 19), s, p);
            dst[k] = j + ((uint64_t)r << 19);
        }
        v[k] = __builtin_nontemporal_load(in + src[k]);
    }
    if (threadIdx.x == 4095) dummy[0] = v[0];  // never true: keeps the LDS allocation (2 WG/CU like k_pass)
#pragma unroll
    for (int k = 0; k < 16; k++) __builtin_nontemporal_store(v[k], out + dst[k]);
}

int main() {
    const uint64_t n = 1ull << 28;
    const uint64_t wcap = n + n / 8 + (1ull << 22);  // room for every padded layout below
    d2* y;
    if (hipMalloc(&y, n * 16)) return 1;
    (void)hipMemset(y, 0, n * 16);
    (void)hipFuncSetAttribute((const void*)k_copy<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
    (void)hipFuncSetAttribute((const void*)k_copy<3>, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto time = [&](auto launch) {
        for (int w = 0; w < 2; w++) launch();
        (void)hipEventRecord(e0);
        for (int it = 0; it < 10; it++) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / 10;
    };
    // (s, p): none; 256 B per 16 KiB; 256 B / 4 KiB / 64 KiB / 1 MiB + 256 B per 8 MiB row
    const int pads[][2] = {{0, 0}, {10, 16}, {19, 16}, {19, 256}, {19, 4096}, {19, 65536 + 16}};
    const uint32_t ntiles = (uint32_t)(n >> 13);
    for (int a = 0; a < 8; a++) {
        d2* w;
        if (hipMalloc(&w, wcap * 16)) return 1;  // kept: the next W lands elsewhere
        (void)hipMemset(w, 0, wcap * 16);
        printf("W %d (%#llx, y %#llx):", a, (unsigned long long)(uintptr_t)w & 0xffffffffffull,
               (unsigned long long)(uintptr_t)y & 0xffffffffffull);
        for (const auto& pd : pads) {
            const int s = pd[0], p = pd[1];
            const float t2 = time([&] { hipLaunchKernelGGL(k_copy<2>, dim3(ntiles), dim3(512), 72 * 1024, 0, y, w, s, p); });
            const float t3 = time([&] { hipLaunchKernelGGL(k_copy<3>, dim3(ntiles), dim3(512), 72 * 1024, 0, w, y, s, p); });
            printf("  [%d,%d] %.3f %.3f", s, p, t2, t3);
        }
        printf("\n");
        fflush(stdout);
    }
    if (hipGetLastError() != hipSuccess) return 2;
    return 0;
}
