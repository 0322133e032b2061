// tools/probe_shift.hip -- standalone probe (not part of the product).
// With padded workspace rows (16 KiB + 256 B per 8 MiB row) the C4 passes 2
// and 3 still run in a fast or a slow state per (W, y) allocation pair, both
// passes together (profiles/r02_wpad.log).  Does shifting W's base by whole
// 2 MiB pages inside one allocation move a pair between the states, i.e.
// could a plan pick a good W offset at run time?  Copies with the exact
// index maps of pass 2 (y -> W) and pass 3 (W -> y), W padded by 1040
// elements per row, for W offsets of 0..62 MiB in 2 MiB steps, over several
// fresh W allocations against one y.
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_shift.hip -o tools/probe_shift
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

constexpr uint64_t PAD = 1040;  // elements per 2^19-element W row

// pass 2: line j < 2^19 reads y[j + r 2^19], writes W[(j>>10)<<19 + (j&1023) + r 1024 + (j>>10) PAD]
// pass 3: line j < 2^19 reads W[j + r (2^19 + PAD)], writes y[j + r 2^19]      (r < 512, C = 16)
template <int PASS>
__global__ __launch_bounds__(512, 2) void k_copy(const d2* __restrict__ in, d2* __restrict__ out) {
    extern __shared__ d2 dummy[];
    const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    d2 v[16];
    uint64_t dst[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + k * 512;
        const int c = g & 15, r = g >> 4;
        const uint64_t j = tile * 16 + c;
        uint64_t src;
        if (PASS == 2) {
            src = j + ((uint64_t)r << 19);
            dst[k] = ((j >> 10) << 19) + (j & 1023) + ((uint64_t)r << 10) + (j >> 10) * PAD;
        } else {
            src = j + (uint64_t)r * ((1ull << 19) + PAD);
            dst[k] = j + ((uint64_t)r << 19);
        }
        v[k] = __builtin_nontemporal_load(in + src);
    }
    if (threadIdx.x == 4095) dummy[0] = v[0];  // never true: keeps the LDS allocation (2 WG/CU like k_pass)
#pragma unroll
    for (int k = 0; k < 16; k++) __builtin_nontemporal_store(v[k], out + dst[k]);
}

int main() {
    const uint64_t n = 1ull << 28;
    const uint64_t wlen = n + 512 * PAD;           // padded W
    const uint64_t slack = (64ull << 20) / 16;     // 64 MiB of offsets
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
        for (int it = 0; it < 8; it++) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / 8;
    };
    const uint32_t ntiles = (uint32_t)(n >> 13);
    for (int a = 0; a < 6; a++) {
        d2* wbase;
        if (hipMalloc(&wbase, (wlen + slack) * 16)) return 1;  // kept: the next W lands elsewhere
        (void)hipMemset(wbase, 0, (wlen + slack) * 16);
        printf("W %d:", a);
        for (int mib = 0; mib < 64; mib += 2) {
            d2* w = wbase + ((uint64_t)mib << 20) / 16;
            const float t2 = time([&] { hipLaunchKernelGGL(k_copy<2>, dim3(ntiles), dim3(512), 72 * 1024, 0, y, w); });
            const float t3 = time([&] { hipLaunchKernelGGL(k_copy<3>, dim3(ntiles), dim3(512), 72 * 1024, 0, w, y); });
            printf(" %d:%.3f", mib, t2 + t3);
        }
        printf("\n");
        fflush(stdout);
    }
    if (hipGetLastError() != hipSuccess) return 2;
    return 0;
}
