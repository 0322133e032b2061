// tools/probe_c2_store.hip -- standalone probe (not part of the product).
// Config 2 (fp64 N=2^20, all 8 workers on one GPU) ends with its last pass
// (R = 256, C = 8: 128 threads x 16 values) writing slice-major, then a
// separate interleave launch into natural order (bin bitrev3(q) + 8 k of
// worker q).  Would the last pass storing natural order directly (16-B
// pieces 128 B apart; the 16 MiB output stays in L2 / the Infinity Cache)
// beat the extra launch?  Copies with the exact index maps:
//   slice : tile of worker q reads q 2^17 + j + 512 r, writes the same index
//   inter : the interleave: out[bitrev3(q) + 8 k] = in[q 2^17 + k]
//   nat   : the pass writing (j + 512 r) 8 + bitrev3(q) directly
//   wi<CW>: (round 2, second form) a "worker-interleaved" tile: CW lines of
//           ALL 8 workers per workgroup, loaded CW x 16 B at a time per worker
//           row, stored with the 8 workers' values of one output adjacent
//           (8 x CW consecutive natural outputs per row, coalesced)
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_c2_store.hip -o tools/probe_c2_store
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double __attribute__((ext_vector_type(2))) d2;

__device__ __forceinline__ uint32_t brev3(uint32_t q) { return ((q & 1) << 2) | (q & 2) | ((q >> 2) & 1); }

template <int NAT, int NT_ST>
__global__ __launch_bounds__(128) void k_last(const d2* __restrict__ in, d2* __restrict__ out) {
    // 512 tiles: worker q = tile >> 6, line block jb = tile & 63 (8 lines of 512)
    const uint32_t q = blockIdx.x >> 6, jb = blockIdx.x & 63;
    d2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + 128 * k, c = g & 7, r = g >> 3;
        v[k] = __builtin_nontemporal_load(in + ((uint64_t)q << 17) + jb * 8 + c + 512 * r);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + 128 * k, c = g & 7, r = g >> 3;
        const uint64_t e = jb * 8 + c + 512 * r;
        d2* p = NAT ? out + (e << 3) + brev3(q) : out + ((uint64_t)q << 17) + e;
        if (NT_ST) __builtin_nontemporal_store(v[k], p);
        else *p = v[k];
    }
}

template <int CW>
__global__ __launch_bounds__(128 * CW) void k_wi(const d2* __restrict__ in, d2* __restrict__ out) {
    constexpr int NT = 128 * CW;
    const uint32_t t = blockIdx.x;  // lines t CW .. t CW + CW - 1 of every worker
    d2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + NT * k, cw = g % CW, q = (g / CW) & 7, r = g / (8 * CW);
        v[k] = __builtin_nontemporal_load(in + ((uint64_t)q << 17) + t * CW + cw + 512 * r);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + NT * k, q = g & 7, cw = (g >> 3) % CW, r = g / (8 * CW);
        out[((uint64_t)(t * CW + cw + 512 * r) << 3) + brev3(q)] = v[k];
    }
}

__global__ __launch_bounds__(256) void k_inter(const d2* __restrict__ in, d2* __restrict__ out) {
    // natural-order writes, 8 consecutive outputs from the 8 slices
    const uint64_t i = blockIdx.x * 256ull + threadIdx.x;  // natural index
    const uint32_t r = i & 7;
    const uint64_t k = i >> 3;
    out[i] = in[((uint64_t)brev3(r) << 17) + k];
}

int main() {
    const uint64_t n = 1ull << 20;
    d2 *x, *y, *z;
    if (hipMalloc(&x, n * 16) || hipMalloc(&y, n * 16) || hipMalloc(&z, n * 16)) return 1;
    (void)hipMemset(x, 0, n * 16);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto time = [&](auto launch) {
        for (int w = 0; w < 20; w++) launch();
        (void)hipEventRecord(e0);
        for (int it = 0; it < 200; it++) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms * 1000 / 200;
    };
    for (int round = 0; round < 3; round++) {
        const float a = time([&] { hipLaunchKernelGGL((k_last<0, 1>), dim3(512), dim3(128), 0, 0, x, y); });
        const float ai = time([&] {
            hipLaunchKernelGGL((k_last<0, 1>), dim3(512), dim3(128), 0, 0, x, y);
            hipLaunchKernelGGL(k_inter, dim3(n / 256), dim3(256), 0, 0, y, z);
        });
        const float b1 = time([&] { hipLaunchKernelGGL((k_last<1, 1>), dim3(512), dim3(128), 0, 0, x, z); });
        const float b0 = time([&] { hipLaunchKernelGGL((k_last<1, 0>), dim3(512), dim3(128), 0, 0, x, z); });
        const float w1 = time([&] { hipLaunchKernelGGL(k_wi<1>, dim3(512), dim3(128), 0, 0, x, z); });
        const float w2 = time([&] { hipLaunchKernelGGL(k_wi<2>, dim3(256), dim3(256), 0, 0, x, z); });
        const float w4 = time([&] { hipLaunchKernelGGL(k_wi<4>, dim3(128), dim3(512), 0, 0, x, z); });
        printf("round %d (us): last pass slice-major %.2f, + interleave launch %.2f | natural store nt %.2f, plain %.2f"
               " | worker-interleaved tile CW=1 %.2f, CW=2 %.2f, CW=4 %.2f\n",
               round, a, ai, b1, b0, w1, w2, w4);
        fflush(stdout);
    }
    return hipGetLastError() != hipSuccess ? 2 : 0;
}
