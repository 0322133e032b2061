// tools/probe_fuse12.hip -- standalone probe (not part of the product).
// Emulates (data movement only) passes 1+2 of the 2^28 fp64 plan
// (radix 1024 x 512 x 512) two ways:
//   hbm     pass 1: tiles of 8 columns x 1024 rows read at a 2^18-element row
//           stride (128-B segments), written contiguous to T (4 GiB);
//           pass 2: tiles of 16 columns x 512 rows read from T at a 2^19
//           stride (256-B segments), written the same way to B
//   chunked the same per chunk of CH columns of the 2^19-point column FFTs
//           (CH x 8 MiB): pass 1 tiles write into a CH x 8 MiB scratch laid
//           out [k_top][n_mid][col] (128-B segments), pass 2 tiles read it
//           contiguous (128 KiB) and write B with 256-B segments; the
//           scratch is reused by every chunk (Infinity-Cache resident?)
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_fuse12.hip -o tools/probe_fuse12
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double __attribute__((ext_vector_type(2))) d2;

// x viewed as [n_top 1024][n_mid 512][col 512] (col = lowest digit)
// pass-1 tile: cols [c0, c0+8), fixed n_mid, all n_top.  512 threads x 16.
// dst layouts: T (hbm variant): tile-contiguous; scratch (chunked): [k_top][n_mid][col - chunk0]
template <int CHUNKED>
__global__ __launch_bounds__(512) void p1(const d2* __restrict__ x, d2* __restrict__ dst, int ch, int chunk0) {
    const int tiles_per_mid = ch / 8;
    const int tile = blockIdx.x;
    const int n_mid = tile / tiles_per_mid, c0 = chunk0 + (tile % tiles_per_mid) * 8;
    d2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + k * 512, c = g & 7, r = g >> 3;  // r = n_top
        v[k] = __builtin_nontemporal_load(x + ((uint64_t)r << 18) + ((uint64_t)n_mid << 9) + c0 + c);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + k * 512, c = g & 7, r = g >> 3;
        if (CHUNKED) dst[((uint64_t)r * 512 + n_mid) * ch + (c0 - chunk0) + c] = v[k];
        else __builtin_nontemporal_store(v[k], dst + (uint64_t)tile * 8192 + g);
    }
}

// pass-2 tile: 16 columns, fixed k_top, all 512 n_mid; writes B with 256-B
// segments at a 2^19 stride ([k_mid][k_top][col]-like)
template <int CHUNKED>
__global__ __launch_bounds__(512) void p2(const d2* __restrict__ src, d2* __restrict__ out, int ch, int chunk0) {
    const int tiles_per_top = ch / 16;
    const int tile = blockIdx.x;
    const int k_top = tile / tiles_per_top, cc = (tile % tiles_per_top) * 16;
    d2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + k * 512, c = g & 15, r = g >> 4;  // r = n_mid
        if (CHUNKED) v[k] = src[((uint64_t)k_top * 512 + r) * ch + cc + c];
        else v[k] = __builtin_nontemporal_load(src + ((uint64_t)r << 19) + ((uint64_t)k_top << 9) + chunk0 + cc + c);
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + k * 512, c = g & 15, r = g >> 4;  // r = k_mid
        __builtin_nontemporal_store(v[k], out + ((uint64_t)r << 19) + ((uint64_t)k_top << 9) + chunk0 + cc + c);
    }
}

int main() {
    const uint64_t n = 1ull << 28;
    d2 *x, *t, *b, *sc;
    if (hipMalloc(&x, n * 16) || hipMalloc(&t, n * 16) || hipMalloc(&b, n * 16) || hipMalloc(&sc, 512ull << 20))
        return 1;
    (void)hipMemset(x, 0, n * 16);
    (void)hipMemset(t, 0, n * 16);
    (void)hipMemset(b, 0, n * 16);
    (void)hipMemset(sc, 0, 512ull << 20);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto timeit = [&](auto&& body) {
        body();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < 4; r++) body();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / 4;
    };
    // hbm: two full passes (the whole 512 columns as one "chunk")
    float m1 = timeit([&] { hipLaunchKernelGGL(p1<0>, dim3(512 * 64), dim3(512), 0, 0, x, t, 512, 0); });
    float m2 = timeit([&] { hipLaunchKernelGGL(p2<0>, dim3(1024 * 32), dim3(512), 0, 0, t, b, 512, 0); });
    printf("hbm\tpass1 %.3f ms (%.0f GB/s)\tpass2 %.3f ms (%.0f GB/s)\tsum %.3f ms\n", m1, 2.0 * n * 16 / m1 / 1e6, m2,
           2.0 * n * 16 / m2 / 1e6, m1 + m2);
    for (int ch = 8; ch <= 64; ch *= 2) {
        if (ch < 16) continue;  // pass-2 tiles need 16 columns
        const int nch = 512 / ch;
        float ms = timeit([&] {
            for (int c = 0; c < nch; c++) {
                hipLaunchKernelGGL(p1<1>, dim3(512 * (ch / 8)), dim3(512), 0, 0, x, sc, ch, c * ch);
                hipLaunchKernelGGL(p2<1>, dim3(1024 * (ch / 16)), dim3(512), 0, 0, sc, b, ch, c * ch);
            }
        });
        printf("chunked\t%d cols (%d MiB scratch)\t%.3f ms\tvs hbm %.3f ms\n", ch, ch * 8, ms, m1 + m2);
    }
    return 0;
}
