// tools/probe_copy.hip -- standalone probe (not part of the product).
// What does a plain 4 GiB HBM copy reach on this MI355X, and with which
// shape?  Varies per-thread unroll U (16-B accesses in flight per lane),
// workgroup size, grid (persistent grid-stride vs one tile per workgroup),
// non-temporal hints; also read-only and write-only.
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_copy.hip -o tools/probe_copy
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float __attribute__((ext_vector_type(4))) f4;

template <int U, bool NT>
__device__ __forceinline__ f4 ld(const f4* p) { return NT ? __builtin_nontemporal_load(p) : *p; }
template <int U, bool NT>
__device__ __forceinline__ void st(f4* p, f4 v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// one tile of U*blockDim elements per workgroup (no grid-stride)
template <int U, bool NT, int MODE>  // MODE 0 copy, 1 read, 2 write
__global__ void tile_k(const f4* __restrict__ in, f4* __restrict__ out, uint64_t n) {
    const uint64_t base = (uint64_t)blockIdx.x * blockDim.x * U + threadIdx.x;
    f4 v[U];
    if (MODE != 2) {
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ld<U, NT>(in + base + (uint64_t)u * blockDim.x);
    } else {
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = f4{(float)u, 0, 0, 0};
    }
    if (MODE == 1) {
        float s = 0;
#pragma unroll
        for (int u = 0; u < U; u++) s += v[u].x;
        if (s == 1234.5f) out[0] = v[0];
        return;
    }
#pragma unroll
    for (int u = 0; u < U; u++) st<U, NT>(out + base + (uint64_t)u * blockDim.x, v[u]);
}

// one tile per workgroup, at most W loads in flight per lane (sliding window):
// does a 128-KiB tile copy gain from fewer bytes in flight chip-wide?
#define PC_STR2(x) #x
#define PC_STR(x) PC_STR2(x)
template <int U, int W>
__global__ void tile_win_k(const f4* __restrict__ in, f4* __restrict__ out, uint64_t n) {
    const uint64_t base = (uint64_t)blockIdx.x * blockDim.x * U + threadIdx.x;
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        v[u] = __builtin_nontemporal_load(in + base + (uint64_t)u * blockDim.x);
        if constexpr (W == 1) { if (u < U - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
        if constexpr (W == 2) { if (u >= 1 && u < U - 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); }
        if constexpr (W == 4) { if (u >= 3 && u < U - 1) asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); }
        if constexpr (W == 8) { if (u >= 7 && u < U - 1) asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); }
    }
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_nontemporal_store(v[u], out + base + (uint64_t)u * blockDim.x);
}

// persistent grid-stride
template <int U, bool NT>
__global__ void gs_k(const f4* __restrict__ in, f4* __restrict__ out, uint64_t n) {
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x * U;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x * U + threadIdx.x; base < n; base += step) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = ld<U, NT>(in + base + (uint64_t)u * blockDim.x);
#pragma unroll
        for (int u = 0; u < U; u++) st<U, NT>(out + base + (uint64_t)u * blockDim.x, v[u]);
    }
}

int main() {
    const uint64_t S = 1ull << 32, n = S / 16;
    f4 *A, *B;
    if (hipMalloc(&A, S) || hipMalloc(&B, S)) return 1;
    (void)hipMemset(A, 0, S);
    (void)hipMemset(B, 0, S);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto timeit = [&](auto&& body) {
        body();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < 5; r++) body();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms / 5;
    };
#define TILE(U, NT, MODE, BS)                                                                                 \
    {                                                                                                         \
        const unsigned grid = (unsigned)(n / ((uint64_t)BS * U));                                             \
        float ms = timeit([&] { hipLaunchKernelGGL((tile_k<U, NT, MODE>), dim3(grid), dim3(BS), 0, 0, A, B, n); }); \
        const double by = (MODE == 0 ? 2.0 : 1.0) * S;                                                        \
        printf("tile\tU=%d\tnt=%d\tmode=%d\tbs=%d\t%.3f ms\t%.0f GB/s\n", U, NT, MODE, BS, ms, by / ms / 1e6);  \
    }
#define GS(U, NT, BS, G)                                                                                      \
    {                                                                                                         \
        float ms = timeit([&] { hipLaunchKernelGGL((gs_k<U, NT>), dim3(G), dim3(BS), 0, 0, A, B, n); });      \
        printf("gs\tU=%d\tnt=%d\tgrid=%d\tbs=%d\t%.3f ms\t%.0f GB/s\n", U, NT, G, BS, ms, 2.0 * S / ms / 1e6);   \
    }
    TILE(1, 0, 0, 256) TILE(2, 0, 0, 256) TILE(4, 0, 0, 256) TILE(8, 0, 0, 256) TILE(16, 0, 0, 256)
    TILE(1, 1, 0, 256) TILE(2, 1, 0, 256) TILE(4, 1, 0, 256) TILE(8, 1, 0, 256) TILE(16, 1, 0, 256)
    TILE(4, 0, 0, 512) TILE(4, 1, 0, 512) TILE(8, 1, 0, 512) TILE(16, 1, 0, 512) TILE(4, 1, 0, 1024)
    TILE(4, 0, 1, 256) TILE(4, 1, 1, 256) TILE(16, 1, 1, 256) TILE(4, 0, 2, 256) TILE(4, 1, 2, 256) TILE(16, 1, 2, 256)
    GS(4, 0, 256, 1024) GS(4, 1, 256, 1024) GS(4, 1, 256, 2048) GS(4, 1, 256, 4096) GS(8, 1, 256, 2048)
    GS(4, 1, 512, 2048) GS(16, 1, 256, 1024) GS(4, 1, 1024, 1024)
#define WIN(U, W, BS)                                                                                         \
    {                                                                                                         \
        const unsigned grid = (unsigned)(n / ((uint64_t)BS * U));                                             \
        float ms = timeit([&] { hipLaunchKernelGGL((tile_win_k<U, W>), dim3(grid), dim3(BS), 0, 0, A, B, n); }); \
        printf("win\tU=%d\tW=%d\tbs=%d\t%.3f ms\t%.0f GB/s\n", U, W, BS, ms, 2.0 * S / ms / 1e6);               \
    }
    WIN(16, 16, 512) WIN(16, 8, 512) WIN(16, 4, 512) WIN(16, 2, 512) WIN(16, 1, 512) WIN(16, 16, 512)
    TILE(1, 1, 0, 256)
    return 0;
}
