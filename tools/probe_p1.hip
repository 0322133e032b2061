// tools/probe_p1.hip -- standalone probe (not part of the product): which side
// limits the C4 first pass (fp64 N = 2^28, R = 1024, C = 8: line j < 2^18 reads
// j + r 2^18 for r < 1024 -- 128-B row segments -- and writes j 1024 + r,
// contiguous)?  Round-3 verdict item 7.  Kernels, all with the k_pass tile
// (8192 values, 512 threads x 16, 70 KiB of LDS held so 2 workgroups fit per
// CU, XCD-grouped tiles) unless noted:
//   copy   : the pass's loads and stores (its copy ceiling, 1.70 ms in round 2)
//   read   : the loads only (a dependent-free sum; nothing stored)
//   write  : the stores only (no loads)
//   lds    : the read side through direct-to-LDS loads (global_load_lds_dwordx4:
//            HBM -> LDS without VGPRs), half tiles (8 lines x 512 rows, 64 KiB
//            of LDS) so 2 workgroups fit per CU; stores from LDS
//   half   : the same half tile through registers (8 values per thread)
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_p1.hip -o tools/probe_p1
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <vector>

typedef double __attribute__((ext_vector_type(2))) d2;
#define LDS_AS __attribute__((address_space(3)))

constexpr int LOG_STRIDE = 18;  // M / R at 2^28, R = 1024
constexpr int C = 8;

__device__ __forceinline__ uint64_t xcd_tile(uint32_t b, uint32_t nblocks) {
    const uint32_t log_xg = 2;
    if (nblocks & ((8u << log_xg) - 1)) return b;
    const uint32_t xcd = b & 7, slot = b >> 3, gmask = (1u << log_xg) - 1;
    return ((uint64_t)(slot >> log_xg) << (log_xg + 3)) + ((uint64_t)xcd << log_xg) + (slot & gmask);
}

// element g (< 8192) of tile t: line c = g % 8, row r = g / 8 (c-fast, as the
// k_pass strided side)
__device__ __forceinline__ void addr(uint64_t tile, int g, int rows_log, uint64_t& src, uint64_t& dst) {
    const int c = g & (C - 1), r = g >> 3;
    const uint64_t j = tile * C + c;
    src = j + ((uint64_t)r << LOG_STRIDE);
    dst = (j << 10) + r;
    (void)rows_log;
}

__global__ __launch_bounds__(512, 2) void k_copy(const d2* __restrict__ in, d2* __restrict__ out) {
    extern __shared__ d2 dummy[];
    const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    d2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint64_t s, d;
        addr(tile, threadIdx.x + k * 512, 10, s, d);
        v[k] = __builtin_nontemporal_load(in + s);
    }
    if (threadIdx.x == 4095) dummy[0] = v[0];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint64_t s, d;
        addr(tile, threadIdx.x + k * 512, 10, s, d);
        __builtin_nontemporal_store(v[k], out + d);
    }
}

__global__ __launch_bounds__(512, 2) void k_read(const d2* __restrict__ in, d2* __restrict__ out) {
    extern __shared__ d2 dummy[];
    const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    d2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint64_t s, d;
        addr(tile, threadIdx.x + k * 512, 10, s, d);
        v[k] = __builtin_nontemporal_load(in + s);
    }
    d2 acc = v[0];
#pragma unroll
    for (int k = 1; k < 16; k++) acc += v[k];
    if (acc.x == 1234.5678) out[blockIdx.x * 512 + threadIdx.x] = acc;  // never: keeps the loads
    if (threadIdx.x == 4095) dummy[0] = acc;
}

__global__ __launch_bounds__(512, 2) void k_write(const d2* __restrict__ in, d2* __restrict__ out) {
    extern __shared__ d2 dummy[];
    const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const d2 val = {(double)threadIdx.x, (double)blockIdx.x};
    if (threadIdx.x == 4095) dummy[0] = val;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint64_t s, d;
        addr(tile, threadIdx.x + k * 512, 10, s, d);
        __builtin_nontemporal_store(val, out + d);
    }
    (void)in;
}

// half tile (8 lines x 512 rows = 4096 values, 64 KiB): rows [0, 512) of the
// tile's lines for even blocks, [512, 1024) for odd blocks
__global__ __launch_bounds__(512, 2) void k_half(const d2* __restrict__ in, d2* __restrict__ out) {
    extern __shared__ d2 dummy[];
    const uint64_t tile = xcd_tile(blockIdx.x >> 1, gridDim.x >> 1);
    const int r0 = (blockIdx.x & 1) * 512;
    d2 v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int g = threadIdx.x + k * 512, c = g & 7, r = r0 + (g >> 3);
        const uint64_t j = tile * C + c;
        v[k] = __builtin_nontemporal_load(in + j + ((uint64_t)r << LOG_STRIDE));
    }
    if (threadIdx.x == 4095) dummy[0] = v[0];
#pragma unroll
    for (int k = 0; k < 8; k++) {
        // store side: lanes along a line (contiguous 16-B runs of the output)
        const int g = threadIdx.x + k * 512, c = g >> 9, r = r0 + (g & 511);
        const uint64_t j = tile * C + c;
        (void)c;
        __builtin_nontemporal_store(v[k], out + (j << 10) + r);
    }
}

// the same half tile through direct-to-LDS loads: wave w, issue k loads rows
// 8 (8 w + k) .. +7 (64 lanes = 8 rows x 8 lines, 16 B each) into LDS at
// (8 w + k) 64 + lane; then lanes along a line read their values from LDS
__global__ __launch_bounds__(512, 2) void k_lds(const d2* __restrict__ in, d2* __restrict__ out) {
    __shared__ d2 tile_lds[4096];
    const uint64_t tile = xcd_tile(blockIdx.x >> 1, gridDim.x >> 1);
    const int r0 = (blockIdx.x & 1) * 512;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int blk = 8 * w + k;               // 64-value block: rows 8 blk .. 8 blk + 7
        const int c = lane & 7, r = r0 + 8 * blk + (lane >> 3);
        const uint64_t j = tile * C + c;
        __builtin_amdgcn_global_load_lds((const void*)(in + j + ((uint64_t)r << LOG_STRIDE)),
                                         (LDS_AS void*)(tile_lds + blk * 64), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0): this wave's LDS loads have landed
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const int g = threadIdx.x + k * 512, c = g >> 9, rr = g & 511;  // row rr of line c
        const d2 v = tile_lds[rr * 8 + c];
        const uint64_t j = tile * C + c;
        __builtin_nontemporal_store(v, out + (j << 10) + r0 + rr);
    }
}

int main() {
    const uint64_t n = 1ull << 28;
    d2 *x, *y;
    if (hipMalloc(&x, n * 16) || hipMalloc(&y, n * 16)) return 1;
    (void)hipMemset(x, 0, n * 16);
    (void)hipMemset(y, 0, n * 16);
    const size_t dyn = 70 * 1024;
    for (const void* f : {(const void*)k_copy, (const void*)k_read, (const void*)k_write, (const void*)k_half})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const uint32_t tiles = (uint32_t)((n >> 10) / C);  // 2^15 tiles of 8192 values
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
    const double gb = 2.0 * n * 16 * 1e-9, gb1 = n * 16 * 1e-9;
    for (int rep = 0; rep < 2; rep++) {
        float t;
        t = time([&] { hipLaunchKernelGGL(k_copy, dim3(tiles), dim3(512), dyn, 0, x, y); });
        printf("copy  (read + write, 8192-value tile)  %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
        t = time([&] { hipLaunchKernelGGL(k_read, dim3(tiles), dim3(512), dyn, 0, x, y); });
        printf("read  (loads only)                     %.3f ms  %.0f GB/s (read bytes)\n", t, gb1 / t * 1e3);
        t = time([&] { hipLaunchKernelGGL(k_write, dim3(tiles), dim3(512), dyn, 0, x, y); });
        printf("write (stores only)                    %.3f ms  %.0f GB/s (written bytes)\n", t, gb1 / t * 1e3);
        t = time([&] { hipLaunchKernelGGL(k_half, dim3(2 * tiles), dim3(512), dyn, 0, x, y); });
        printf("half  (8 x 512 tile via registers)     %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
        t = time([&] { hipLaunchKernelGGL(k_lds, dim3(2 * tiles), dim3(512), 0, 0, x, y); });
        printf("lds   (8 x 512 tile, direct-to-LDS)    %.3f ms  %.0f GB/s\n", t, gb / t * 1e3);
    }
    // k_lds correctness on a few elements (the copy must be exact)
    std::vector<d2> h(4096);
    for (uint64_t i = 0; i < 4096; i++) h[i] = d2{(double)i, -(double)i};
    (void)hipMemcpy(x, h.data(), 4096 * 16, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_lds, dim3(2 * tiles), dim3(512), 0, 0, x, y);
    d2 o;
    (void)hipMemcpy(&o, y + 5 * 1024, 16, hipMemcpyDeviceToHost);  // line 5, row 0 <- x[5]
    printf("lds copy check: y[5*1024] = (%g, %g), want (5, -5)\n", o.x, o.y);
    return 0;
}
