// tools/probe_pipe.hip -- standalone probe (not part of the product).
// Does software pipelining lift a big-tile strided pass above its one-tile-
// per-workgroup ceiling?  Copies with the exact index maps of the C4 passes
// (fp64 N = 2^28, radices 1024 / 512 / 512; 16-B elements):
//   p1: line j < 2^18 reads j + r 2^18 (r < 1024), writes j 1024 + r   (C = 8)
//   p2: line j < 2^19 reads j + r 2^19 (r < 512), writes (j>>10)<<19 + (j&1023) + r 1024   (C = 16)
//   p3: line j < 2^19 reads j + r 2^19, writes j + r 2^19   (C = 16)
// (and padded intermediate layouts: element e at e + (e >> s) p) in three forms:
//   once : one tile per workgroup, all loads then all stores (the k_pass shape;
//          70 KiB of dummy LDS keeps it at 2 workgroups per CU like k_pass)
//   loop : persistent workgroups (G per CU) walking tiles, same per-tile shape
//   pipe : persistent, double-buffered: tile t+1's loads are issued before
//          tile t's stores (2 x 16 values per thread in registers)
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_pipe.hip -o tools/probe_pipe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double __attribute__((ext_vector_type(2))) d2;

struct Map {
    int log_r, log_c, pass;  // R = 2^log_r, C = 2^log_c
    // padded layouts: element e of a side sits at e + (e >> s) p (p = 0: plain)
    int src_s, src_p, dst_s, dst_p;
};

__device__ __forceinline__ uint64_t padded(uint64_t e, int s, int p) { return e + (p ? (e >> s) * (uint64_t)p : 0); }

__device__ __forceinline__ void addr(const Map& m, uint64_t tile, int g, uint64_t& src, uint64_t& dst) {
    const int C = 1 << m.log_c;
    const int c = g & (C - 1), r = g >> m.log_c;
    const uint64_t j = tile * C + c;
    if (m.pass == 1) {
        src = j + ((uint64_t)r << 18);
        dst = (j << 10) + r;
    } else if (m.pass == 2) {
        src = j + ((uint64_t)r << 19);
        dst = ((j >> 10) << 19) + (j & 1023) + ((uint64_t)r << 10);
    } else if (m.pass == 3) {
        src = j + ((uint64_t)r << 19);
        dst = src;
    } else if (m.pass == 4) {  // two-pass 2^14 x 2^14, first pass: 16-B column gather, contiguous write
        src = j + ((uint64_t)r << 14);
        dst = (j << 14) + r;
    } else if (m.pass == 5) {  // two-pass, second pass: 16-B gather and 16-B scatter
        src = j + ((uint64_t)r << 14);
        dst = src;
    } else if (m.pass == 6) {  // "W" order, pass 1: as p1 in, out (n3, n2, k1): 16-KiB runs 8 MiB apart
        src = j + ((uint64_t)r << 18);
        dst = ((j & 511) << 19) + ((j >> 9) << 10) + r;
    } else if (m.pass == 7) {  // "W" order, passes 2 and 3: windowed read (rows 16 KiB apart), spread write (rows 8 MiB apart)
        src = ((j >> 10) << 19) + ((uint64_t)r << 10) + (j & 1023);
        dst = j + ((uint64_t)r << 19);
    } else {
        // the last pass of an all-8-worker plan at 2^28 (local 2^25 = 512 x 256
        // x 256, last R = 256, Ns = 2^17): tile -> (worker q, line block),
        // lines j < 2^17 of slice q read q 2^25 + j + r 2^17; written
        // slice-major (pass 8) or straight to natural order bitrev(q) + 8 (j +
        // r 2^17) (pass 9: 16-B pieces 128 B apart, the 8 workers' tiles of a
        // line block consecutive, i.e. one XCD group)
        const uint64_t q = tile & 7, jb = tile >> 3;
        const uint64_t jj = jb * C + c;
        const uint64_t rq = ((q & 1) << 2) | (q & 2) | ((q >> 2) & 1);
        src = (q << 25) + jj + ((uint64_t)r << 17);
        dst = m.pass == 8 ? src : rq + ((jj + ((uint64_t)r << 17)) << 3);
    }
    src = padded(src, m.src_s, m.src_p);
    dst = padded(dst, m.dst_s, m.dst_p);
}

__device__ uint32_t g_log_xg = 2;
__device__ __forceinline__ uint64_t xcd_tile(uint32_t b, uint32_t nblocks) {
    const uint32_t log_xg = g_log_xg;
    if (nblocks & ((8u << log_xg) - 1)) return b;
    const uint32_t xcd = b & 7, slot = b >> 3, gmask = (1u << log_xg) - 1;
    return ((uint64_t)(slot >> log_xg) << (log_xg + 3)) + ((uint64_t)xcd << log_xg) + (slot & gmask);
}

template <int NT>
__global__ __launch_bounds__(NT, 1024 / NT) void k_once(const d2* __restrict__ in, d2* __restrict__ out, Map m) {
    extern __shared__ d2 dummy[];
    const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    d2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint64_t s, d;
        addr(m, tile, threadIdx.x + k * NT, s, d);
        v[k] = __builtin_nontemporal_load(in + s);
    }
    if (threadIdx.x == 4095) dummy[0] = v[0];  // never true: keeps the LDS allocation
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint64_t s, d;
        addr(m, tile, threadIdx.x + k * NT, s, d);
        __builtin_nontemporal_store(v[k], out + d);
    }
}

template <int NT>
__global__ __launch_bounds__(NT, 1024 / NT) void k_once_plain(const d2* __restrict__ in, d2* __restrict__ out, Map m) {
    extern __shared__ d2 dummy[];
    const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);
    d2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint64_t s, d;
        addr(m, tile, threadIdx.x + k * NT, s, d);
        v[k] = __builtin_nontemporal_load(in + s);
    }
    if (threadIdx.x == 4095) dummy[0] = v[0];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint64_t s, d;
        addr(m, tile, threadIdx.x + k * NT, s, d);
        out[d] = v[k];
    }
}

// tiles of one persistent workgroup: blockIdx + i gridDim, in the XCD-aware order
__global__ __launch_bounds__(512, 1) void k_loop(const d2* __restrict__ in, d2* __restrict__ out, Map m,
                                                 uint32_t ntiles) {
    for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t tile = xcd_tile(t, ntiles);
        d2 v[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            uint64_t s, d;
            addr(m, tile, threadIdx.x + k * 512, s, d);
            v[k] = __builtin_nontemporal_load(in + s);
        }
#pragma unroll
        for (int k = 0; k < 16; k++) {
            uint64_t s, d;
            addr(m, tile, threadIdx.x + k * 512, s, d);
            __builtin_nontemporal_store(v[k], out + d);
        }
    }
}

__global__ __launch_bounds__(512, 1) void k_pipe(const d2* __restrict__ in, d2* __restrict__ out, Map m,
                                                 uint32_t ntiles) {
    d2 a[16], b[16];
    uint32_t t = blockIdx.x;
    if (t >= ntiles) return;
    uint64_t tile = xcd_tile(t, ntiles);
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint64_t s, d;
        addr(m, tile, threadIdx.x + k * 512, s, d);
        a[k] = __builtin_nontemporal_load(in + s);
    }
    while (true) {
        const uint32_t tn = t + gridDim.x;
        const uint64_t tilen = xcd_tile(tn < ntiles ? tn : t, ntiles);
        if (tn < ntiles) {
#pragma unroll
            for (int k = 0; k < 16; k++) {
                uint64_t s, d;
                addr(m, tilen, threadIdx.x + k * 512, s, d);
                b[k] = __builtin_nontemporal_load(in + s);
            }
        }
#pragma unroll
        for (int k = 0; k < 16; k++) {
            uint64_t s, d;
            addr(m, tile, threadIdx.x + k * 512, s, d);
            __builtin_nontemporal_store(a[k], out + d);
        }
        if (tn >= ntiles) break;
        t = tn;
        tile = tilen;
#pragma unroll
        for (int k = 0; k < 16; k++) a[k] = b[k];
    }
}

int main() {
    const uint64_t n = 1ull << 28;
    d2 *x, *y;
    if (hipMalloc(&x, n * 17) || hipMalloc(&y, n * 17)) return 1;  // room for padded layouts
    (void)hipMemset(x, 0, n * 17);
    (void)hipMemset(y, 0, n * 17);
    (void)hipFuncSetAttribute((const void*)k_once<512>, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
    (void)hipFuncSetAttribute((const void*)k_once<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, 140 * 1024);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
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
    // (padded layouts, profiles/r02_probe_pipe.log: no gain.)  Two-pass 2^14 x
    // 2^14: one 16384-value column per workgroup (1024 threads), 16-B accesses
    // on the column side; 8 (or 2^xg) adjacent columns on one XCD share lines
    // through its L2.  Against the three-pass copies of the same box.
    // (A vs W layout orders: profiles/r02_probe_pipe.log.)  The last pass of an
    // all-worker plan written slice-major (then a separate interleave pass)
    // vs straight into natural order; plain and nt stores; XCD groups of 8
    // (k_once loads 16 values x 512 threads = 8192 per tile: only R x C = 8192 maps)
    const Map maps[] = {{8, 5, 8, 0, 0, 0, 0}, {8, 5, 9, 0, 0, 0, 0}};
    for (int round = 0; round < 3; round++) {
        for (uint32_t xg : {2u, 3u}) {
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_log_xg), &xg, 4);
            for (const Map& m : maps) {
                const uint32_t ntiles = (uint32_t)(n >> (m.log_r + m.log_c));
                const float t = time([&] { hipLaunchKernelGGL(k_once<512>, dim3(ntiles), dim3(512), 72 * 1024, 0, x, y, m); });
                const float tp = time([&] { hipLaunchKernelGGL(k_once_plain<512>, dim3(ntiles), dim3(512), 72 * 1024, 0, x, y, m); });
                printf("round %d xg %u R=%d C=%d %s: nt %.3f ms %.0f GB/s   plain stores %.3f ms %.0f GB/s\n", round, xg,
                       1 << m.log_r, 1 << m.log_c, m.pass == 8 ? "slice-major" : "natural   ", t, 2.0 * n * 16 / t / 1e6,
                       tp, 2.0 * n * 16 / tp / 1e6);
            }
        }
        fflush(stdout);
    }
    if (hipGetLastError() != hipSuccess) return 2;
    return 0;
}
