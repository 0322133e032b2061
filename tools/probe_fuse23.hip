// tools/probe_fuse23.hip -- standalone probe (not part of the product).
// Can passes 2 and 3 of the C4 plan (fp64 2^28, radices 1024 / 512 / 512)
// hand their intermediate over through the 256 MiB Infinity Cache instead of
// HBM?  After pass 1 the transform is 1024 independent 2^18-point
// sub-transforms, one per k1 (the first radix's output index), interleaved at
// a 16-B granule.  Copies with the exact index maps of passes 2 and 3 (R = 512,
// C = 16, 512 threads x 16 values, 2 workgroups per CU like k_pass):
//   full    : pass 2 over the whole array, then pass 3 (the product today)
//   grouped : for each group of K consecutive k1 (K x 4 MiB): pass 2 of the
//             group into a compact scratch slot (K x 16-B pieces), then pass 3
//             of the group from that slot -- the slot is re-read while it is
//             still in the Infinity Cache
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_fuse23.hip -o tools/probe_fuse23
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double __attribute__((ext_vector_type(2))) d2;

struct Map {
    int kind;   // 2 / 3 full passes; 12 / 13 grouped pass 2 / pass 3
    int log_k;  // group: K = 2^log_k consecutive k1
    uint32_t g; // group index
    int scratch_nt;
};

__device__ __forceinline__ void addr(const Map& m, uint64_t tile, int s, uint64_t& src, uint64_t& dst) {
    const int c = s & 15, r = s >> 4;
    const uint64_t jl = tile * 16 + c;
    if (m.kind == 2) {
        src = jl + ((uint64_t)r << 19);
        dst = ((jl >> 10) << 19) + (jl & 1023) + ((uint64_t)r << 10);
    } else if (m.kind == 3) {
        src = jl + ((uint64_t)r << 19);
        dst = src;
    } else {
        const uint64_t K = 1ull << m.log_k;
        const uint64_t k1 = jl & (K - 1), hi = jl >> m.log_k;  // hi = n2 (low part of n2 in pass 2)
        const uint64_t j = (hi << 10) + (uint64_t)m.g * K + k1;
        if (m.kind == 12) {
            src = j + ((uint64_t)r << 19);
            dst = ((hi * 512 + r) << m.log_k) + k1;  // compact scratch
        } else {
            src = (((uint64_t)r * 512 + hi) << m.log_k) + k1;
            dst = j + ((uint64_t)r << 19);
        }
    }
}

__device__ __forceinline__ uint64_t xcd_tile(uint32_t b, uint32_t nblocks) {
    const uint32_t log_xg = 2;
    if (nblocks & ((8u << log_xg) - 1)) return b;
    const uint32_t xcd = b & 7, slot = b >> 3, gmask = (1u << log_xg) - 1;
    return ((uint64_t)(slot >> log_xg) << (log_xg + 3)) + ((uint64_t)xcd << log_xg) + (slot & gmask);
}

__device__ __forceinline__ void copy_tile(const d2* __restrict__ in, d2* __restrict__ out, const Map& m,
                                          uint64_t tile, d2* dummy) {
    d2 v[16];
    const bool nt_in = m.kind != 13 || m.scratch_nt == 1, nt_out = m.kind != 12 || m.scratch_nt == 1;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint64_t s, d;
        addr(m, tile, threadIdx.x + k * 512, s, d);
        v[k] = nt_in ? __builtin_nontemporal_load(in + s) : in[s];
    }
    if (threadIdx.x == 4095) dummy[0] = v[0];  // never true: keeps the LDS allocation
#pragma unroll
    for (int k = 0; k < 16; k++) {
        uint64_t s, d;
        addr(m, tile, threadIdx.x + k * 512, s, d);
        if (m.scratch_nt == 2 && m.kind == 12)  // write-through (sc1) scratch stores
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(out + d), "v"(v[k]) : "memory");
        else if (nt_out)
            __builtin_nontemporal_store(v[k], out + d);
        else
            out[d] = v[k];
    }
}

__global__ __launch_bounds__(512, 2) void k_copy(const d2* __restrict__ in, d2* __restrict__ out, Map m) {
    extern __shared__ d2 dummy[];
    copy_tile(in, out, m, xcd_tile(blockIdx.x, gridDim.x), dummy);
}

// two independent halves in one launch: blocks [0, na) copy with map a, the
// rest with map b (the skewed pipeline: pass 3 of group g beside pass 2 of g+1)
__global__ __launch_bounds__(512, 2) void k_copy2(const d2* __restrict__ ia, d2* __restrict__ oa, Map a,
                                                  const d2* __restrict__ ib, d2* __restrict__ ob, Map b, uint32_t na,
                                                  int interleave) {
    extern __shared__ d2 dummy[];
    const uint32_t nb = gridDim.x - na;
    uint32_t blk = blockIdx.x;
    bool first;
    if (interleave) {  // alternate halves by groups of 8 blocks (one per XCD)
        first = ((blk >> 3) & 1) == 0;
        blk = ((blk >> 4) << 3) + (blk & 7);
    } else {
        first = blk < na;
        if (!first) blk -= na;
    }
    if (first)
        copy_tile(ia, oa, a, xcd_tile(blk, na), dummy);
    else
        copy_tile(ib, ob, b, xcd_tile(blk, nb), dummy);
}

// One launch for all of passes 2 and 3, in skewed group order, workgroups
// taking tickets (one per workgroup, in the order they start): block k of T
// tickets is pass 2 or pass 3 of one group (blk_kind / blk_group).  A pass-3
// tile waits until the T pass-2 tiles of its group have published
// (plain stores, release fence, counter); a pass-2 tile reusing a slot waits
// until the pass-3 tiles that read it have finished.  Every wait is on
// smaller tickets (running or done), polls are capped (err flag) so the grid
// always drains.
__device__ uint32_t g_ticket, g_err;
__device__ uint32_t g_cnt2[64], g_cnt3[64];

__device__ __forceinline__ void wait_count(uint32_t* c, uint32_t want) {
    uint32_t it = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        __builtin_amdgcn_s_sleep(2);
        if (++it > (1u << 22)) {
            __hip_atomic_fetch_add(&g_err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
    }
}

__global__ __launch_bounds__(512, 2) void k_pipe23(const d2* __restrict__ x, d2* __restrict__ y, d2* sc,
                                                   uint64_t slot, const int* blk_kind, const int* blk_group,
                                                   int log_k, uint32_t T, int nslots, int wt) {
    extern __shared__ d2 dummy[];
    __shared__ uint32_t sh_t;
    if (threadIdx.x == 0) sh_t = __hip_atomic_fetch_add(&g_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const uint32_t t = sh_t, blk = t / T, within = t % T;
    const int kind = blk_kind[blk];
    const uint32_t g = (uint32_t)blk_group[blk];
    d2* sl = sc + (uint64_t)(g % nslots) * slot;
    const uint64_t tile = xcd_tile(within, T);
    const Map m{kind, log_k, g, wt};
    if (kind == 12) {
        if (g >= (uint32_t)nslots) {
            if (threadIdx.x == 0) wait_count(&g_cnt3[g - nslots], T);
            __syncthreads();
        }
        copy_tile(x, sl, m, tile, dummy);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(&g_cnt2[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    } else {
        if (threadIdx.x == 0) {
            wait_count(&g_cnt2[g], T);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        copy_tile(sl, y, m, tile, dummy);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(&g_cnt3[g], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ unsigned long long g_diff;
__global__ void k_diff(const d2* a, const d2* b, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const d2 u = a[i], v = b[i];
        if (u.x != v.x || u.y != v.y) atomicAdd(&g_diff, 1ull);
    }
}
__global__ void k_fill(d2* a, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        a[i] = d2{(double)i, -(double)i};
}

int main() {
    const uint64_t n = 1ull << 28;
    d2 *x, *y, *sc, *ref;
    const uint64_t slot = (1ull << 18) * 64;  // up to K = 64
    if (hipMalloc(&x, n * 16) || hipMalloc(&y, n * 16) || hipMalloc(&sc, 3 * slot * 16) || hipMalloc(&ref, n * 16)) return 1;
    (void)hipMemset(x, 0, n * 16);
    (void)hipMemset(y, 0, n * 16);
    (void)hipMemset(sc, 0, 3 * slot * 16);
    hipStream_t sa, sb;
    (void)hipStreamCreateWithFlags(&sa, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&sb, hipStreamNonBlocking);
    hipEvent_t ev2[64], ev3[64], eg0, eg1;
    for (int i = 0; i < 64; i++) {
        (void)hipEventCreateWithFlags(&ev2[i], hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&ev3[i], hipEventDisableTiming);
    }
    (void)hipEventCreate(&eg0);
    (void)hipEventCreate(&eg1);
    (void)hipFuncSetAttribute((const void*)k_copy, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
    (void)hipFuncSetAttribute((const void*)k_copy2, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
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

    (void)hipFuncSetAttribute((const void*)k_pipe23, hipFuncAttributeMaxDynamicSharedMemorySize, 72 * 1024);
    {
        // correctness of the one-launch pipeline: same permutation as the grouped launches
        hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, n);
        (void)hipDeviceSynchronize();
    }
    const uint32_t full_tiles = (uint32_t)(n / 8192);
    const double bytes = 2.0 * 2.0 * n * 16;  // two passes, read + write
    for (int round = 0; round < 3; round++) {
        const float tf = time([&] {
            hipLaunchKernelGGL(k_copy, dim3(full_tiles), dim3(512), 72 * 1024, 0, x, y, Map{2, 0, 0, 0});
            hipLaunchKernelGGL(k_copy, dim3(full_tiles), dim3(512), 72 * 1024, 0, y, x, Map{3, 0, 0, 0});
        });
        printf("round %d full passes 2+3: %.3f ms (%.0f GB/s of pass bytes)\n", round, tf, bytes / tf / 1e6);
        for (int log_k : {4, 5}) {
            for (int nslots : {2, 3}) for (int wt : {0}) {  // (wt 2: sc1 inline-asm scratch stores -- miscompared, void)
                const uint32_t groups = 1024u >> log_k, T = (uint32_t)((1ull << 18 << log_k) / 8192);
                // block order: p2(0), p2(1), then p3(g), p2(g + 2) ...
                int hk[256], hg[256], nb = 0;
                hk[nb] = 12; hg[nb++] = 0;
                hk[nb] = 12; hg[nb++] = 1;
                for (uint32_t g = 0; g < groups; g++) {
                    hk[nb] = 13; hg[nb++] = (int)g;
                    if (g + 2 < groups) { hk[nb] = 12; hg[nb++] = (int)g + 2; }
                }
                int *dk, *dg;
                (void)hipMalloc(&dk, sizeof(hk));
                (void)hipMalloc(&dg, sizeof(hg));
                (void)hipMemcpy(dk, hk, sizeof(hk), hipMemcpyHostToDevice);
                (void)hipMemcpy(dg, hg, sizeof(hg), hipMemcpyHostToDevice);
                uint32_t *pt, *pc2, *pc3, *perr;
                (void)hipGetSymbolAddress((void**)&pt, HIP_SYMBOL(g_ticket));
                (void)hipGetSymbolAddress((void**)&pc2, HIP_SYMBOL(g_cnt2));
                (void)hipGetSymbolAddress((void**)&pc3, HIP_SYMBOL(g_cnt3));
                (void)hipGetSymbolAddress((void**)&perr, HIP_SYMBOL(g_err));
                auto launch = [&] {
                    (void)hipMemsetAsync(pt, 0, 4, 0);
                    (void)hipMemsetAsync(pc2, 0, 256, 0);
                    (void)hipMemsetAsync(pc3, 0, 256, 0);
                    hipLaunchKernelGGL(k_pipe23, dim3(nb * T), dim3(512), 72 * 1024, 0, x, y, sc, slot, dk, dg, log_k, T,
                                       nslots, wt);
                };
                // check: the pipeline's y against the grouped launches' (launch boundaries as the
                // hand-off), once idle and once after the timed runs
                auto check = [&](const char* when) {
                    for (uint32_t g = 0; g < groups; g++) {
                        d2* sl = sc + (g & 1) * slot;
                        hipLaunchKernelGGL(k_copy, dim3(T), dim3(512), 72 * 1024, 0, x, sl, Map{12, log_k, g, 0});
                        hipLaunchKernelGGL(k_copy, dim3(T), dim3(512), 72 * 1024, 0, sl, ref, Map{13, log_k, g, 0});
                    }
                    (void)hipMemset(y, 0, n * 16);
                    launch();
                    unsigned long long zero = 0, diff = 0;
                    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_diff), &zero, 8);
                    hipLaunchKernelGGL(k_diff, dim3(4096), dim3(256), 0, 0, y, ref, n);
                    (void)hipMemcpyFromSymbol(&diff, HIP_SYMBOL(g_diff), 8);
                    printf("round %d one-launch pipeline K=%d, %d slots: check (%s): %llu of %llu elements differ\n", round,
                           1 << log_k, nslots, when, diff, (unsigned long long)n);
                };
                (void)hipMemset(perr, 0, 4);
                check("idle");
                const float tp = time(launch);
                uint32_t err = 0;
                (void)hipMemcpy(&err, perr, 4, hipMemcpyDeviceToHost);
                printf("round %d one-launch pipeline K=%d, %d slots, scratch stores %s: %.3f ms (%.0f GB/s of pass bytes), poll caps hit %u\n",
                       round, 1 << log_k, nslots, wt ? "sc1" : "plain", tp, bytes / tp / 1e6, err);
                check("after timing");
                (void)hipFree(dk);
                (void)hipFree(dg);
            }
        }

        for (int log_k : {4, 5, 6}) {
            for (int snt : {0, 1}) {
                const uint32_t groups = 1024u >> log_k, tiles = (uint32_t)((1ull << 18 << log_k) / 8192);
                const float tg = time([&] {
                    for (uint32_t g = 0; g < groups; g++) {
                        d2* s = sc + (g & 1) * slot;
                        hipLaunchKernelGGL(k_copy, dim3(tiles), dim3(512), 72 * 1024, 0, x, s, Map{12, log_k, g, snt});
                        hipLaunchKernelGGL(k_copy, dim3(tiles), dim3(512), 72 * 1024, 0, s, y, Map{13, log_k, g, snt});
                    }
                });
                const float t2 = time([&] {
                    for (uint32_t g = 0; g < groups; g++)
                        hipLaunchKernelGGL(k_copy, dim3(tiles), dim3(512), 72 * 1024, 0, x, sc + (g & 1) * slot,
                                           Map{12, log_k, g, snt});
                });
                const float t3 = time([&] {
                    for (uint32_t g = 0; g < groups; g++)
                        hipLaunchKernelGGL(k_copy, dim3(tiles), dim3(512), 72 * 1024, 0, sc + (g & 1) * slot, y,
                                           Map{13, log_k, g, snt});
                });
                float tk[2];
                for (int il = 0; il < 2; il++)
                    tk[il] = time([&] {
                        // launch g: pass 3 of group g - 1 beside pass 2 of group g (slots alternate)
                        for (uint32_t g = 0; g <= groups; g++) {
                            d2* sp = sc + (g & 1) * slot;        // written by pass 2 of g
                            d2* sq = sc + ((g + 1) & 1) * slot;  // read by pass 3 of g - 1
                            if (g == 0)
                                hipLaunchKernelGGL(k_copy, dim3(tiles), dim3(512), 72 * 1024, 0, x, sp,
                                                   Map{12, log_k, g, snt});
                            else if (g == groups)
                                hipLaunchKernelGGL(k_copy, dim3(tiles), dim3(512), 72 * 1024, 0, sq, y,
                                                   Map{13, log_k, g - 1, snt});
                            else
                                hipLaunchKernelGGL(k_copy2, dim3(2 * tiles), dim3(512), 72 * 1024, 0, sq, y,
                                                   Map{13, log_k, g - 1, snt}, x, sp, Map{12, log_k, g, snt}, tiles,
                                                   il);
                        }
                    });
                float ts[2];
                for (int ns = 2; ns <= 3; ns++) {
                    // two streams: pass 2 of each group on sa, pass 3 on sb; pass 3 of g waits for
                    // pass 2 of g, pass 2 of g waits for pass 3 of g - ns (slot reuse)
                    auto run = [&] {
                        (void)hipEventRecord(eg0, 0);
                        (void)hipStreamWaitEvent(sa, eg0, 0);
                        (void)hipStreamWaitEvent(sb, eg0, 0);
                        for (uint32_t g = 0; g < groups; g++) {
                            d2* sl = sc + (g % ns) * slot;
                            if (g >= (uint32_t)ns) (void)hipStreamWaitEvent(sa, ev3[g - ns], 0);
                            hipLaunchKernelGGL(k_copy, dim3(tiles), dim3(512), 72 * 1024, sa, x, sl, Map{12, log_k, g, snt});
                            (void)hipEventRecord(ev2[g], sa);
                            (void)hipStreamWaitEvent(sb, ev2[g], 0);
                            hipLaunchKernelGGL(k_copy, dim3(tiles), dim3(512), 72 * 1024, sb, sl, y, Map{13, log_k, g, snt});
                            (void)hipEventRecord(ev3[g], sb);
                        }
                        (void)hipEventRecord(eg1, sb);
                        (void)hipStreamWaitEvent(0, eg1, 0);
                    };
                    ts[ns - 2] = groups <= 64 ? time(run) : -1.f;
                }
                printf("round %d   K=%d scratch %s: two streams, 2 slots %.3f ms, 3 slots %.3f ms\n", round,
                       1 << log_k, snt ? "nt" : "plain", ts[0], ts[1]);
                printf("round %d   K=%d scratch %s: pass-2 groups alone %.3f ms, pass-3 groups alone %.3f ms, "
                       "skewed pairs %.3f ms (halves interleaved: %.3f ms)\n",
                       round, 1 << log_k, snt ? "nt" : "plain", t2, t3, tk[0], tk[1]);
                printf("round %d grouped K=%d (%d MiB slot, %u launches, scratch %s): %.3f ms (%.0f GB/s of pass bytes)\n",
                       round, 1 << log_k, 4 << log_k, 2 * groups, snt ? "nt" : "plain", tg, bytes / tg / 1e6);
            }
        }
        fflush(stdout);
    }
    if (hipGetLastError() != hipSuccess) return 2;
    return 0;
}
