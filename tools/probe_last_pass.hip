// tools/probe_last_pass.hip -- standalone probe (not part of the product), round 6.
// The copy ceiling of the headline's dominant kernel at its own access map, on
// the same buffers and in the same process as the kernel:
//   k_pass<double,1024,8,2,1,0,16>  (fp64 2^28, the last of 512.512.1024)
//   k_pass<float,1024,16,2,1,0,32>  (fp32 2^28, the reference's own data_t)
// Both read the plan's padded workspace W (rows 2^18 + w_pad elements apart)
// and write the caller's output Y (rows 2^18 apart): C-element row segments
// (128 B at fp64 C = 8, 128 B at fp32 C = 16) on both sides.
// "copy(maps)" loads every value with the kernel's first-stage thread map and
// stores it with the kernel's last-stage map (Stage<...>::map, the same
// address formulas, non-temporal as the kernel; no twiddles, no DFT, no LDS
// exchange): the kernel's data movement alone.  Its LDS allocation is kept so
// that the same workgroups per CU are resident.  Variants: plain loads /
// stores, and a flat contiguous copy of the same bytes (the chip's copy rate).
// Twiddle tables are zero (timing does not depend on values).
//   hipcc -O3 -std=c++17 -w --offload-arch=gfx950 -ffp-contract=off \
//     -I cs87project-msolano2_amd/csrc tools/probe_last_pass.hip -o tools/probe_last_pass_bin
#include "pifft_kernels.h"

#include <stdio.h>
#include <stdlib.h>

using namespace pifft;

#define CHK(x)                                                                   \
    do {                                                                         \
        hipError_t e_ = (x);                                                     \
        if (e_ != hipSuccess) {                                                  \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                             \
        }                                                                        \
    } while (0)

// LD/ST: 1 non-temporal (the kernel's form), 0 plain
template <typename T, int R, int C, int VPT, int LD, int ST>
__global__ __launch_bounds__((PassCfg<R, C, VPT>::NT), (PassCfg<R, C, VPT>::waves_per_eu))
void k_copy_maps(PassArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    using Sh = PassShape<R, VPT>;
    using S0 = Stage<R, C, 2, 0, VPT>;
    using SL = Stage<R, C, 2, Sh::NSTG - 1, VPT>;
    using C2 = cx<T>;
    const int tid = (int)threadIdx.x;
    const uint64_t tile = tile_of_block(blockIdx.x, a.log_xg, gridDim.x);
    const uint64_t lb_mask = (1ull << a.log_lb) - 1;
    C2 v[Sh::Q];
    const C2* __restrict__ in = static_cast<const C2*>(a.in);
#pragma unroll
    for (int u = 0; u < S0::U; u++) {
        int c, b;
        S0::map(tid, u, c, b);
        const uint64_t line = tile * C + c, bt = line >> a.log_lb, j = line & lb_mask;
        const uint64_t rs = (1ull << a.log_lb) + a.in_pad;
        const C2* row = in + bt * a.in_bstride + j + (uint64_t)b * rs;
#pragma unroll
        for (int k = 0; k < S0::q; k++) v[u * S0::q + k] = ld_stream<LD != 0>(row + (uint64_t)(k * S0::NB) * rs);
    }
    if (tid == 100000) smem[0] = 1;  // never true: keeps the LDS allocation
    C2* __restrict__ out = static_cast<C2*>(a.out);
#pragma unroll
    for (int u = 0; u < SL::U; u++) {
        int c, b;
        SL::map(tid, u, c, b);
        const uint64_t line = tile * C + c, bt = line >> a.log_lb, j = line & lb_mask;
        const uint32_t lns = a.log_ns;
        const uint64_t pos = ((j >> lns) << (lns + Sh::LOGR)) + (j & ((1ull << lns) - 1)) + ((uint64_t)b << lns);
        C2* dst = out + bt * a.out_bstride + pos;
#pragma unroll
        for (int k = 0; k < SL::q; k++) st_stream<ST != 0>(dst + ((uint64_t)(k * SL::NB) << lns), v[u * SL::q + k]);
    }
}

// the same bytes, contiguous: each thread 16 B x V per 512-thread tile row
typedef double __attribute__((ext_vector_type(2))) d2v;
__global__ __launch_bounds__(512) void k_copy_flat(const d2v* __restrict__ x, d2v* __restrict__ y, uint64_t n16) {
    // 16-B units, grid-stride, non-temporal both sides
    for (uint64_t i = (uint64_t)blockIdx.x * 512 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 512)
        __builtin_nontemporal_store(__builtin_nontemporal_load(x + i), y + i);
}

static hipEvent_t e0, e1;

template <typename K>
static float time_launch(K launch, int reps) {
    for (int w = 0; w < 3; w++) launch();
    CHK(hipEventRecord(e0));
    for (int it = 0; it < reps; it++) launch();
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

template <typename T, int R, int C, int VPT>
static void probe(const char* name, uint32_t log_m, int rounds) {
    using C2 = cx<T>;
    const size_t esz = sizeof(C2);
    const uint64_t M = 1ull << log_m;
    const uint32_t log_lb = log_m - ilog2c(R);
    const uint64_t w_pad = (16384 + 256) / esz;  // the plan's padded workspace rows (pifft.hip)
    const uint64_t rows = M >> log_lb;
    const uint64_t w_elems = M + rows * w_pad;
    constexpr int LDSB = pass_lds_bytes<T, R, C, 2, VPT>();
    void *W, *Y, *twr, *tlo, *thi;
    CHK(hipMalloc(&W, w_elems * esz));
    CHK(hipMalloc(&Y, M * esz));
    CHK(hipMalloc(&twr, R * esz));
    CHK(hipMalloc(&tlo, (1u << 14) * esz));
    CHK(hipMalloc(&thi, (1u << 14) * esz));
    CHK(hipMemset(W, 0, w_elems * esz));
    CHK(hipMemset(twr, 0, R * esz));
    CHK(hipMemset(tlo, 0, (1u << 14) * esz));
    CHK(hipMemset(thi, 0, (1u << 14) * esz));
    PassArgs a{};
    a.in = W;
    a.out = Y;
    a.tw_r = twr;
    a.tw_lo = tlo;
    a.tw_hi = thi;
    a.in_bstride = w_elems;
    a.out_bstride = M;
    a.nlines = M >> ilog2c(R);
    a.log_lb = log_lb;
    a.log_ns = log_lb;  // the last pass: Ns = M / R
    a.tw_h = 14;
    a.tw_shift = 0;
    a.log_xg = 2;
    a.in_pad = (uint32_t)w_pad;
    const dim3 grid((unsigned)(a.nlines / C)), block(PassCfg<R, C, VPT>::NT);
    auto kp = k_pass<T, R, C, 2, 1, 0, VPT>;
    auto c11 = k_copy_maps<T, R, C, VPT, 1, 1>;
    auto c00 = k_copy_maps<T, R, C, VPT, 0, 0>;
    auto c10 = k_copy_maps<T, R, C, VPT, 1, 0>;
    auto c01 = k_copy_maps<T, R, C, VPT, 0, 1>;
    for (auto f : {(const void*)kp, (const void*)c11, (const void*)c00, (const void*)c10, (const void*)c01})
        CHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDSB));
    const double bytes = 2.0 * M * esz;
    const int reps = 20;
    printf("%s: M=2^%u, R=%d C=%d VPT=%d, %d threads, LDS %d B, grid %u, W rows %llu + %llu pad, %.3f GB/launch\n",
           name, log_m, R, C, VPT, PassCfg<R, C, VPT>::NT, LDSB, grid.x, (unsigned long long)(1ull << log_lb),
           (unsigned long long)w_pad, bytes / 1e9);
    for (int rd = 0; rd < rounds; rd++) {
        const float tk = time_launch([&] { hipLaunchKernelGGL(kp, grid, block, LDSB, 0, a); }, reps);
        const float t11 = time_launch([&] { hipLaunchKernelGGL(c11, grid, block, LDSB, 0, a); }, reps);
        const float t00 = time_launch([&] { hipLaunchKernelGGL(c00, grid, block, LDSB, 0, a); }, reps);
        const float t10 = time_launch([&] { hipLaunchKernelGGL(c10, grid, block, LDSB, 0, a); }, reps);
        const float t01 = time_launch([&] { hipLaunchKernelGGL(c01, grid, block, LDSB, 0, a); }, reps);
        const uint64_t n16 = M * esz / 16;
        const float tf = time_launch(
            [&] { hipLaunchKernelGGL(k_copy_flat, dim3(8192), dim3(512), 0, 0, (const d2v*)W, (d2v*)Y, n16); },
            reps);
        auto tb = [&](float ms) { return bytes / (ms * 1e-3) / 1e12; };
        printf("  round %d: kernel %.4f ms (%.3f TB/s, frac %.4f) | copy(maps) nt/nt %.4f ms (%.3f TB/s) -> kernel/copy "
               "%.3f | plain/plain %.4f (%.3f) | nt-load/plain-store %.4f (%.3f) | plain-load/nt-store %.4f (%.3f) | "
               "flat copy %.4f (%.3f)\n",
               rd, tk, tb(tk), tb(tk) / 8.0, t11, tb(t11), tk / t11, t00, tb(t00), t10, tb(t10), t01, tb(t01), tf,
               tb(tf));
        fflush(stdout);
    }
    CHK(hipGetLastError());
    CHK(hipFree(W));
    CHK(hipFree(Y));
    CHK(hipFree(twr));
    CHK(hipFree(tlo));
    CHK(hipFree(thi));
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    probe<double, 1024, 8, 16>("fp64 C4 last pass k_pass<double,1024,8,2,1,0,16>", 28, rounds);
    probe<float, 1024, 16, 32>("fp32 C4 last pass k_pass<float,1024,16,2,1,0,32>", 28, rounds);
    return 0;
}
