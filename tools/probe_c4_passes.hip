// tools/probe_c4_passes.hip -- standalone probe (not part of the product), round 6.
// Every pass of the headline plan (fp64 2^28: 512.512.1024 at C = 16/16/8)
// and of its fp32 twin (C = 32/32/16, 32 values per thread), each against a
// copy with exactly that pass's load and store maps, on the plan's own
// buffers in one process: the input X, the output Y and the padded workspace
// W (rows 2^18 + w_pad apart), chained as the plan runs them
//   pass 1 (MODE 1): X -> Y   strided read (C-element row segments), contiguous lines out
//   pass 2 (MODE 2): Y -> W   strided both sides, W's padded rows
//   pass 3 (MODE 2): W -> Y   strided both sides (the dominant kernel)
// "copy" = k_copy_pass: every value loaded with the kernel's first-stage
// thread map and stored with its last-stage map (Stage<...>::map, the same
// address formulas and non-temporal forms; no twiddles, no DFT, no LDS
// exchange), the kernel's LDS allocation kept so the same workgroups per CU
// are resident.  Twiddle tables are zero (timing does not depend on values).
//   hipcc -O3 -std=c++17 -w --offload-arch=gfx950 -ffp-contract=off \
//     -I cs87project-msolano2_amd/csrc tools/probe_c4_passes.hip -o tools/probe_c4_passes_bin
#include "pifft_kernels.h"

#include <stdio.h>
#include <stdlib.h>

using namespace pifft;

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

template <typename T, int R, int C, int MODE, int VPT>
__global__ __launch_bounds__((PassCfg<R, C, VPT>::NT), (PassCfg<R, C, VPT>::waves_per_eu))
void k_copy_pass(PassArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    using Sh = PassShape<R, VPT>;
    using S0 = Stage<R, C, MODE, 0, VPT>;
    using SL = Stage<R, C, MODE, Sh::NSTG - 1, VPT>;
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
        for (int k = 0; k < S0::q; k++) v[u * S0::q + k] = ld_stream<true>(row + (uint64_t)(k * S0::NB) * rs);
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
        const uint64_t pad = (j >> a.out_pad_log) * a.out_pad;
        C2* dst = out + bt * a.out_bstride + pos + pad;
#pragma unroll
        for (int k = 0; k < SL::q; k++) st_stream<true>(dst + ((uint64_t)(k * SL::NB) << lns), v[u * SL::q + k]);
    }
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

struct Launch {
    const void* fn;
    dim3 grid, block;
    int lds;
    PassArgs a;
    void go() const {
        PassArgs x = a;
        void* args[] = {&x};
        (void)hipLaunchKernel(fn, grid, block, args, (size_t)lds, 0);
    }
};

template <typename T, int R, int C, int MODE, int VPT>
static void make(Launch& k, Launch& c, const PassArgs& a) {
    constexpr int LDSB = pass_lds_bytes<T, R, C, MODE, VPT>();
    k.fn = (const void*)&k_pass<T, R, C, MODE, 1, 0, VPT>;
    c.fn = (const void*)&k_copy_pass<T, R, C, MODE, VPT>;
    for (const void* f : {k.fn, c.fn}) CHK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDSB));
    k.grid = c.grid = dim3((unsigned)(a.nlines / C));
    k.block = c.block = dim3(PassCfg<R, C, VPT>::NT);
    k.lds = c.lds = LDSB;
    k.a = c.a = a;
}

// the three passes R1.R2.R3 = 512.512.1024 of an M = 2^28 transform
template <typename T, int C1, int C2_, int C3, int VPT>
static void probe(const char* name, int rounds) {
    using CT = cx<T>;
    const size_t esz = sizeof(CT);
    const uint32_t log_m = 28;
    const uint64_t M = 1ull << log_m;
    const uint64_t w_pad = (16384 + 256) / esz;      // pifft.hip: PIFFT_W_PAD default
    const uint64_t w_rows = M >> (log_m - 10);       // the reading pass (R = 1024): 2^10 rows
    const uint64_t w_tr = M + w_rows * w_pad;
    void *X, *Y, *W, *tw;
    CHK(hipMalloc(&X, M * esz));
    CHK(hipMalloc(&Y, M * esz));
    CHK(hipMalloc(&W, w_tr * esz));
    CHK(hipMalloc(&tw, (1u << 16) * esz));
    CHK(hipMemset(X, 0, M * esz));
    CHK(hipMemset(tw, 0, (1u << 16) * esz));
    const char* twb = (const char*)tw;
    PassArgs base{};
    base.tw_r = twb;
    base.tw_lo = twb + (1u << 14) * esz;
    base.tw_hi = twb + (2u << 14) * esz;
    base.tw_h = 14;
    base.log_xg = 2;
    PassArgs p1 = base, p2 = base, p3 = base;
    // pass 1: R = 512, first pass, X -> Y
    p1.in = X; p1.out = Y; p1.in_bstride = M; p1.out_bstride = M; p1.nlines = M >> 9;
    p1.log_lb = log_m - 9; p1.log_ns = 0; p1.tw_shift = log_m - 9;
    // pass 2: R = 512, Ns = 512, Y -> W (padded rows: + (j >> 9) w_pad)
    p2.in = Y; p2.out = W; p2.in_bstride = M; p2.out_bstride = w_tr; p2.nlines = M >> 9;
    p2.log_lb = log_m - 9; p2.log_ns = 9; p2.tw_shift = log_m - 18;
    p2.out_pad = (uint32_t)w_pad; p2.out_pad_log = (log_m - 10) - 9;
    // pass 3: R = 1024, Ns = 2^18, W -> Y
    p3.in = W; p3.out = Y; p3.in_bstride = w_tr; p3.out_bstride = M; p3.nlines = M >> 10;
    p3.log_lb = log_m - 10; p3.log_ns = log_m - 10; p3.tw_shift = 0; p3.in_pad = (uint32_t)w_pad;
    Launch k[3], c[3];
    make<T, 512, C1, 1, VPT>(k[0], c[0], p1);
    make<T, 512, C2_, 2, VPT>(k[1], c[1], p2);
    make<T, 1024, C3, 2, VPT>(k[2], c[2], p3);
    const double bytes = 2.0 * M * esz;
    const int reps = 20;
    printf("%s: 2^28 x %zu B, passes 512 (C=%d, MODE 1) . 512 (C=%d, MODE 2) . 1024 (C=%d, MODE 2), VPT %d, "
           "W pad %llu per 2^18-element row, %.3f GB per pass\n",
           name, esz, C1, C2_, C3, VPT, (unsigned long long)w_pad, bytes / 1e9);
    for (int rd = 0; rd < rounds; rd++) {
        float tk[3], tc[3];
        for (int i = 0; i < 3; i++) {
            tk[i] = time_launch([&] { k[i].go(); }, reps);
            tc[i] = time_launch([&] { c[i].go(); }, reps);
        }
        const float step_k = time_launch([&] { for (auto& l : k) l.go(); }, reps);
        const float step_c = time_launch([&] { for (auto& l : c) l.go(); }, reps);
        auto tb = [&](float ms) { return bytes / (ms * 1e-3) / 1e12; };
        printf("  round %d:", rd);
        for (int i = 0; i < 3; i++)
            printf(" | pass %d kernel %.4f ms (%.2f TB/s) copy %.4f (%.2f) k/c %.3f", i + 1, tk[i], tb(tk[i]), tc[i],
                   tb(tc[i]), tk[i] / tc[i]);
        printf(" | step: kernels %.4f ms, copies %.4f ms, k/c %.3f\n", step_k, step_c, step_k / step_c);
        fflush(stdout);
    }
    CHK(hipGetLastError());
    CHK(hipFree(X));
    CHK(hipFree(Y));
    CHK(hipFree(W));
    CHK(hipFree(tw));
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 3;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    probe<double, 16, 16, 8, 16>("fp64 C4", rounds);
    probe<float, 32, 32, 16, 32>("fp32 C4", rounds);
    return 0;
}
