// tools/probe_coop.hip -- bounded experiment for a TWO-pass fp64 2^28 plan
// (round-3 verdict, "Next" item 4): the data movement of one 2^14-point
// column pass done by a group of workgroups that cooperate through an
// XCD-local L2 scratch, without the FFT arithmetic.
//
// The 2^28 transform as 2^14 x 2^14: every pass of a two-pass plan needs all
// 2^14 points of a column, 256 KiB at fp64 -- more than one workgroup holds.
// A group of G = 16 workgroups on one XCD (blocks b, b + 8, ... share an XCD's
// L2) takes 8 adjacent columns (128-B row segments, 2 MiB):
//   step 1: workgroup w loads rows n1 + 128 n2 (n1 in [8w, 8w+8), n2 < 128)
//           -- the inputs of its 8 x 8 128-point sub-FFTs -- and writes them to
//           the group's scratch S[n2][n1][c] (1-KiB runs);
//   barrier: MODE 3 (the valid form, MI355X_MICROARCH.md "Valid forms"):
//           every wave's s_waitcnt, a workgroup barrier, lane 0's agent-scope
//           release (buffer_wbl2) and relaxed counter add; the consumer's one
//           relaxed poll, agent-scope acquire (buffer_inv sc1), s_waitcnt and
//           barrier before its plain loads.  MODE 0 drops both fences -- racy,
//           NOT a valid hand-off, only the optimistic lower bound of the
//           design's time (same-XCD L2-resident scratch, free hand-off);
//   step 2: workgroup w reads S[k2][*][*] for k2 in [8w, 8w+8) (the inputs of
//           its second-stage sub-FFTs) and writes the column's outputs
//           out[(c0 + c) 2^14 + k2 + 128 k1] (128-B runs).
// Compared in the same process with
//   mode 1 (self): the same two steps, each workgroup reading back only its
//           own scratch rows (no cross-workgroup hand-off, no barrier);
//   mode 2 (copy): step 1's loads stored straight to the same positions of
//           out (128-B segments both sides: the current last pass's pattern);
// and the three-pass plan's measured passes (1.38 / 1.41 / 1.66 ms).
// If one cooperative column pass cannot move its 8.6 GB well under ~2 ms, two
// of them plus the arithmetic cannot beat the three-pass 4.44 ms.
//
// Persistent grid: 512 workgroups (2 per CU, all co-resident), groups of 16
// per XCD, 2048 column blocks; every workgroup reaches every barrier of its
// group (the loop bounds are uniform), and every spin is bounded (2^20 polls,
// then it gives up and flags counters[GROUPS * 32]), so the grid always drains.
//
// build: hipcc -O3 --offload-arch=gfx950 tools/probe_coop.hip -o /tmp/probe_coop
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#define CHK(x)                                                                        \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int LOGW = 14;               // 2^14 x 2^14 points
constexpr uint64_t W = 1ull << LOGW;
constexpr int G = 16;                   // workgroups per group
constexpr int NT = 512;                 // threads per workgroup
constexpr int VPT = 16;                 // values per thread (8192 per workgroup)
constexpr int NWG = 512;                // persistent grid: 2 per CU
constexpr int GROUPS = NWG / G;         // 32 groups, 4 per XCD
constexpr int NCB = (int)(W / 8);       // 2048 column blocks of 8 columns
constexpr int SCR = 8 * (int)W;         // scratch values per group (2 MiB)

struct c64 {
    double re, im;
};

__device__ __forceinline__ c64 ldnt(const c64* p) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2*>(p));
    return c64{v.x, v.y};
}
__device__ __forceinline__ void stnt(c64* p, c64 v) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2 r;
    r.x = v.re;
    r.y = v.im;
    __builtin_nontemporal_store(r, reinterpret_cast<d2*>(p));
}

// lane 0 of the workgroup: arrive on *ctr and wait for `want` arrivals (bounded)
template <bool FENCES>
__device__ __forceinline__ void group_barrier(unsigned* ctr, unsigned want, unsigned* err) {
    __builtin_amdgcn_s_waitcnt(0);  // this wave's stores have left it
    __syncthreads();
    if (threadIdx.x == 0) {
        if (FENCES) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1 << 20)) {
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        if (FENCES) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __builtin_amdgcn_s_waitcnt(0);
    }
    __syncthreads();
}

// Addresses: a per-thread 32-bit byte offset from a base that is uniform per
// value index k (row strides of 256 KiB x 1024 do not fit an immediate), so
// the 16 loads in flight cost one VGPR of address each.
template <typename P>
__device__ __forceinline__ P* at(P* base, uint64_t uniform_elems, uint32_t off_bytes) {
    using B = typename std::conditional<std::is_const<P>::value, const char, char>::type;
    return reinterpret_cast<P*>(reinterpret_cast<B*>(base + uniform_elems) + off_bytes);
}

template <int MODE>
__global__ __launch_bounds__(NT, 4) void k_coop(  // 4 waves per SIMD: 2 workgroups per CU
    const c64* __restrict__ x, c64* __restrict__ out, c64* scratch, unsigned* counters) {
    const int b = blockIdx.x, t = threadIdx.x;
    const int xcd = b & 7, slot = b >> 3;               // 64 workgroups per XCD
    const int grp = xcd * (64 / G) + slot / G, w = slot % G;
    c64* S = scratch + (size_t)grp * SCR;
    unsigned* ctr = counters + grp * 32;                // one 128-B line per counter
    // value k of thread t: e = t + 512 k; step 1 / scratch stores: c = t & 7,
    // n1o = (t >> 3) & 7, n2 = (t >> 6) + 8 k; step 2: k2o = t & 7,
    // c = (t >> 3) & 7, n1 = (t >> 6) + 8 k
    const uint32_t c_a = t & 7, n1o = (t >> 3) & 7, q = t >> 6;
    const uint32_t off_x = (uint32_t)(((8 * w + n1o + 128 * q) * W + c_a) * sizeof(c64));  // + row 1024 k, + c0
    const uint32_t off_s = (uint32_t)(((q * 128 + 8 * w + n1o) * 8 + c_a) * sizeof(c64));  // + 8 k rows of 128 x 8
    const uint32_t k2o = t & 7, c_b = (t >> 3) & 7;
    const uint32_t off_r = (uint32_t)((((8 * w + k2o) * 128 + q) * 8 + c_b) * sizeof(c64));  // + n1 8 k
    const uint32_t off_o = (uint32_t)((c_b * W + 8 * w + k2o + 128 * q) * sizeof(c64));      // + 1024 k, + c0 W
    c64 v[VPT];
    int iter = 0;
    for (int cb = grp; cb < NCB; cb += GROUPS, iter++) {
        const uint64_t c0 = (uint64_t)cb * 8;
        // ---- step 1: rows 8w + n1o + 128 n2, 8 columns (lanes across c) ----
#pragma unroll
        for (int k = 0; k < VPT; k++) v[k] = ldnt(at(x, (uint64_t)k * 1024 * W + c0, off_x));
        if constexpr (MODE == 2) {
            // plain strided copy: the same positions of out
#pragma unroll
            for (int k = 0; k < VPT; k++) stnt(at(out, (uint64_t)k * 1024 * W + c0, off_x), v[k]);
            continue;
        }
        // scratch S[n2][n1][c] (1-KiB runs per n2)
#pragma unroll
        for (int k = 0; k < VPT; k++) *at(S, (uint64_t)k * 8 * 128 * 8, off_s) = v[k];
        if constexpr (MODE == 0 || MODE == 3) {
            group_barrier<MODE == 3>(ctr, (unsigned)(G * (iter + 1)), counters + GROUPS * 32);
        } else {
            __syncthreads();
        }
        // ---- step 2: k2 in [8w, 8w+8) (MODE 1: the rows this workgroup wrote) ----
#pragma unroll
        for (int k = 0; k < VPT; k++) {
            if constexpr (MODE == 0 || MODE == 3) {
                v[k] = *at(S, (uint64_t)k * 8 * 8, off_r);
            } else {
                // own rows (n2 = n1 index here): the transpose of what this workgroup holds
                v[k] = *at(S, (uint64_t)k * 8 * 128 * 8, off_s);
            }
        }
#pragma unroll
        for (int k = 0; k < VPT; k++) stnt(at(out, c0 * W + (uint64_t)k * 1024, off_o), v[k]);
        if constexpr (MODE == 0 || MODE == 3) {
            // the next iteration's step 1 overwrites S: every group member must
            // have read it (second counter, no payload behind it: no fences)
            group_barrier<false>(ctr + 16, (unsigned)(G * (iter + 1)), counters + GROUPS * 32);
        } else {
            __syncthreads();
        }
    }
}

__global__ void k_fill(c64* x, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        x[i] = c64{(double)(i & 1023), (double)(i >> 10)};
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    const uint64_t n = W * W;
    c64 *x, *y, *s;
    unsigned* ctr;
    CHK(hipMalloc(&x, n * sizeof(c64)));
    CHK(hipMalloc(&y, n * sizeof(c64)));
    CHK(hipMalloc(&s, (size_t)GROUPS * SCR * sizeof(c64)));
    CHK(hipMalloc(&ctr, (GROUPS * 32 + 32) * sizeof(unsigned)));
    CHK(hipMemset(ctr, 0, (GROUPS * 32 + 32) * sizeof(unsigned)));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, x, n);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const char* names[4] = {"coop, no fences (racy lower bound)", "self (L2 scratch, no hand-off)",
                            "copy (128-B segments both sides)", "coop, agent release/acquire (valid)"};
    for (int round = 0; round < 2; round++) {
        for (int mode = 0; mode < 4; mode++) {
            float best = 1e30f, sum = 0.0f;
            for (int r = 0; r < reps; r++) {
                CHK(hipMemset(ctr, 0, GROUPS * 32 * sizeof(unsigned)));
                CHK(hipEventRecord(e0, 0));
                if (mode == 0) hipLaunchKernelGGL(k_coop<0>, dim3(NWG), dim3(NT), 0, 0, x, y, s, ctr);
                if (mode == 1) hipLaunchKernelGGL(k_coop<1>, dim3(NWG), dim3(NT), 0, 0, x, y, s, ctr);
                if (mode == 2) hipLaunchKernelGGL(k_coop<2>, dim3(NWG), dim3(NT), 0, 0, x, y, s, ctr);
                if (mode == 3) hipLaunchKernelGGL(k_coop<3>, dim3(NWG), dim3(NT), 0, 0, x, y, s, ctr);
                CHK(hipGetLastError());
                CHK(hipEventRecord(e1, 0));
                CHK(hipEventSynchronize(e1));
                float ms;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
                sum += ms;
            }
            // check the coop / self permutation on a few elements
            const double gb = 2.0 * n * sizeof(c64) / 1e9;
            printf("round %d  %-44s best %.3f ms  mean %.3f ms  %.2f TB/s (best)\n", round, names[mode], best,
                   sum / reps, gb / best);  // GB per ms = TB/s
            fflush(stdout);
        }
    }
    // correctness of the valid coop permutation: out[(c0+c) W + k2 + 128 n1] = x[(n1 + 128 k2) W + c0 + c]
    CHK(hipMemset(y, 0, n * sizeof(c64)));
    CHK(hipMemset(ctr, 0, GROUPS * 32 * sizeof(unsigned)));
    hipLaunchKernelGGL(k_coop<3>, dim3(NWG), dim3(NT), 0, 0, x, y, s, ctr);
    CHK(hipDeviceSynchronize());
    unsigned err = 0;
    CHK(hipMemcpy(&err, ctr + GROUPS * 32, sizeof err, hipMemcpyDeviceToHost));
    printf("spin limit reached: %s\n", err ? "YES (a group was not co-resident)" : "never");
    int bad = 0;
    for (int probe = 0; probe < 64; probe++) {
        const uint64_t col = (probe * 2654435761u) % W, n1 = (probe * 40503u) % 128, k2 = (probe * 977u) % 128;
        c64 got, want;
        CHK(hipMemcpy(&got, y + col * W + k2 + 128 * n1, sizeof got, hipMemcpyDeviceToHost));
        const uint64_t src = (n1 + 128 * k2) * W + col;
        want = c64{(double)(src & 1023), (double)(src >> 10)};
        bad += got.re != want.re || got.im != want.im;
    }
    printf("coop permutation check: %s (%d of 64 wrong)\n", bad ? "FAIL" : "ok", bad);
    return bad || err ? 1 : 0;
}
