// tools/probe_mall.hip -- standalone probe (not part of the product).
// Question: can the 256 MiB Infinity Cache (MALL) hold the intermediate of a
// two-launch sub-pass pair, so that a 2^28 fp64 transform moves 4S of HBM
// traffic (two logical passes) instead of 6S (three passes)?
//
// Emulates it with copies of S = 4 GiB:
//   full       A -> B                      (1 pass, reference)
//   two        A -> T -> B                 (2 passes through HBM)
//   chunked K  for each K-byte chunk c: A[c] -> S, S -> B[c]   (S reused)
// If the MALL absorbs S, "chunked" costs about one pass, else two.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_mall.hip -o tools/probe_mall
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef float __attribute__((ext_vector_type(4))) f4;

template <bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_k(const f4* __restrict__ in, f4* __restrict__ out, uint64_t n) {
    constexpr int U = 4;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; base < n; base += stride * U) {
        f4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = base + u * stride;
            if (i < n) v[u] = NTL ? __builtin_nontemporal_load(in + i) : in[i];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t i = base + u * stride;
            if (i < n) {
                if (NTS) __builtin_nontemporal_store(v[u], out + i);
                else out[i] = v[u];
            }
        }
    }
}

typedef void (*copy_fn)(const f4*, f4*, uint64_t);

static void launch(int ntl, int nts, const f4* in, f4* out, uint64_t n, hipStream_t s) {
    const uint64_t want = (n + 256 * 4 - 1) / (256 * 4);
    const unsigned grid = (unsigned)(want < 65536 ? want : 65536);
    if (ntl && nts) hipLaunchKernelGGL((copy_k<true, true>), dim3(grid), dim3(256), 0, s, in, out, n);
    else if (ntl) hipLaunchKernelGGL((copy_k<true, false>), dim3(grid), dim3(256), 0, s, in, out, n);
    else if (nts) hipLaunchKernelGGL((copy_k<false, true>), dim3(grid), dim3(256), 0, s, in, out, n);
    else hipLaunchKernelGGL((copy_k<false, false>), dim3(grid), dim3(256), 0, s, in, out, n);
}

int main() {
    const uint64_t S = 1ull << 32;  // bytes
    const uint64_t n = S / 16;
    f4 *A, *B, *T, *Sc;
    if (hipMalloc(&A, S) || hipMalloc(&B, S) || hipMalloc(&T, S) || hipMalloc(&Sc, 512ull << 20)) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(A, 0, S);
    hipMemset(B, 0, S);
    hipMemset(T, 0, S);
    hipMemset(Sc, 0, 512ull << 20);
    hipStream_t s0, s1;
    hipStreamCreate(&s0);
    hipStreamCreate(&s1);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int reps = 3;
    auto timeit = [&](auto&& body) {
        body();
        hipDeviceSynchronize();
        hipEventRecord(e0, s0);
        for (int r = 0; r < reps; r++) body();
        hipEventRecord(e1, s0);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        return ms / reps;
    };
    printf("case\tchunk_MiB\tnt_hbm\tms\tGBps_1pass_equiv\n");
    for (int nt = 0; nt < 2; nt++) {
        float ms = timeit([&] { launch(nt, nt, A, B, n, s0); });
        printf("full\t-\t%d\t%.3f\t%.0f\n", nt, ms, 2.0 * S / ms / 1e6);
        ms = timeit([&] { launch(nt, nt, A, T, n, s0); launch(nt, nt, T, B, n, s0); });
        printf("two\t-\t%d\t%.3f\t%.0f\n", nt, ms, 2.0 * S / ms / 1e6);
        for (uint64_t K = 8ull << 20; K <= (256ull << 20); K *= 2) {
            const uint64_t kn = K / 16, nch = S / K;
            ms = timeit([&] {
                for (uint64_t c = 0; c < nch; c++) {
                    launch(nt, 0, A + c * kn, Sc, kn, s0);
                    launch(0, nt, Sc, B + c * kn, kn, s0);
                }
            });
            printf("chunked\t%llu\t%d\t%.3f\t%.0f\n", (unsigned long long)(K >> 20), nt, ms, 2.0 * S / ms / 1e6);
        }
        // double-buffered scratch on two streams: chunk c+1's first copy
        // overlaps chunk c's second copy
        for (uint64_t K = 16ull << 20; K <= (128ull << 20); K *= 2) {
            const uint64_t kn = K / 16, nch = S / K;
            hipEvent_t evA[2], evB[2];
            for (int b = 0; b < 2; b++) {
                hipEventCreateWithFlags(&evA[b], hipEventDisableTiming);
                hipEventCreateWithFlags(&evB[b], hipEventDisableTiming);
            }
            ms = timeit([&] {
                for (uint64_t c = 0; c < nch; c++) {
                    const int b = (int)(c & 1);
                    f4* sc = Sc + b * kn;
                    if (c >= 2) hipStreamWaitEvent(s0, evB[b], 0);  // chunk c-2 done reading sc
                    launch(nt, 0, A + c * kn, sc, kn, s0);
                    hipEventRecord(evA[b], s0);
                    hipStreamWaitEvent(s1, evA[b], 0);
                    launch(0, nt, sc, B + c * kn, kn, s1);
                    hipEventRecord(evB[b], s1);
                }
                hipEventRecord(evB[0], s1);
                hipStreamWaitEvent(s0, evB[0], 0);
            });
            printf("chunked2s\t%llu\t%d\t%.3f\t%.0f\n", (unsigned long long)(K >> 20), nt, ms, 2.0 * S / ms / 1e6);
        }
    }
    // per-phase timing: A = HBM -> scratch, B = scratch -> HBM, for scratch
    // policies: sc = 0 default, 1 nt on the scratch side too
    for (int scnt = 0; scnt < 2; scnt++)
        for (uint64_t K = 32ull << 20; K <= (256ull << 20); K *= 2) {
            const uint64_t kn = K / 16, nch = S / K;
            hipEvent_t ev[3];
            for (int i = 0; i < 3; i++) (void)hipEventCreate(&ev[i]);
            double ta = 0, tb = 0;
            for (int rep = 0; rep < 2; rep++)
                for (uint64_t c = 0; c < nch; c++) {
                    (void)hipEventRecord(ev[0], s0);
                    launch(1, scnt, A + c * kn, Sc, kn, s0);
                    (void)hipEventRecord(ev[1], s0);
                    launch(scnt, 1, Sc, B + c * kn, kn, s0);
                    (void)hipEventRecord(ev[2], s0);
                    (void)hipEventSynchronize(ev[2]);
                    float m1, m2;
                    (void)hipEventElapsedTime(&m1, ev[0], ev[1]);
                    (void)hipEventElapsedTime(&m2, ev[1], ev[2]);
                    if (rep) { ta += m1; tb += m2; }
                }
            printf("phase\tscratch_nt=%d\tchunk=%lluMiB\tA %.1f us (%.0f GB/s)\tB %.1f us (%.0f GB/s)\n", scnt,
                   (unsigned long long)(K >> 20), 1e3 * ta / nch, 2.0 * K / (ta / nch) / 1e6, 1e3 * tb / nch,
                   2.0 * K / (tb / nch) / 1e6);
        }
    // HBM-only references for the same chunk sizes: read-only-ish copy HBM->HBM
    for (uint64_t K = 32ull << 20; K <= (256ull << 20); K *= 2) {
        const uint64_t kn = K / 16, nch = S / K;
        float ms = timeit([&] {
            for (uint64_t c = 0; c < nch; c++) launch(1, 1, A + c * kn, B + c * kn, kn, s0);
        });
        printf("hbmchunks\t%llu\t%.3f ms\t%.0f GB/s\n", (unsigned long long)(K >> 20), ms, 2.0 * S / ms / 1e6);
    }
    return 0;
}
