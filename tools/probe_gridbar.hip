// tools/probe_gridbar.hip -- bounded experiment for config 2's one-GPU slice
// (round-3 verdict, "Next" item 5: cut a launch): what does a launch boundary
// between the slice's two passes cost, against a grid-wide barrier inside one
// launch?
//
// The slice's shape: 64 workgroups x 256 threads, each pass moving 2 MiB in
// and 2 MiB out (8 16-B values per thread), pass 2 reading what OTHER
// workgroups wrote in pass 1 (a transpose-like hand-off: workgroup w reads
// the 1/64 of every workgroup's output, as a Stockham pass does).
//   two:  pass 1 and pass 2 as two launches back to back (today's plan);
//   bar:  one launch, pass 1, a grid barrier (every wave's s_waitcnt, a
//         workgroup barrier, lane 0's agent-scope release and counter add, a
//         bounded poll, agent-scope acquire), pass 2;
//   one:  pass 1 alone (one launch's floor).
// Loops of L launches back to back between two marker events; the counter
// is monotonic (launch i waits for 64 (i + 1) arrivals), every poll is
// bounded (2^20 polls, then it gives up and flags *err), so the grid always
// drains.  All 64 workgroups are co-resident (256 CUs).
//
// build: hipcc -O3 --offload-arch=gfx950 tools/probe_gridbar.hip -o tools/probe_gridbar_bin
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x)                                                                        \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

constexpr int NWG = 64, NT = 256, V = 8;
constexpr size_t ELEMS = (size_t)NWG * NT * V;  // 131072 values = 2 MiB at 16 B

typedef double d2 __attribute__((ext_vector_type(2)));

// pass 1: workgroup w reads its own contiguous 32 KiB, writes it contiguous
__device__ __forceinline__ void pass1(const d2* __restrict__ a, d2* __restrict__ b) {
    const size_t base = (size_t)blockIdx.x * NT * V;
    d2 v[V];
#pragma unroll
    for (int k = 0; k < V; k++) v[k] = a[base + (size_t)k * NT + threadIdx.x];
#pragma unroll
    for (int k = 0; k < V; k++) b[base + (size_t)k * NT + threadIdx.x] = v[k] * 1.0000001;
}

// pass 2: workgroup w reads 1/64 of every workgroup's pass-1 output
// (64-value runs: 1 KiB contiguous), writes contiguous
__device__ __forceinline__ void pass2(const d2* __restrict__ b, d2* __restrict__ c) {
    const int w = blockIdx.x;
    d2 v[V];
#pragma unroll
    for (int k = 0; k < V; k++) {
        const int j = k * NT + threadIdx.x;     // 0 .. 2047 of this workgroup's inputs
        const int src = j >> 5, off = j & 31;   // 32 values from each of the 64 workgroups
        v[k] = b[(size_t)src * NT * V + (size_t)w * 32 + off];
    }
#pragma unroll
    for (int k = 0; k < V; k++) c[(size_t)w * NT * V + (size_t)k * NT + threadIdx.x] = v[k] + 1.0;
}

__device__ __forceinline__ void grid_barrier(unsigned* ctr, unsigned want, unsigned* err) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1 << 20)) {
                __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __builtin_amdgcn_s_waitcnt(0);
    }
    __syncthreads();
}

__global__ __launch_bounds__(NT) void k_p1(const d2* a, d2* b) { pass1(a, b); }
__global__ __launch_bounds__(NT) void k_p2(const d2* b, d2* c) { pass2(b, c); }
__global__ __launch_bounds__(NT) void k_bar(const d2* a, d2* b, d2* c, unsigned* ctr, unsigned want, unsigned* err) {
    pass1(a, b);
    grid_barrier(ctr, want, err);
    pass2(b, c);
}

int main(int argc, char** argv) {
    const int L = argc > 1 ? atoi(argv[1]) : 2000;
    d2 *a, *b, *c;
    unsigned *ctr, *err;
    CHK(hipMalloc(&a, ELEMS * 16));
    CHK(hipMalloc(&b, ELEMS * 16));
    CHK(hipMalloc(&c, ELEMS * 16));
    CHK(hipMalloc(&ctr, 4));
    CHK(hipMalloc(&err, 4));
    CHK(hipMemset(a, 0, ELEMS * 16));
    CHK(hipMemset(ctr, 0, 4));
    CHK(hipMemset(err, 0, 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    unsigned launches = 0;
    auto run = [&](int mode, int n) {
        for (int i = 0; i < n; i++) {
            if (mode == 0) {
                k_p1<<<NWG, NT>>>(a, b);
                k_p2<<<NWG, NT>>>(b, c);
            } else if (mode == 1) {
                launches++;
                k_bar<<<NWG, NT>>>(a, b, c, ctr, launches * NWG, err);
            } else {
                k_p1<<<NWG, NT>>>(a, b);
            }
        }
    };
    const char* names[] = {"two launches (pass 1, pass 2)", "one launch + grid barrier", "pass 1 alone"};
    for (int rep = 0; rep < 3; rep++)
        for (int mode = 0; mode < 3; mode++) {
            run(mode, 50);
            CHK(hipEventRecord(e0, 0));
            run(mode, L);
            CHK(hipEventRecord(e1, 0));
            CHK(hipEventSynchronize(e1));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            printf("rep %d  %-32s %8.3f us per step\n", rep, names[mode], ms * 1e3 / L);
        }
    CHK(hipDeviceSynchronize());
    unsigned h_err = 0, h_ctr = 0;
    CHK(hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(&h_ctr, ctr, 4, hipMemcpyDeviceToHost));
    printf("barrier arrivals %u (expected %u), poll give-ups %u\n", h_ctr, launches * NWG, h_err);
    return h_err != 0 || h_ctr != launches * NWG;
}
