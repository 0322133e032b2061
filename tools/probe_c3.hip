// tools/probe_c3.hip -- standalone probe (not part of the product).
// The floor of the C3 share (fp32 4096-point transforms x 512, one transform
// per 256-thread workgroup, 16 values per thread, 2 workgroups per CU): copies
// with the single pass's exact shape, against the k_pass time (9 us).
//   c8   : 16 loads of 8 B per thread (element t + 256 k), then 16 stores
//   c16  : 8 loads of 16 B per thread (elements 2t, 2t+1 + 512 k), 8 stores
//   c8x  : c8 + the pass's two LDS exchanges (one component at a time, 7 barriers)
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_c3.hip -o tools/probe_c3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef float __attribute__((ext_vector_type(2))) f2;
typedef float __attribute__((ext_vector_type(4))) f4;

template <int NT>
__global__ __launch_bounds__(256, 2) void k_c8(const f2* __restrict__ in, f2* __restrict__ out) {
    extern __shared__ float lds[];
    const uint64_t base = (uint64_t)blockIdx.x * 4096;
    f2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = NT ? __builtin_nontemporal_load(in + base + threadIdx.x + 256 * k)
                                          : in[base + threadIdx.x + 256 * k];
    if (threadIdx.x == 4095) lds[0] = v[0].x;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        if (NT) __builtin_nontemporal_store(v[k], out + base + threadIdx.x + 256 * k);
        else out[base + threadIdx.x + 256 * k] = v[k];
    }
}

template <int NT>
__global__ __launch_bounds__(256, 2) void k_c16(const f4* __restrict__ in, f4* __restrict__ out) {
    extern __shared__ float lds[];
    const uint64_t base = (uint64_t)blockIdx.x * 2048;
    f4 v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) v[k] = NT ? __builtin_nontemporal_load(in + base + threadIdx.x + 256 * k)
                                         : in[base + threadIdx.x + 256 * k];
    if (threadIdx.x == 4095) lds[0] = v[0].x;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        if (NT) __builtin_nontemporal_store(v[k], out + base + threadIdx.x + 256 * k);
        else out[base + threadIdx.x + 256 * k] = v[k];
    }
}

// c8 plus two exchanges shaped like the pass's (write 16 scalars, barrier,
// read 16 scalars, per component; the first write of the tile unbarriered)
template <int NT>
__global__ __launch_bounds__(256, 2) void k_c8x(const f2* __restrict__ in, f2* __restrict__ out) {
    extern __shared__ float lds[];
    const uint64_t base = (uint64_t)blockIdx.x * 4096;
    f2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = NT ? __builtin_nontemporal_load(in + base + threadIdx.x + 256 * k)
                                          : in[base + threadIdx.x + 256 * k];
    const int t = threadIdx.x;
#pragma unroll
    for (int s = 0; s < 2; s++) {
#pragma unroll
        for (int comp = 0; comp < 2; comp++) {
            if (s > 0 || comp > 0) __syncthreads();
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int r = t * 16 + k;
                lds[r + (r >> 4)] = comp ? v[k].y : v[k].x;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int r = t + 256 * k;
                const float x = lds[r + (r >> 4)];
                if (comp) v[k].y = x; else v[k].x = x;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        if (NT) __builtin_nontemporal_store(v[k], out + base + threadIdx.x + 256 * k);
        else out[base + threadIdx.x + 256 * k] = v[k];
    }
}

int main() {
    const int batches[] = {512, 1024, 4096};
    const uint64_t nmax = 4096ull * 4096;
    f2 *x, *y;
    if (hipMalloc(&x, nmax * 8) || hipMalloc(&y, nmax * 8)) return 1;
    (void)hipMemset(x, 0, nmax * 8);
    (void)hipMemset(y, 0, nmax * 8);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto time = [&](auto launch) {
        for (int w = 0; w < 10; w++) launch();
        (void)hipEventRecord(e0);
        for (int it = 0; it < 100; it++) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        return ms * 1000 / 100;  // us
    };
    const int lds = 4352 * 4;
    for (int round = 0; round < 2; round++) {
        for (int b : batches) {
            const float a0 = time([&] { hipLaunchKernelGGL(k_c8<0>, dim3(b), dim3(256), lds, 0, x, y); });
            const float a1 = time([&] { hipLaunchKernelGGL(k_c8<1>, dim3(b), dim3(256), lds, 0, x, y); });
            const float b0 = time([&] { hipLaunchKernelGGL(k_c16<0>, dim3(b), dim3(256), lds, 0, (const f4*)x, (f4*)y); });
            const float b1 = time([&] { hipLaunchKernelGGL(k_c16<1>, dim3(b), dim3(256), lds, 0, (const f4*)x, (f4*)y); });
            const float c0 = time([&] { hipLaunchKernelGGL(k_c8x<0>, dim3(b), dim3(256), lds, 0, x, y); });
            const float c1 = time([&] { hipLaunchKernelGGL(k_c8x<1>, dim3(b), dim3(256), lds, 0, x, y); });
            const float d0 = time([&] { (void)hipMemcpyAsync(y, x, (size_t)b * 4096 * 8, hipMemcpyDeviceToDevice, 0); });
            printf("round %d batch %4d (us/launch): c8 %.2f / nt %.2f | c16 %.2f / nt %.2f | c8 + exchanges %.2f / nt %.2f | "
                   "hipMemcpy D2D %.2f\n", round, b, a0, a1, b0, b1, c0, c1, d0);
        }
        fflush(stdout);
    }
    return hipGetLastError() != hipSuccess ? 2 : 0;
}
