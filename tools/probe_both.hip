// tools/probe_both.hip -- standalone probe (not part of the product).
// Pass 2 and pass 3 of the 2^28 fp64 plan are the same kernel (R = 512,
// C = 16, strided on both sides) but pass 3 runs ~12 % slower; they differ in
// the write side's row stride (16 KiB vs 8 MiB).  A tile copy with the exact
// Stockham index maps of both passes (and with the write map swapped) shows
// whether the write stride alone sets the difference.
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_both.hip -o tools/probe_both
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double __attribute__((ext_vector_type(2))) d2;

// line j < M/R, element r < R: in[j + r M/R]; out[(j/Ns) Ns R + j%Ns + r Ns]
__global__ __launch_bounds__(512) void pass_copy(const d2* __restrict__ in, d2* __restrict__ out, int log_lb,
                                                 int log_ns_w, int C) {
    const int R = 512, NT = 512;
    const uint64_t tile = blockIdx.x;
    d2 v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + k * NT;
        const int c = g % C, r = g / C;
        const uint64_t j = tile * C + c;
        v[k] = __builtin_nontemporal_load(in + j + ((uint64_t)r << log_lb));
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int g = threadIdx.x + k * NT;
        const int c = g % C, r = g / C;
        const uint64_t j = tile * C + c;
        const uint64_t ns_mask = (1ull << log_ns_w) - 1;
        const uint64_t pos = ((j >> log_ns_w) << (log_ns_w + 9)) + (j & ns_mask) + ((uint64_t)r << log_ns_w);
        __builtin_nontemporal_store(v[k], out + pos);
    }
    (void)R;
}

int main() {
    const uint64_t n = 1ull << 28;
    d2 *a, *b;
    if (hipMalloc(&a, n * 16) || hipMalloc(&b, n * 16)) return 1;
    (void)hipMemset(a, 0, n * 16);
    (void)hipMemset(b, 0, n * 16);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int log_lb = 19;  // M/R = 2^19 lines
    const int C = 16;
    const unsigned tiles = (unsigned)((n >> 9) / C);
    printf("write_Ns\twrite_stride_KiB\tms\tGB/s\n");
    const int ns_list[] = {0, 10, 14, 19, 10, 19};
    for (int li = 0; li < 6; li++) {
        const int lns = ns_list[li];
        for (int it = 0; it < 2; it++) hipLaunchKernelGGL(pass_copy, dim3(tiles), dim3(512), 0, 0, a, b, log_lb, lns, C);
        (void)hipEventRecord(e0, 0);
        for (int it = 0; it < 5; it++) hipLaunchKernelGGL(pass_copy, dim3(tiles), dim3(512), 0, 0, a, b, log_lb, lns, C);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        printf("2^%d\t%llu\t%.3f\t%.0f\n", lns, (unsigned long long)((16ull << lns) / 1024), ms, 2.0 * n * 16 / ms / 1e6);
    }
    return 0;
}
