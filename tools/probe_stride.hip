// tools/probe_stride.hip -- standalone probe (not part of the product).
// Does the row stride of a strided tile (not just its segment width) set the
// bandwidth of a Stockham-shaped pass?  A workgroup copies a tile of C
// adjacent columns x R rows (16-B elements, rows S elements apart) of a
// 4 GiB array viewed as (n/S rows) x S columns, reading strided and writing
// contiguous (like pass 1) or reading contiguous and writing strided.  The
// segment width C*16 B is held fixed while S sweeps 2^10 .. n/R elements
// (16 KiB .. 8 MiB): a drop at large S points at address translation / DRAM
// page effects rather than segment width.
//   hipcc -O3 -w --offload-arch=gfx950 tools/probe_stride.hip -o tools/probe_stride
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef double __attribute__((ext_vector_type(2))) d2;

template <int Q>
__global__ __launch_bounds__(512) void tile_copy(const d2* __restrict__ in, d2* __restrict__ out, int C, int R, int log_s, int strided_in) {
    const int NT = blockDim.x;
    const uint64_t tile = blockIdx.x;
    const uint64_t S = 1ull << log_s;
    const uint64_t tiles_per_rowblock = S / C;
    const uint64_t rb = tile / tiles_per_rowblock;
    const uint64_t j0 = (tile % tiles_per_rowblock) * C;
    d2 v[Q];
#pragma unroll
    for (int k = 0; k < Q; k++) {
        const int g = threadIdx.x + k * NT;
        const int c = g % C, r = g / C;
        const uint64_t strided = (rb * R + r) * S + j0 + c;
        const uint64_t contig = tile * (uint64_t)C * R + g;
        v[k] = __builtin_nontemporal_load(in + (strided_in ? strided : contig));
    }
#pragma unroll
    for (int k = 0; k < Q; k++) {
        const int g = threadIdx.x + k * NT;
        const int c = g % C, r = g / C;
        const uint64_t strided = (rb * R + r) * S + j0 + c;
        const uint64_t contig = tile * (uint64_t)C * R + g;
        __builtin_nontemporal_store(v[k], out + (strided_in ? contig : strided));
    }
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
    printf("C\tR\tside\tstride_KiB\tGB/s\n");
    const int shapes[][2] = {{8, 1024}, {16, 512}, {32, 256}, {64, 128}};
    for (auto& sh : shapes) {
        const int C = sh[0], R = sh[1];
        const int nt = 512;
        int log_max = 0;
        while ((1ull << log_max) * (uint64_t)R < n) log_max++;
        for (int sin = 1; sin >= 0; sin--)
            for (int log_s = 10; log_s <= log_max; log_s++) {
                const uint64_t S = 1ull << log_s;
                const uint64_t tiles = n / ((uint64_t)C * R);
                if ((n / S) % R) continue;
                for (int it = 0; it < 2; it++)
                    hipLaunchKernelGGL(tile_copy<16>, dim3(tiles), dim3(nt), 0, 0, a, b, C, R, log_s, sin);
                (void)hipEventRecord(e0, 0);
                const int reps = 4;
                for (int it = 0; it < reps; it++)
                    hipLaunchKernelGGL(tile_copy<16>, dim3(tiles), dim3(nt), 0, 0, a, b, C, R, log_s, sin);
                (void)hipEventRecord(e1, 0);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                ms /= reps;
                printf("%d\t%d\t%s\t%llu\t%.0f\n", C, R, sin ? "read-strided" : "write-strided",
                       (unsigned long long)(S * 16 / 1024), 2.0 * n * 16 / ms / 1e6);
            }
    }
    // occupancy: the same C=8 x R=1024 strided-read tile, with dynamic LDS
    // reserved so that only 1, 2 or 3 workgroups fit per CU (the pass kernel
    // holds ~70 KiB LDS and ~126 VGPRs: 2 per CU)
    (void)hipFuncSetAttribute((const void*)tile_copy<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const int lds_kib[] = {0, 40, 60, 75, 100};
    for (int li = 0; li < 5; li++) {
        const int C = 8, R = 1024, log_s = 18;
        const uint64_t tiles = n / ((uint64_t)C * R);
        const size_t lds = (size_t)lds_kib[li] * 1024;
        for (int it = 0; it < 2; it++)
            hipLaunchKernelGGL(tile_copy<16>, dim3(tiles), dim3(512), lds, 0, a, b, C, R, log_s, 1);
        (void)hipEventRecord(e0, 0);
        for (int it = 0; it < 4; it++)
            hipLaunchKernelGGL(tile_copy<16>, dim3(tiles), dim3(512), lds, 0, a, b, C, R, log_s, 1);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= 4;
        printf("occupancy\tC=8 R=1024 read-strided\tlds %d KiB\t%.3f ms\t%.0f GB/s\n", lds_kib[li], ms,
               2.0 * n * 16 / ms / 1e6);
    }
    return 0;
}
