// tools/probe_bw.hip -- standalone HBM access-pattern probe (not part of the product).
// Measures the bandwidth of tile copies shaped like one Stockham pass:
// a workgroup moves C adjacent columns x R rows of 16-B elements, rows S
// elements apart on the read and/or write side.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_bw.hip -o tools/probe_bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

struct alignas(16) d2 { double x, y; };

template <int Q>
__global__ void tile_copy(const d2* __restrict__ in, d2* __restrict__ out, int C, int R, int log_s,
                          int strided_in, int strided_out, int mode) {
    // thread t handles elements g = t + k*NT of the C*R tile, k < Q; c-fast
    const int NT = blockDim.x;
    const uint64_t tile = blockIdx.x;
    const uint64_t S = 1ull << log_s;         // row stride (elements) = number of columns
    const uint64_t tiles_per_row = S / C;
    const uint64_t rb = tile / tiles_per_row; // row block (0: R rows cover n)
    const uint64_t j0 = (tile % tiles_per_row) * C;
    d2 v[Q];
#pragma unroll
    for (int k = 0; k < Q; k++) {
        const int g = threadIdx.x + k * NT;
        const int c = g % C, r = g / C;
        const uint64_t row = rb * R + r;
        const uint64_t src = strided_in ? (row * S + j0 + c) : (tile * (uint64_t)C * R + g);
        if (mode != 2) v[k] = in[src]; else v[k] = d2{(double)g, 0.0};
    }
    if (mode == 1) {  // read only: keep the values alive
        double s = 0;
#pragma unroll
        for (int k = 0; k < Q; k++) s += v[k].x;
        if (s == 12345.678) out[0] = v[0];
        return;
    }
#pragma unroll
    for (int k = 0; k < Q; k++) {
        const int g = threadIdx.x + k * NT;
        const int c = g % C, r = g / C;
        const uint64_t row = rb * R + r;
        const uint64_t dst = strided_out ? (row * S + j0 + c) : (tile * (uint64_t)C * R + g);
        out[dst] = v[k];
    }
}

int main(int argc, char** argv) {
    const int logn = 28;
    const uint64_t n = 1ull << logn;
    d2 *a, *b;
    if (hipMalloc(&a, n * 16) || hipMalloc(&b, n * 16)) { printf("alloc failed\n"); return 1; }
    hipMemset(a, 0, n * 16);
    hipMemset(b, 0, n * 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct Cfg { int C, R, sin, sout, mode, nt; };
    const int Cs[] = {4, 8, 16, 32, 64};
    const char* mname[] = {"copy", "read", "write"};
    printf("C\tR\tNT\tin\tout\tmode\tGB/s\n");
    for (int mode = 0; mode < 3; mode++)
    for (int sin = 0; sin < 2; sin++)
    for (int sout = 0; sout < 2; sout++) {
        if (mode == 1 && sout) continue;
        if (mode == 2 && sin) continue;
        for (int ci = 0; ci < 5; ci++) {
            const int C = Cs[ci];
            const int R = 8192 / C;  // 128 KiB tiles
            const int Q = 16;
            const int nt = C * R / Q;   // 512
            // R rows of S = n/R elements: the tile grid covers exactly n elements
            int log_s = 0;
            while ((1ull << log_s) * (uint64_t)R < n) log_s++;
            const uint64_t S = 1ull << log_s;
            const uint64_t tiles = n / ((uint64_t)C * R);
            // host-side bound check of the largest index either side can touch
            const uint64_t max_strided = (((tiles - 1) / (S / C)) * R + (R - 1)) * S + (S - C) + (C - 1);
            const uint64_t max_contig = tiles * (uint64_t)C * R - 1;
            if (S * R != n || max_strided >= n || max_contig >= n || S % C) {
                printf("bad geometry C=%d R=%d\n", C, R);
                return 1;
            }
            for (int it = 0; it < 2; it++)
                hipLaunchKernelGGL(tile_copy<16>, dim3(tiles), dim3(nt), 0, 0, a, b, C, R, log_s, sin, sout, mode);
            hipEventRecord(e0, 0);
            const int reps = 5;
            for (int it = 0; it < reps; it++)
                hipLaunchKernelGGL(tile_copy<16>, dim3(tiles), dim3(nt), 0, 0, a, b, C, R, log_s, sin, sout, mode);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= reps;
            const double bytes = (mode == 0 ? 2.0 : 1.0) * n * 16;
            printf("%d\t%d\t%d\t%s\t%s\t%s\t%.0f\n", C, R, nt, sin ? "strided" : "contig", sout ? "strided" : "contig",
                   mname[mode], bytes / ms / 1e6);
        }
    }
    return 0;
}
