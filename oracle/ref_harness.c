/*
 * oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY.  Builds (in this
 * container only, into oracle/_ref/) a driver around the REFERENCE source
 * itself, compiled where it lies under /root/reference (no source is copied):
 *
 *   gcc ... -DREF_SRC='"<ref>/fourier-parallel-pi-cpu-pthreads.c"' ref_harness.c
 *
 * The reference's main() is renamed away; this driver feeds it an input read
 * from stdin and dumps either
 *   fft  : the natural-order output of all P workers run in test mode
 *          (run_thread, CPU.c:388-512, with test_mode=1 so every worker
 *          scatters its segment to out[], CPU.c:496-499), or
 *   tree : worker q's segment after the tree stage, produced by the
 *          reference's own butterfly_left/butterfly_right (CPU.c:540-576)
 *          driven in the loop order of CPU.c:419-448.
 * With -Dfloat=double the reference's data_t becomes the fp64 variant.
 *
 * usage: ref_harness {fft|tree} N P [q]   (binary data_t[N] on stdin)
 */
#define main pifft_reference_main
#include REF_SRC
#undef main

static int read_all(void* p, size_t n) {
    size_t got = 0;
    while (got < n) {
        size_t r = fread((char*)p + got, 1, n - got, stdin);
        if (r == 0) return -1;
        got += r;
    }
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s {fft|tree} N P [q]\n", argv[0]);
        return 2;
    }
    const char* mode = argv[1];
    uint32_t N = (uint32_t)strtoul(argv[2], NULL, 10);
    uint32_t P = (uint32_t)strtoul(argv[3], NULL, 10);
    uint32_t q = (argc > 4) ? (uint32_t)strtoul(argv[4], NULL, 10) : 0;
    if (N < 2 || !is_power_of_two((int)N) || P < 1 || !is_power_of_two((int)P) || P > N) {
        fprintf(stderr, "bad N/P\n");
        return 2;
    }
    data_t* in = (data_t*)malloc(sizeof(data_t) * N);
    data_t* out = (data_t*)calloc(N, sizeof(data_t));
    if (!in || !out || read_all(in, sizeof(data_t) * N)) {
        fprintf(stderr, "input read failed\n");
        return 2;
    }

    if (strcmp(mode, "fft") == 0) {
        tr_t t;
        memset(&t, 0, sizeof t);
        t.N = N;
        t.P = P;
        t.in = in;
        t.out = out;
        t.test_mode = 1;
        t.no_header = 1;
        for (uint32_t pi = 0; pi < P; pi++) {
            tr_t w = t;
            w.Pi = pi;
            run_thread(&w);
        }
        fwrite(out, sizeof(data_t), N, stdout);
    } else if (strcmp(mode, "tree") == 0) {
        tr_t t;
        memset(&t, 0, sizeof t);
        t.N = N;
        t.P = P;
        t.Pi = q;
        t.tmp_in = (data_t*)malloc(sizeof(data_t) * N);
        t.tmp_out = (data_t*)malloc(sizeof(data_t) * N);
        memcpy(t.tmp_in, in, sizeof(data_t) * N);
        uint32_t size, iter, offset, which_butterfly, which_half;
        for (size = t.N, iter = ilog2(t.P); size > t.N / t.P; size /= 2, iter--) {
            which_butterfly = (t.Pi >> iter);
            offset = which_butterfly * size;
            which_half = ((t.Pi >> (iter - 1)) % 2 == 0);
            if (which_half) butterfly_left(t.tmp_out + offset, t.tmp_in + offset, size, t.N);
            else butterfly_right(t.tmp_out + offset, t.tmp_in + offset, size, t.N);
            swap_scratchpads(&t);
        }
        fwrite(t.tmp_in + (uint64_t)(N / P) * q, sizeof(data_t), N / P, stdout);
    } else {
        fprintf(stderr, "unknown mode %s\n", mode);
        return 2;
    }
    return 0;
}
