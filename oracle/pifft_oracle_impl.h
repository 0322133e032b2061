/*
 * oracle/pifft_oracle_impl.h -- TEST INFRASTRUCTURE ONLY (the parity checker).
 *
 * Precision-generic body of the CPU restatement of the reference "pi" FFT
 * (benchmark/fourier/parallel/pi/cpu/pthreads/fourier-parallel-pi-cpu-pthreads.c,
 * abbreviated CPU.c below).  Included twice by pifft_oracle.c, once with
 * REAL=float/SUF=f32 (the reference's data_t, CPU.c:33-36) and once with
 * REAL=double/SUF=f64 (the reference built with -Dfloat=double).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
 * this code.  The product library never links it.
 *
 * Every arithmetic step keeps the reference's operation order and operand
 * types; the file must be compiled with -ffp-contract=off so that no FMA is
 * formed (the reference's x86-64 -O0/-O2 builds have none).
 */

#define PIFFT_CAT_(a, b) a##b
#define PIFFT_CAT(a, b) PIFFT_CAT_(a, b)
#define CX PIFFT_CAT(oracle_cx_, SUF)
#define FN(name) PIFFT_CAT(PIFFT_CAT(oracle_, name), PIFFT_CAT(_, SUF))

/* CPU.c:584-591 */
static inline CX FN(add)(CX a, CX b) {
    CX c;
    c.re = a.re + b.re;
    c.im = a.im + b.im;
    return c;
}

/* CPU.c:602-609 */
static inline CX FN(sub)(CX a, CX b) {
    CX c;
    c.re = a.re - b.re;
    c.im = a.im - b.im;
    return c;
}

/* CPU.c:620-627: re = ar*br - ai*bi ; im = ar*bi + ai*br, evaluated in REAL. */
static inline CX FN(mul)(CX a, CX b) {
    CX c;
    c.re = a.re * b.re - a.im * b.im;
    c.im = a.re * b.im + a.im * b.re;
    return c;
}

/* CPU.c:644-651: omega(N,k) = (cos(2.0*M_PI/N*k), -sin(2.0*M_PI/N*k)), the
 * argument evaluated in double exactly as ((2.0*M_PI)/N)*k, rounded to REAL.
 * gcc at -O1 and up compiles the reference's cos()/sin() pair into ONE glibc
 * sincos() call, and glibc's sincos differs from its separate cos/sin in the
 * last fp64 bit for ~0.1% of angles.  The pinned reference build (-O2, the
 * fixtures) is the sincos one, so it is spelled out here rather than left to
 * the optimiser (an -O0 build of this file would otherwise drift). */
CX FN(omega)(uint64_t N, uint64_t k) {
    CX o;
    double s, c;
    sincos(2.0 * M_PI / (double)N * (double)k, &s, &c);
    o.re = c;
    o.im = -s;
    return o;
}

/* CPU.c:540-552 (butterfly_left) -- writes the first half of a size-`size`
 * block: out[b] = in[b] + in[b+size/2]. */
static void FN(half_left)(CX* out, const CX* in, uint64_t size) {
    const uint64_t h = size / 2;
    for (uint64_t b = 0; b < h; b++) out[b] = FN(add)(in[b], in[b + h]);
}

/* CPU.c:561-576 (butterfly_right) -- the second half of the block, written
 * here to out[0..size/2): out[b] = (in[b] - in[b+size/2]) * omega(N, b*(N/size)). */
static void FN(half_right)(CX* out, const CX* in, uint64_t size, uint64_t N) {
    const uint64_t h = size / 2;
    const uint64_t step = N / size;
    for (uint64_t b = 0; b < h; b++)
        out[b] = FN(mul)(FN(sub)(in[b], in[b + h]), FN(omega)(N, b * step));
}

/* Tree ("funnel") stage of worker q, CPU.c:419-448.  The reference keeps two
 * full-length scratchpads and addresses the block containing the worker's
 * segment at `offset`; only that block is ever read back, so the restatement
 * keeps the block compacted: stage t maps a block of size s=N>>t to the half
 * (left iff bit log2P-t-1 of q is 0, CPU.c:429) of size s/2.  The result is the
 * worker's N/P segment (the reference's tmp_in[q*N/P ..]) written to `seg`.
 * `work` must hold N/2 + N/4 elements (unused when P == 1). */
void FN(tree)(const CX* in, CX* seg, uint64_t N, uint32_t P, uint32_t q, CX* work) {
    uint32_t lp = 0;
    while ((1u << lp) < P) lp++;
    if (lp == 0) {
        memcpy(seg, in, sizeof(CX) * N);
        return;
    }
    CX* bufA = work;           /* N/2 */
    CX* bufB = work + N / 2;   /* N/4 */
    const CX* cur = in;
    uint64_t size = N;
    for (uint32_t t = 0; t < lp; t++, size /= 2) {
        const uint32_t iter = lp - t;                      /* CPU.c:419 */
        const int left = ((q >> (iter - 1)) % 2 == 0);     /* CPU.c:429 */
        CX* dst = (t == lp - 1) ? seg : ((t % 2 == 0) ? bufA : bufB);
        if (left) FN(half_left)(dst, cur, size);
        else FN(half_right)(dst, cur, size, N);
        cur = dst;
    }
}

/* Cylinder ("tube") stage, CPU.c:463-478: log2(M) radix-2 DIF passes of the
 * reference's butterfly (CPU.c:522-531), every twiddle omega(N, b*(N/size))
 * taken with the GLOBAL N.  Ping-pongs between seg and tmp; returns the buffer
 * holding the result (the reference's tmp_in after the last swap). */
CX* FN(cylinder)(CX* seg, CX* tmp, uint64_t M, uint64_t N) {
    CX* a = seg;
    CX* b = tmp;
    for (uint64_t size = M; size > 1; size /= 2) {
        for (uint64_t off = 0; off < M; off += size) {
            FN(half_left)(b + off, a + off, size);
            FN(half_right)(b + off + size / 2, a + off, size, N);
        }
        CX* t = a; a = b; b = t;                       /* swap_scratchpads */
    }
    return a;
}

/* One worker of the reference in test mode (CPU.c:388-512 incl. the scatter
 * at :496-499): tree + cylinder, then out[bit_reverse(q*M+i, log2 N)] = seg[i].
 * Optionally returns the two stage times in ms (CPU.c:414-481). */
int FN(worker)(const CX* in, CX* out, uint64_t N, uint32_t P, uint32_t q,
               double* ms_tree, double* ms_cyl) {
    const uint64_t M = N / P;
    const uint32_t lg = oracle_ilog2_u64(N);
    CX* seg = (CX*)malloc(sizeof(CX) * M);
    CX* tmp = (CX*)malloc(sizeof(CX) * M);
    CX* work = (P > 1) ? (CX*)malloc(sizeof(CX) * (N / 2 + N / 4 + 1)) : NULL;
    if (!seg || !tmp || (P > 1 && !work)) {
        free(seg); free(tmp); free(work);
        return -1;
    }
    double t0 = oracle_now_ms();
    FN(tree)(in, seg, N, P, q, work);
    double t1 = oracle_now_ms();
    CX* res = FN(cylinder)(seg, tmp, M, N);
    double t2 = oracle_now_ms();
    if (ms_tree) *ms_tree = t1 - t0;
    if (ms_cyl) *ms_cyl = t2 - t1;
    if (out) {
        for (uint64_t i = 0; i < M; i++)
            out[oracle_bit_reverse(q * M + i, lg)] = res[i];
    }
    free(seg); free(tmp); free(work);
    return 0;
}

/* Tree stage only, for the post-tree fixtures: worker q's N/P segment. */
int FN(tree_segment)(const CX* in, CX* seg, uint64_t N, uint32_t P, uint32_t q) {
    CX* work = (P > 1) ? (CX*)malloc(sizeof(CX) * (N / 2 + N / 4 + 1)) : NULL;
    if (P > 1 && !work) return -1;
    FN(tree)(in, seg, N, P, q, work);
    free(work);
    return 0;
}

typedef struct {
    const CX* in;
    CX* out;
    uint64_t N;
    uint32_t P, q;
    double ms_tree, ms_cyl;
    int rc;
} PIFFT_CAT(oracle_job_, SUF);

static void* FN(thread_main)(void* arg) {
    PIFFT_CAT(oracle_job_, SUF)* j = (PIFFT_CAT(oracle_job_, SUF)*)arg;
    j->rc = FN(worker)(j->in, j->out, j->N, j->P, j->q, &j->ms_tree, &j->ms_cyl);
    return NULL;
}

/* The whole transform, P workers (CPU.c:312-380).  Workers run on up to
 * `nthreads` pthreads (0 = one per worker); each writes a disjoint set of
 * natural-order output bins.  ms_tree/ms_cyl receive worker 0's stage times
 * (the reference prints worker 0's timers, CPU.c:485-491); ms_wall the time
 * across the join. */
int FN(fft)(const CX* in, CX* out, uint64_t N, uint32_t P, uint32_t nthreads,
            double* ms_tree, double* ms_cyl, double* ms_wall) {
    if (N < 2 || (N & (N - 1)) || P == 0 || (P & (P - 1)) || P > N) return -1;
    if (nthreads == 0 || nthreads > P) nthreads = P;
    PIFFT_CAT(oracle_job_, SUF)* jobs =
        (PIFFT_CAT(oracle_job_, SUF)*)calloc(P, sizeof(PIFFT_CAT(oracle_job_, SUF)));
    pthread_t* tids = (pthread_t*)calloc(nthreads, sizeof(pthread_t));
    if (!jobs || !tids) { free(jobs); free(tids); return -1; }
    for (uint32_t q = 0; q < P; q++) {
        jobs[q].in = in; jobs[q].out = out; jobs[q].N = N; jobs[q].P = P; jobs[q].q = q;
    }
    double w0 = oracle_now_ms();
    int rc = 0;
    for (uint32_t base = 0; base < P; base += nthreads) {
        uint32_t n = (P - base < nthreads) ? P - base : nthreads;
        for (uint32_t k = 0; k < n; k++)
            if (pthread_create(&tids[k], NULL, FN(thread_main), &jobs[base + k])) rc = -1;
        for (uint32_t k = 0; k < n; k++) pthread_join(tids[k], NULL);
    }
    double w1 = oracle_now_ms();
    for (uint32_t q = 0; q < P; q++) rc |= jobs[q].rc;
    if (ms_tree) *ms_tree = jobs[0].ms_tree;
    if (ms_cyl) *ms_cyl = jobs[0].ms_cyl;
    if (ms_wall) *ms_wall = w1 - w0;
    free(jobs); free(tids);
    return rc;
}

/* Synthetic input shared by every leg: element e of the
 * stream takes draws 2e and 2e+1 of splitmix64(seed) for re and im, each mapped
 * to (2u-1)/sqrt(n) with u = top 53 bits / 2^53 -- the reference's
 * U[-1,1]/sqrt(N) distribution (CPU.c:244-247) from a portable generator.
 * 2u-1 is exact and the division is correctly rounded, so the device
 * generator (pifft_generate_device) reproduces these bytes exactly. */
void FN(generate)(CX* x, uint64_t count, uint64_t n, uint64_t seed, uint64_t first) {
    const double scale = sqrt((double)n);
    for (uint64_t e = 0; e < count; e++) {
        uint64_t d = 2 * (first + e);
        x[e].re = (REAL)((2.0 * oracle_u01(seed, d) - 1.0) / scale);
        x[e].im = (REAL)((2.0 * oracle_u01(seed, d + 1) - 1.0) / scale);
    }
}

#undef CX
#undef FN
