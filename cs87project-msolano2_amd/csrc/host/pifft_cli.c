/*
 * pifft_cli.c -- C host of the MI355X pi-FFT: the reference's command line
 * and output contract, with the transform running on GPUs through the
 * C-ABI of libpifft.so (include/pifft.h).
 *
 * Mirrors benchmark/fourier/parallel/pi/cpu/pthreads/fourier-parallel-pi-cpu-pthreads.c
 * (CPU.c):   main            CPU.c:98-113
 *            setup_from_args CPU.c:125-211   same flags, same messages
 *            initialize_data CPU.c:220-275   (synthetic input, or the -t vector)
 *            run             CPU.c:312-380   (workers -> GPUs instead of pthreads)
 *            show_usage, print_input/print_output, verify_results (CPU.c:293-302, 659-705)
 *
 *   pifft { -n <n> -p <p> [-o] | -t } [-f 32|64] [-b batch] [-s seed] [-g gpus]
 *         [-w file] [-r] [-u] [-x] [-W warmups] [-l]
 *
 * Output: the reference's 5-column TSV "n p total stage1 stage2" in ms
 * (CPU.c:485-492), once.  stage 1 = tree, stage 2 = local FFT (+ reorder),
 * each the device wall time from before its first launch to after its last
 * (the reference's tm_funnel / tm_tube wall-clock timers, CPU.c:414-481).
 * With several GPUs the time is the slowest GPU's (the reference prints worker
 * 0's own timers without a barrier; here all GPUs are waited for).
 * Extensions: -f precision (default 32 = the reference's data_t), -b batch of
 * independent transforms, -s seed (default: hash of the time, as CPU.c:244),
 * -g number of GPUs the P workers are spread over (default 1), -w dump the
 * natural-order output (binary), -r keep the output in the reference's own
 * scratch order (bit-reversed, tmp_in before CPU.c:496-499's scatter; no
 * reorder launch), -u keep the tree its own launch (never fused into the first
 * pass: stage 1 = the tree alone, as the reference's funnel timer, for the
 * cost-law fit of analyze-results.R:56), -x extra columns (GFLOP/s, GB/s over
 * the wall total, then the kernel-only stage sums: stage times without the
 * gaps between launches),
 * -W untimed warm-up runs before the timed one (default 1; code-object load),
 * -l list GPUs (the how-many-* utilities), -R rehearse a -g split with every
 * plan on GPU 0 (a one-GPU box runs the multi-plan path).  -n is parsed as
 * 64-bit.
 *
 * -t with -g G > 1 also checks the split itself: the G-plan result against a
 * one-GPU all-worker plan of the same input (rel-L2 within the north star's
 * tolerance) and every plan's bins against the same worker range replayed on
 * GPU 0 (bit for bit) -- the multi-GPU path proving its own output.
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "pifft.h"

#define stderr_out(...) fprintf(stderr, __VA_ARGS__), fflush(stderr)
#define print_out(...) printf(__VA_ARGS__), fflush(stdout)

typedef struct tr {
    uint64_t N;          /* input size                         (CPU.c:41) */
    uint32_t P;          /* number of workers                  (CPU.c:42) */
    void* in;            /* input                              (CPU.c:44) */
    void* out;           /* output, natural order              (CPU.c:45) */
    uint32_t test_mode;  /* -t                                 (CPU.c:48) */
    uint32_t no_header;  /* -o                                 (CPU.c:49) */
    int prec;            /* -f: 32 or 64 */
    uint32_t batch;      /* -b */
    uint64_t seed;       /* -s */
    int seed_given;
    uint32_t gpus;       /* -g */
    const char* dump;    /* -w */
    int extra;           /* -x */
    int warmups;         /* -W */
    int bitrev;          /* -r */
    int separate_tree;   /* -u */
    int rehearse;        /* -R */
} tr_t;

static void show_usage(void) {
    print_out("\nusage:\n"
              "  pifft { -n <n> -p <p> [-o] | -t } [-f 32|64] [-b <batch>] [-s <seed>]\n"
              "        [-g <gpus>] [-w <file>] [-r] [-u] [-x] [-W <warmups>] [-l] [-R]\n"
              "\noptions:\n"
              "  -n <n>     power of two input size\n"
              "  -p <p>     power of two number of processors (less than n)\n"
              "  -o         omit timing headers\n"
              "  -t         compare against precomputed input/output\n"
              "  -f 32|64   precision (default 32, the reference's data_t)\n"
              "  -b <b>     batch of independent transforms (default 1)\n"
              "  -s <seed>  input seed (default: hash of the time)\n"
              "  -g <g>     GPUs to spread the p workers over (default 1)\n"
              "  -w <file>  write the output (binary data_t; natural order unless -r)\n"
              "  -r         output in the reference's bit-reversed scratch order\n"
              "  -u         tree stage as its own launch (stage 1 = the tree alone)\n"
              "  -x         extra columns: GFLOP/s, algorithmic GB/s, kernel-only stage 1 / 2 ms\n"
              "  -W <w>     untimed warm-up runs (default 1)\n"
              "  -l         list GPUs and exit\n"
              "  -R         rehearse the -g split with every plan on GPU 0\n"
              "\n");
}

static int is_power_of_two_u64(uint64_t x) { return x && !(x & (x - 1)); }

/* CPU.c:769-774 (Wang hash), used to seed from the time like CPU.c:244 */
static uint32_t hash(uint32_t x) {
    x = (x + 0x7ed55d16U) + (x << 12);
    x = (x ^ 0xc761c23cU) ^ (x >> 19);
    x = (x + 0x165667b1U) + (x << 5);
    x = (x + 0xd3a2646cU) ^ (x << 9);
    x = (x + 0xfd7046c5U) + (x << 3);
    x = (x ^ 0xb55a4f09U) ^ (x >> 16);
    return x;
}

static int parse_u64(const char* s, uint64_t* v) {
    char* end = NULL;
    if (!s || !*s) return -1;
    unsigned long long x = strtoull(s, &end, 10);
    if (*end) return -1;
    *v = (uint64_t)x;
    return 0;
}

/* CPU.c:125-211: later options override earlier ones (so "-t -n 16" keeps the
 * test vector but transforms 16 points, as in the reference). */
int setup_from_args(tr_t* t, int argc, char** argv) {
    int ret;
    uint64_t num = 0;
    memset(t, 0, sizeof(tr_t));
    t->prec = PIFFT_F32;
    t->batch = 1;
    t->gpus = 1;
    t->warmups = 1;
    while ((ret = getopt(argc, argv, "n:p:tof:b:s:g:w:ruxW:lR")) != -1) {
        switch (ret) {
            case 'n':
                if (parse_u64(optarg, &num) || !(num > 1) || !is_power_of_two_u64(num)) {
                    stderr_out("Invalid input size (should be 2^i for i>0)\n");
                    show_usage();
                    goto err;
                }
                t->N = num;
                break;
            case 'p':
                if (parse_u64(optarg, &num) || !(num > 0) || !is_power_of_two_u64(num) || num > 0x80000000ULL) {
                    stderr_out("Invalid number of procs (should be 2^i for i>0)\n");
                    show_usage();
                    goto err;
                }
                t->P = (uint32_t)num;
                break;
            case 'o':
                t->no_header = 1;
                break;
            case 't':
                print_out("Test mode (ignoring provided input size, if any)...\n");
                t->N = 8;
                t->test_mode = 1;
                break;
            case 'f':
                if (strcmp(optarg, "32") && strcmp(optarg, "64")) {
                    stderr_out("Invalid precision (should be 32 or 64)\n");
                    show_usage();
                    goto err;
                }
                t->prec = atoi(optarg);
                break;
            case 'b':
                if (parse_u64(optarg, &num) || num < 1 || num > 0xFFFFFFFFULL) {
                    stderr_out("Invalid batch (should be >= 1)\n");
                    goto err;
                }
                t->batch = (uint32_t)num;
                break;
            case 's':
                if (parse_u64(optarg, &num)) {
                    stderr_out("Invalid seed\n");
                    goto err;
                }
                t->seed = num;
                t->seed_given = 1;
                break;
            case 'g':
                if (parse_u64(optarg, &num) || !(num > 0) || !is_power_of_two_u64(num) || num > 1024) {
                    stderr_out("Invalid number of GPUs (should be 2^i)\n");
                    goto err;
                }
                t->gpus = (uint32_t)num;
                break;
            case 'w':
                t->dump = optarg;
                break;
            case 'r':
                t->bitrev = 1;
                break;
            case 'u':
                t->separate_tree = 1;
                break;
            case 'x':
                t->extra = 1;
                break;
            case 'R':
                t->rehearse = 1;
                break;
            case 'W':
                if (parse_u64(optarg, &num) || num > 1000) {
                    stderr_out("Invalid warm-up count\n");
                    goto err;
                }
                t->warmups = (int)num;
                break;
            case 'l': {
                int n = pifft_gpu_count();
                if (n < 0) {
                    stderr_out("%s\n", pifft_last_error());
                    goto err;
                }
                print_out("%d\n", n);
                exit(EXIT_SUCCESS);
            }
            case '?':
                stderr_out("Unknown or missing arg %c\n", optopt);
                show_usage();
                goto err;
        }
    }
    if (!t->N) {
        stderr_out("Missing option: -n\n");
        show_usage();
        goto err;
    }
    if (!t->P) {
        stderr_out("Missing option: -p\n");
        show_usage();
        goto err;
    }
    if (t->P > t->N) {
        stderr_out("More processors than inputs!\n");
        show_usage();
        goto err;
    }
    {
        int ngpu = pifft_gpu_count();
        if (ngpu < 1) {
            stderr_out("No GPU available (%s)\n", pifft_last_error());
            goto err;
        }
        if (t->gpus > (uint32_t)ngpu && !t->rehearse) {
            stderr_out("Too many GPUs! (only %d GPUs available)\n", ngpu);
            goto err;
        }
        if (t->gpus > t->P) t->gpus = t->P; /* at least one worker per GPU */
    }
    return 0;
err:
    stderr_out("Could not setup the transform from the cmdline args\n");
    return -1;
}

static size_t esz(const tr_t* t) { return t->prec == PIFFT_F64 ? 16 : 8; }

static double re_at(const tr_t* t, const void* a, uint64_t i) {
    return t->prec == PIFFT_F64 ? ((const double*)a)[2 * i] : ((const float*)a)[2 * i];
}
static double im_at(const tr_t* t, const void* a, uint64_t i) {
    return t->prec == PIFFT_F64 ? ((const double*)a)[2 * i + 1] : ((const float*)a)[2 * i + 1];
}
static void set_at(const tr_t* t, void* a, uint64_t i, double re, double im) {
    if (t->prec == PIFFT_F64) {
        ((double*)a)[2 * i] = re;
        ((double*)a)[2 * i + 1] = im;
    } else {
        ((float*)a)[2 * i] = (float)re;
        ((float*)a)[2 * i + 1] = (float)im;
    }
}

/* splitmix64 -> (2u-1)/sqrt(N): the same bytes as pifft_generate_device */
static uint64_t splitmix64(uint64_t seed, uint64_t draw) {
    uint64_t z = seed + (draw + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static void print_input(const tr_t* t) {
    print_out("Input:\n");
    for (uint64_t b = 0; b < t->N; b++) print_out("%.1f+%.1fi, ", re_at(t, t->in, b), im_at(t, t->in, b));
    print_out("\n");
}

static void print_output(const tr_t* t) {
    print_out("Output:\n");
    for (uint64_t b = 0; b < t->N; b++) print_out("%.1f+%.1fi, ", re_at(t, t->out, b), im_at(t, t->out, b));
    print_out("\n");
}

/* CPU.c:689-705 */
static void verify_results(const tr_t* t) {
    static const double want[8] = {4, 0, 0, 0, -4, 0, 0, 0};
    static const double want_brev[8] = {4, -4, 0, 0, 0, 0, 0, 0};  /* tmp_in order */
    int ok = t->N >= 8;
    const double* w = t->bitrev ? want_brev : want;
    for (int i = 0; ok && i < 8; i++) ok = re_at(t, t->out, i) == w[i] && im_at(t, t->out, i) == 0.0;
    print_out(ok ? "Output is correct. Test passed.\n\n" : "Output is incorrect! Test failed.\n\n");
}

/* CPU.c:220-275 */
static int initialize_data(tr_t* t) {
    const uint64_t total = t->N * (uint64_t)t->batch;
    t->in = calloc(total, esz(t));
    t->out = calloc(total, esz(t));
    if (!t->in || !t->out) {
        perror("malloc error");
        stderr_out("Could not initialize the data\n");
        return -1;
    }
    if (!t->test_mode) {
        uint64_t seed = t->seed_given ? t->seed : (uint64_t)hash((uint32_t)time(NULL));
        const double scale = sqrt((double)t->N);
        for (uint64_t e = 0; e < total; e++) {
            double ur = (double)(splitmix64(seed, 2 * e) >> 11) * 0x1.0p-53;
            double ui = (double)(splitmix64(seed, 2 * e + 1) >> 11) * 0x1.0p-53;
            set_at(t, t->in, e, (2.0 * ur - 1.0) / scale, (2.0 * ui - 1.0) / scale);
        }
    } else {
        /* 0,1,0,1,0,1,0,1 (CPU.c:251-260) in every transform of the batch */
        for (uint32_t b = 0; b < t->batch; b++)
            for (uint64_t i = 0; i < 8 && i < t->N; i++) set_at(t, t->in, b * t->N + i, (double)(i & 1), 0.0);
        print_input(t);
    }
    return 0;
}

static void cleanup_data(tr_t* t) {
    free(t->in);
    free(t->out);
    t->in = t->out = NULL;
}

static int device_of(const tr_t* t, uint32_t g) { return t->rehearse ? 0 : (int)g; }

/* -t with -g G > 1: the split checks itself (see the header).  Returns 0 when
 * both checks pass, 1 when one fails, -1 on an error. */
static int check_split(const tr_t* t, pifft_plan* const* plans) {
    const uint64_t total = t->N * (uint64_t)t->batch;
    const uint32_t G = t->gpus, per = t->P / G;
    void* ref = calloc(total, esz(t));
    void* rep = malloc(total * esz(t));
    pifft_plan* one = NULL;
    int rc = -1;
    if (!ref || !rep) goto out;
    /* the whole transform on GPU 0, all P workers (same order as the split) */
    if (pifft_plan_create_slices(&one, t->N, t->P, 0, t->P, t->batch, t->prec, 0,
                                 t->bitrev ? PIFFT_OUT_BITREV : PIFFT_OUT_NATURAL) ||
        pifft_execute(one, t->in, ref, NULL, NULL)) {
        stderr_out("%s\n", pifft_last_error());
        goto out;
    }
    pifft_plan_destroy(one);
    one = NULL;
    double num = 0, den = 0;
    for (uint64_t i = 0; i < total; i++) {
        const double dr = re_at(t, t->out, i) - re_at(t, ref, i), di = im_at(t, t->out, i) - im_at(t, ref, i);
        num += dr * dr + di * di;
        den += re_at(t, ref, i) * re_at(t, ref, i) + im_at(t, ref, i) * im_at(t, ref, i);
    }
    const double err = den > 0 ? sqrt(num / den) : sqrt(num);
    const double tol = t->prec == PIFFT_F64 ? 1e-12 : 1e-5 * log2((double)t->N);
    /* every plan's worker range again, on GPU 0: its bins bit for bit */
    int same = 1;
    for (uint32_t g = 0; g < G && same; g++) {
        memset(rep, 0xff, total * esz(t));  /* NaN pattern: positions the plan does not write */
        pifft_plan* p = NULL;
        if (pifft_plan_create_slices(&p, t->N, t->P, g * per, per, t->batch, t->prec, 0,
                                     t->bitrev ? PIFFT_OUT_BITREV : PIFFT_OUT_SLICES) ||
            pifft_execute(p, t->in, rep, NULL, NULL)) {
            stderr_out("%s\n", pifft_last_error());
            if (p) pifft_plan_destroy(p);
            goto out;
        }
        pifft_plan_destroy(p);
        const size_t e = esz(t);
        uint64_t written = 0;
        for (uint64_t i = 0; i < total && same; i++) {
            static const unsigned char nanpat[16] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff,
                                                     0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
            const char* a = (const char*)rep + i * e;
            if (!memcmp(a, nanpat, e)) continue;
            written++;
            same = !memcmp(a, (const char*)t->out + i * e, e);
        }
        same = same && written == total / G;
    }
    print_out("Split check (%u plans vs one GPU): rel-L2 %.3e (tolerance %.1e), worker ranges replayed bit for bit: %s\n",
              G, err, tol, same ? "yes" : "NO");
    print_out(err <= tol && same ? "Split check passed.\n\n" : "Split check FAILED.\n\n");
    rc = err <= tol && same ? 0 : 1;
out:
    if (one) pifft_plan_destroy(one);
    free(ref);
    free(rep);
    return rc;
}

/* CPU.c:312-380: the P workers go to t->gpus GPUs, P/gpus consecutive workers
 * each, and run concurrently; no data moves between GPUs.  Returns 0, -1 on
 * an error (as the reference's run), or 1 when -t -g G's split check ran and
 * failed (main exits with EXIT_FAILURE on anything but 0). */
int run(tr_t* t) {
    pifft_plan* plans[1024] = {0};
    const uint32_t G = t->gpus;
    const uint32_t per = t->P / G;
    int rc = -1, split = 0;
    double s1 = 0, s2 = 0;
    if (initialize_data(t)) goto done;
    const int sep = t->separate_tree ? PIFFT_SEPARATE_TREE : 0;
    for (uint32_t g = 0; g < G; g++) {
        int r = (G == 1) ? pifft_plan_create_slices(&plans[g], t->N, t->P, 0, t->P, t->batch, t->prec, 0,
                                                    (t->bitrev ? PIFFT_OUT_BITREV : PIFFT_OUT_NATURAL) | sep)
                         : pifft_plan_create_slices(&plans[g], t->N, t->P, g * per, per, t->batch, t->prec,
                                                    device_of(t, g), (t->bitrev ? PIFFT_OUT_BITREV : PIFFT_OUT_SLICES) | sep);
        if (r) {
            stderr_out("(GPU %u): %s\n", g, pifft_last_error());
            goto done;
        }
    }
    for (int w = 0; w < t->warmups; w++) {
        if (pifft_execute_group(plans, (int)G, t->in, NULL, NULL, NULL)) {
            stderr_out("%s\n", pifft_last_error());
            goto done;
        }
    }
    if (pifft_execute_group(plans, (int)G, t->in, t->out, &s1, &s2)) {
        stderr_out("%s\n", pifft_last_error());
        goto done;
    }
    if (!t->test_mode) {
        if (!t->no_header) print_out("n\tp\ttime (total)\ttime (stage 1)\ttime (stage 2)%s\n",
                                     t->extra ? "\tGFLOP/s\tGB/s\tkernels (stage 1)\tkernels (stage 2)" : "");
        if (t->extra) {
            pifft_plan_info info;
            uint64_t bytes = 0;
            for (uint32_t g = 0; g < G; g++) {
                pifft_plan_get_info(plans[g], &info);
                for (int i = 0; i < info.num_launches && i < PIFFT_MAX_LAUNCH_INFO; i++) bytes += info.launch_bytes[i];
            }
            const double ms = s1 + s2;
            const double flops = 5.0 * (double)t->N * log2((double)t->N) * t->batch;
            double k1 = 0, k2 = 0;
            if (pifft_execute_group_kernel_times(plans, (int)G, &k1, &k2)) {
                stderr_out("%s\n", pifft_last_error());
                goto done;
            }
            print_out("%llu\t%u\t%lf\t%lf\t%lf\t%lf\t%lf\t%lf\t%lf\n", (unsigned long long)t->N, t->P, ms, s1, s2,
                      flops / (ms * 1e6), (double)bytes / G / (ms * 1e6), k1, k2);
        } else {
            print_out("%llu\t%u\t%lf\t%lf\t%lf\n", (unsigned long long)t->N, t->P, s1 + s2, s1, s2);
        }
    } else {
        print_output(t);
        verify_results(t);
        if (G > 1) {
            /* test-only (PIFFT_TUNING=1 PIFFT_FAULT=split_check): one wrong
             * output bit, so the failing branch of the check runs */
            const char* tu = getenv("PIFFT_TUNING");
            const char* fa = getenv("PIFFT_FAULT");
            if (tu && !strcmp(tu, "1") && fa && !strcmp(fa, "split_check")) ((unsigned char*)t->out)[0] ^= 1;
            split = check_split(t, plans);
            if (split < 0) goto done;
        }
    }
    if (t->dump) {
        FILE* f = fopen(t->dump, "wb");
        if (!f || fwrite(t->out, esz(t), t->N * (uint64_t)t->batch, f) != t->N * (uint64_t)t->batch) {
            perror("output dump");
            if (f) fclose(f);
            goto done;
        }
        fclose(f);
    }
    /* a failed split check ran to the end but is not a success: exit status 1 */
    rc = split ? 1 : 0;
done:
    for (uint32_t g = 0; g < G; g++)
        if (plans[g]) pifft_plan_destroy(plans[g]);
    cleanup_data(t);
    if (rc < 0) stderr_out("Could not run the transform\n");
    return rc;
}

int main(int argc, char** argv) {
    tr_t t;
    if (setup_from_args(&t, argc, argv)) exit(EXIT_FAILURE);
    if (run(&t)) exit(EXIT_FAILURE);
    exit(EXIT_SUCCESS);
}
