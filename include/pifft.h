/*
 * include/pifft.h -- C-ABI of libpifft.so, the MI355X-native "pi" FFT.
 *
 * Drop-in boundary for the reference CPU path
 *   benchmark/fourier/parallel/pi/cpu/pthreads/fourier-parallel-pi-cpu-pthreads.c
 * (abbreviated CPU.c).  The reference has no library API: its C entry points
 * are setup_from_args (CPU.c:125), run (CPU.c:312) and the per-worker
 * run_thread (CPU.c:388), which together compute a radix-2 DIF FFT split over
 * P workers that never exchange data.  This header is the shim those entry
 * points call instead (see cs87project-msolano2_amd/csrc/host/pifft_cli.c for
 * the C host that keeps the reference CLI, and INTEGRATION.md for the one-line
 * change to the reference's run()).
 *
 * Conventions (mirroring the reference): functions return 0 on success and
 * -1 on error (CPU.c:102-109, 208-210); the error text is then available from
 * pifft_last_error() (the reference prints to stderr instead).  No C++
 * exception crosses this boundary.  Plain pointers and sizes only.
 *
 * Data: interleaved complex, {float re, im} (PIFFT_F32, the reference's data_t,
 * CPU.c:33-36) or {double re, im} (PIFFT_F64, the reference built with
 * -Dfloat=double).  Transform: unnormalised forward DFT
 * X[k] = sum_n x[n] e^{-2 pi i nk/N}, natural-order input and output (the
 * reference's `out` after its bit-reversed scatter, CPU.c:496-499).
 *
 * Workers: worker q of P owns the natural-order output bins
 *   bitrev_{log2 P}(q) + P*k,  k < N/P
 * (the reference's segment q of its bit-reversed scratch).  A plan computes a
 * contiguous range of workers [first, first+count) on one GPU; a plan with
 * count == P on one GPU is the whole transform.
 *
 * Plans depend only on the arguments: the planner's PIFFT_* tuning variables
 * (used by the repository's measurement tools) are read only when
 * PIFFT_TUNING=1 is set in the environment.
 */
#ifndef PIFFT_H
#define PIFFT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PIFFT_F32 32
#define PIFFT_F64 64

/* plan flags */
#define PIFFT_OUT_NATURAL 0 /* device output in natural order (needs count == P):
                               an interleave launch after the last pass, or, for
                               outputs that stay in L2 / the Infinity Cache, the
                               last pass storing natural order itself          */
#define PIFFT_OUT_SLICES 1  /* device output slice-major: worker q's N/P bins
                               Z_q[k] = X[bitrev(q) + P k] contiguous, q = first.. */
#define PIFFT_OUT_BITREV 2  /* the reference's own scratch order (tmp_in after the
                               cylinder, CPU.c:463-478, before its scatter
                               CPU.c:496-499): slice-major, each slice in
                               bit-reversed order, S_q[i] = Z_q[bitrev_{log2 M}(i)]
                               = X[bitrev_{log2 N}(q M + i)]; with all workers on
                               one plan this is X in bit-reversed order (no
                               interleave launch) */

#define PIFFT_SEPARATE_TREE 4 /* flag bit, OR-ed with one of the orders above: never
                               fuse the tree into the first local-FFT pass, so the
                               stage-1 time is the tree ("funnel") alone, as the
                               reference's tm_funnel (CPU.c:414-448) -- the column
                               its cost-law fit regresses on n(p-1)/p
                               (analyze-results.R:56); CLI -u                  */

typedef struct pifft_plan pifft_plan;

#define PIFFT_MAX_LAUNCH_INFO 256 /* launches described by pifft_plan_info */

/* Layout version of pifft_plan_info and of this header's entry points,
 * bumped at every change a binding compiled against an older header would
 * misread: 1 rounds 1-3; 2 round 4 (chunk_pairs removed, launch_mode added);
 * 3 round 5 (pifft_abi_version added; the struct is unchanged from 2).  A
 * binding checks pifft_abi_version() == the PIFFT_ABI_VERSION it was written
 * against before reading a pifft_plan_info -- cs87project-msolano2_amd/pifft.py
 * does. */
#define PIFFT_ABI_VERSION 3
int pifft_abi_version(void);

typedef struct pifft_plan_info {
    uint64_t n;              /* transform length N                                */
    uint32_t workers;        /* P                                                 */
    uint32_t first_worker;   /* workers [first_worker, first_worker+num_workers)  */
    uint32_t num_workers;
    uint32_t batch;          /* independent transforms per execute               */
    int32_t prec;            /* PIFFT_F32 | PIFFT_F64                             */
    int32_t device;          /* HIP device ordinal                                */
    int32_t flags;
    uint64_t local_n;        /* M = N/P, the per-worker ("cylinder") FFT length   */
    uint64_t in_elems;       /* complex elements expected at d_in  (batch*N)      */
    uint64_t out_elems;      /* complex elements written to d_out                 */
    uint64_t workspace_bytes;
    int32_t num_launches;    /* kernel launches per execute                        */
    int32_t num_passes;      /* Stockham passes of the local FFT                   */
    int32_t tree_launches;   /* launches of the tree ("funnel") stage              */
    int32_t radix[8];        /* LDS-resident sub-FFT length of each pass           */
    int32_t lines[8];        /* columns per workgroup of each pass                 */
    uint64_t launch_bytes[PIFFT_MAX_LAUNCH_INFO]; /* algorithmic bytes of each launch
                                  (read+write of the data, twiddle tables excluded) */
    int32_t launch_kind[PIFFT_MAX_LAUNCH_INFO]; /* 1 tree, 2 pass, 3 interleave, 4 tree fused
                                  into a pass */
    int32_t launch_fn[PIFFT_MAX_LAUNCH_INFO]; /* kernel of each launch: launches with the same id
                                  run the same kernel function (ids 0, 1, ... in order
                                  of first use) -- what rocprof aggregates per kernel */
    int32_t vpt[8];          /* complex values per thread of each pass (16; 32 for the
                                packed fp32 passes of large transforms)            */
    int32_t launch_mode[PIFFT_MAX_LAUNCH_INFO]; /* k_pass MODE of each pass launch (bits 0-1: single /
                                  first / later / fused-tree pass, 4 bit-reversed store, 8
                                  worker-interleaved; other bits reserved, never set);
                                  0 for tree and interleave launches */
    int32_t layout;          /* bit 0: worker-interleaved passes (all P <= 16 workers of a
                                natural-order plan -- P = 32 too for the one-launch plans
                                of P N/P <= 8192 values: the last pass writes natural order);
                                bit 1: the last pass stores natural order from the
                                slice-major layout (small outputs); neither: slice-major
                                passes (+ an interleave launch for natural order)   */
} pifft_plan_info;

/* Last error message of the calling thread ("" if none). */
const char* pifft_last_error(void);

/* Number of visible HIP devices, or -1 (replaces how-many-concurrent-blocks.cu
 * and the core count check of CPU.c:200, 835-837). */
int pifft_gpu_count(void);

/* Whole transform on the current device: all P workers, natural-order output
 * (the reference's run(), CPU.c:312-380).  n, workers: powers of two, 2 <= n,
 * 1 <= workers <= n (CPU.c:139-198).  batch >= 1 transforms laid out back to
 * back.  prec: PIFFT_F32 or PIFFT_F64. */
int pifft_plan_create(pifft_plan** plan, uint64_t n, uint32_t workers, uint32_t batch,
                      int prec);

/* Workers [first, first+count) of a P-worker split on `device` (one GPU of a
 * multi-GPU job; the reference's run_thread for each of those Pi).  count must
 * be a power of two dividing first.  flags: PIFFT_OUT_NATURAL (only when
 * count == workers), PIFFT_OUT_SLICES or PIFFT_OUT_BITREV, optionally with
 * PIFFT_SEPARATE_TREE. */
int pifft_plan_create_slices(pifft_plan** plan, uint64_t n, uint32_t workers, uint32_t first,
                             uint32_t count, uint32_t batch, int prec, int device, int flags);

void pifft_plan_destroy(pifft_plan* plan);

/* The plan pifft_plan_create_slices would build, described without touching
 * a device or allocating (host-side planning only; device = -1 in info). */
int pifft_plan_dry_run(uint64_t n, uint32_t workers, uint32_t first, uint32_t count, uint32_t batch,
                       int prec, int flags, pifft_plan_info* info);

int pifft_plan_get_info(const pifft_plan* plan, pifft_plan_info* info);

/* Diagnostics (no reference counterpart): the registry of compiled k_pass
 * instances, and which of them a plan would launch.  pifft_instance_desc
 * writes {prec, R, C, MODE, NTS, LP, VPT} of instance i (< pifft_instance_count())
 * to desc[0..6].  pifft_plan_dry_run_instances plans as pifft_plan_dry_run does
 * and writes, for each launch i < min(launches, max_ids), the instance index of
 * its k_pass kernel (-1 for tree and interleave launches); it returns the
 * number of launches, or -1.  pifft_instance_found(i) is 1 once the planner
 * has found instance i in this process (it probes instances to choose between
 * plans, so a plan depends on every instance it found, launched or not), 0 if
 * not, -1 for an index out of range.  tests/test_instances.py checks with
 * them that every compiled instance is one some plan depends on. */
int pifft_instance_count(void);
int pifft_instance_desc(int i, int32_t* desc);
int pifft_instance_found(int i);
int pifft_plan_dry_run_instances(uint64_t n, uint32_t workers, uint32_t first, uint32_t count, uint32_t batch,
                                 int prec, int flags, int32_t* ids, int max_ids);

/* The kernel function of launch `launch` (< info.num_launches), demangled as
 * profilers print it (e.g. "void pifft::k_pass<double, 512, 16, 2, 1, 0, 16>
 * (pifft::PassArgs)"), into buf (len bytes, truncated, NUL-terminated): maps a
 * plan's launches onto rocprofv3 --stats rows. */
int pifft_plan_kernel_name(const pifft_plan* plan, int launch, char* buf, size_t len);

/* Device boundary: d_in holds info.in_elems complex values, d_out receives
 * info.out_elems (d_in != d_out; neither is freed).  Asynchronous on `stream`
 * (a hipStream_t; NULL = the default stream, as in other ROCm libraries).
 * A plan owns its workspace (ping-pong and tree buffers): it must not execute
 * concurrently with itself -- two executions of one plan on different streams
 * race on that workspace.  Use one plan per stream (the reference gives each
 * worker its own scratch, CPU.c:396-404). */
int pifft_execute_device(pifft_plan* plan, const void* d_in, void* d_out, void* stream);

/* As pifft_execute_device, but times every launch, waits, and returns each
 * launch's duration in launch_ms[0 .. min(info.num_launches, max_launches)).
 * The events are bound to the kernels' own dispatches (hipExtLaunchKernel
 * start/stop events: the kernel's start and end timestamps, what rocprofv3
 * reports), so timing adds no marker packets between launches. */
int pifft_execute_device_timed(pifft_plan* plan, const void* d_in, void* d_out, void* stream,
                               float* launch_ms, int max_launches);

/* Workspace placement tuning (optional, like a measuring planner): the plan's
 * ping-pong workspace W and the caller's d_out are read and written at the
 * same row offsets by the later passes, and whether their physical pages
 * collide in the DRAM banks depends on where each allocation lands (C4 passes
 * 2 + 3: 2.92 ms in the fast state, 3.13-3.5 ms in the slow one; DESIGN.md
 * section 4).  This call times the plan on (d_in, d_out) with its current W,
 * then with up to tries - 1 freshly allocated ones, and keeps the fastest (one
 * extra W at a time, every loser kept until the call returns; stops early
 * when the device would keep less than another W and 4 GiB free).  *best_ms (may be
 * NULL) receives the kept workspace's mean execution time.  Synchronous.
 * Results are unchanged; only timings move. */
int pifft_plan_tune_workspace(pifft_plan* plan, const void* d_in, void* d_out, void* stream, int tries,
                              float* best_ms);

/* Asynchronous per-launch timing.  After pifft_profile_start(plan, steps,
 * mode) the next `steps` pifft_execute_device calls bind start/stop events to
 * launches (hipExtLaunchKernel: the dispatch's own timestamps, as rocprofv3
 * reports them; no host sync):
 *   PIFFT_PROFILE_ALL     every launch of every execution.  A timed dispatch
 *                         delays the next one by ~9 us, so the launches run
 *                         isolated -- 1-6 % faster than back to back;
 *   PIFFT_PROFILE_SAMPLED in-context: execution k times launch (k/2) mod L
 *                         when k is odd and nothing when k is even, so every
 *                         timed dispatch follows untimed ones, back to back
 *                         as in an unprofiled run (what bench.py's roofline
 *                         uses; steps = 2 L s gives s samples per launch).
 * pifft_profile_read waits for the recorded executions, writes each launch's
 * summed duration (ms) and sample count to launch_ms_sum / launch_samples
 * (either may be NULL; the first min(num_launches, max_launches) launches),
 * stops profiling (also when it fails) and returns the number of executions
 * recorded (or -1).  The profiled executions' own step time is NOT clean. */
#define PIFFT_PROFILE_ALL 0
#define PIFFT_PROFILE_SAMPLED 1
int pifft_profile_start(pifft_plan* plan, int steps, int mode);
int pifft_profile_read(pifft_plan* plan, float* launch_ms_sum, int* launch_samples, int max_launches);

/* A clean loop of some of the plan's launches alone (profiling): after two
 * untimed rounds, `reps` rounds of launches[0 .. nlaunches) back to back
 * between two marker events, then one full execution, so d_out again holds
 * the plan's result.  *mean_ms = the loop's time / (reps * nlaunches): a
 * launch's duration back to back with itself plus its share of the dispatch
 * gaps -- the timed loop's context without bound events, each of which lets
 * the GPU idle ~9 us after its dispatch (a 10-us kernel sampled that way
 * reads 5-8 % faster than back to back; round-4 trace).  Synchronous. */
int pifft_launch_loop(pifft_plan* plan, const int* launches, int nlaunches, int reps, const void* d_in,
                      void* d_out, void* stream, float* mean_ms);

/* Host boundary, the reference's run() shape: copies host_in (batch*N values)
 * to the device (untimed), runs, and if host_out != NULL writes this plan's
 * bins at their natural-order positions of host_out (batch*N values; other
 * positions untouched -- the reference's workers write disjoint `out` entries,
 * CPU.c:496-499).  A PIFFT_OUT_BITREV plan instead writes its workers'
 * scratch segments at host_out[b N + q M + i] (the reference's tmp_in
 * layout, q = first..first+count-1).  ms_stage1 / ms_stage2 receive the
 * device wall time of the tree stage and of the rest, from a marker event
 * before each stage's first launch to one after its last (the reference's
 * two stage timers, CPU.c:414-481: gaps between launches count).  When a plan evaluates its tree inside the first local-FFT
 * pass (one worker per plan, log2 P <= 4, a multi-pass local FFT; see
 * pifft_plan_info.launch_kind 4) that fused launch cannot be split: stage 1 is
 * then the tree PLUS the first pass, and stage 2 the remaining passes
 * (PIFFT_SEPARATE_TREE keeps the tree its own launch). */
int pifft_execute(pifft_plan* plan, const void* host_in, void* host_out, double* ms_stage1,
                  double* ms_stage2);

/* Several plans (normally one per GPU) run concurrently from one host thread:
 * the P-GPU no-communication split.  Stage times are the max over plans.
 * When the plans hold all P workers between them (PIFFT_OUT_SLICES), host_out
 * is filled through pifft_allgather onto the first plan's device (into a
 * batch*N buffer allocated for the call and freed before it returns) and one
 * device-to-host copy; otherwise a plan whose output is natural order or the
 * reference's scratch order (PIFFT_OUT_BITREV) is copied straight into
 * host_out, and a plan holding only some workers has its bins scattered on
 * the host. */
int pifft_execute_group(pifft_plan** plans, int nplans, const void* host_in, void* host_out,
                        double* ms_stage1, double* ms_stage2);

/* Kernel-only stage times: re-runs the plans of the last pifft_execute_group
 * call on their staged input (no host copies) with events bound to every
 * launch, and returns the summed kernel durations of the tree stage and of
 * the rest for the slowest plan -- pifft_execute_group's wall stage times
 * minus the gaps between launches (CLI -x extra columns). */
int pifft_execute_group_kernel_times(pifft_plan** plans, int nplans, double* kernel_ms_stage1,
                                     double* kernel_ms_stage2);

/* The optional final exchange of a multi-GPU job (the
 * reference's counterpart is every worker writing its bins into the shared
 * natural-order `out`, CPU.c:496-499).  plans[i] holds workers
 * [first_i, first_i + count_i) with its slice-major result at d_slices[i] (on
 * plan i's device, PIFFT_OUT_SLICES layout, e.g. the d_out of its
 * pifft_execute_device); between them the plans must cover all P workers
 * exactly once.  For every j with d_natural[j] != NULL, each plan's slices are
 * copied to plan j's device (hipMemcpyPeerAsync over xGMI, one copy stream per
 * source; a device-local copy when both share a device) and interleaved there
 * into natural order: d_natural[j] receives batch*N values.  Call it once the
 * executions that produced d_slices have completed.  No d_natural[j] may
 * overlap any d_slices[i] or another destination (the call fails with -1
 * otherwise: destinations are written while other copies still read the
 * sources).  Synchronous; ms (may be
 * NULL) receives the slowest destination's copy + interleave time.  Uses a
 * plan-owned batch*N gather buffer on each destination device. */
int pifft_allgather(pifft_plan* const* plans, int nplans, const void* const* d_slices, void* const* d_natural,
                    double* ms);

/* Synthetic input on the device: element e (count of them, starting at global
 * element index `first`) = splitmix64(seed) draws 2e, 2e+1 mapped to
 * (2u-1)/sqrt(n) -- bit-identical to the host generator of the test oracle. */
int pifft_generate_device(void* d_x, uint64_t count, uint64_t n, uint64_t seed, uint64_t first,
                          int prec, void* stream);

/* Slice-major -> natural order: out[bitrev_{log2 P}(q) + P k] = slices[q M + k]
 * for all P workers (M = n/P), `batch` transforms (used after an all-gather). */
int pifft_interleave_device(const void* d_slices, void* d_out, uint64_t n, uint32_t workers,
                            uint32_t batch, int prec, void* stream);

/* Tree ("funnel") stage only, for parity checks: writes worker q's N/P segment
 * after the log2 P half-butterfly stages (the reference's tmp_in segment after
 * CPU.c:419-448) for the plan's workers, slice-major. */
int pifft_tree_device(pifft_plan* plan, const void* d_in, void* d_seg, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* PIFFT_H */
