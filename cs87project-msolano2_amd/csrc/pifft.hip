// cs87project-msolano2_amd/csrc/pifft.hip -- libpifft.so: planner + C-ABI shim.
//
// Implements include/pifft.h.  The host side plans the reference's two stages
// (CPU.c:419-448 tree, CPU.c:463-478 cylinder) as a short list of kernel
// launches (pifft_kernels.h) over device buffers:
//
//   tree    : input (batch x N, HBM-resident)  -> Z (batch x count x N/P)
//   passes  : Z -> ... -> Z'   Stockham passes of the N/P-point local FFT,
//             each an LDS-resident R-point sub-FFT over C adjacent lines
//   [interleave: slice-major -> natural order, whole transform on one GPU]
//
// Buffers ping-pong between the caller's output and one plan-owned workspace.
// Twiddles are host-built tables in HBM (w_R per pass, two-level w_M and w_N;
// the tree uses the reference's own omega(N,k) formula up to N = 2^22 so that
// its output is bit-identical to the reference's post-tree segment).
#ifndef _GNU_SOURCE
#define _GNU_SOURCE  // sincos (reference_omega_levels)
#endif
#include "pifft_gather.h"
#include "pifft_kernels.h"
#include "pifft_table.h"
#include "../../include/pifft.h"

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cxxabi.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

using namespace pifft;

namespace {

thread_local std::string g_err;

int fail(const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return -1;
}

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) return fail("%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// Planner tuning variables (PIFFT_* below) are read only when PIFFT_TUNING=1
// is set: a variable inherited from a shell never changes the product's plan
// (tests/test_planner.py::test_stray_tuning_variables_are_ignored).  Each
// default is the measured winner cited where it is read.
bool tuning_on() {
    const char* s = getenv("PIFFT_TUNING");
    return s && s[0] == '1' && s[1] == 0;
}
int env_int(const char* name, int dflt) {
    if (!tuning_on()) return dflt;
    const char* s = getenv(name);
    return (s && *s) ? atoi(s) : dflt;
}

// Test-only fault injection for the multi-GPU error paths, which a one-GPU
// box cannot otherwise reach (tests/test_gpu_parity.py): PIFFT_FAULT=<site>
// (enable_peer, peer_copy, broadcast), read only under PIFFT_TUNING=1, makes
// that call fail as a HIP error would.
bool fault_at(const char* site) {
    if (!tuning_on()) return false;
    const char* s = getenv("PIFFT_FAULT");
    const size_t n = strlen(site);
    if (!s || strncmp(s, site, n)) return false;
    if (s[n] == '\0') return true;  // <site>: every time it is reached
    if (s[n] != ':') return false;
    // <site>:K -- only the K-th time it is reached under this setting (e.g.
    // peer_copy:3 fails the third copy, after two were enqueued)
    static std::mutex mu;
    static std::string last;
    static long count = 0;
    std::lock_guard<std::mutex> lk(mu);
    if (last != s) {
        last = s;
        count = 0;
    }
    return ++count == atol(s + n + 1);
}

// Timing events only time (pifft_execute_device_timed, pifft_profile_*,
// pifft_execute_group's stage timers): no system-scope fence when they are
// recorded, so a timed kernel does not pay an L2 write-back at its end (a
// bound stop event otherwise made C3's 44-us kernel read 50 us)
constexpr unsigned kTimingEventFlags = hipEventDisableSystemFence;

bool is_pow2(uint64_t x) { return x && !(x & (x - 1)); }

// 1-D grid for a grid-stride kernel of `total` items at 256 threads/block:
// capped so the launch's work-item count stays far below 2^32
unsigned stride_grid(uint64_t total) {
    const uint64_t blocks = (total + 255) / 256;
    return (unsigned)(blocks < 262144 ? (blocks ? blocks : 1) : 262144);
}
int ilog2u(uint64_t x) {
    int l = 0;
    while (x > 1) { x >>= 1; l++; }
    return l;
}
uint32_t bitrev(uint32_t x, int m) { return m ? (__builtin_bitreverse32(x) >> (32 - m)) : 0u; }

// ---------------------------------------------------------------------------
// pass kernel instantiations (tables from the pifft_passes.hip parts)
// ---------------------------------------------------------------------------
}  // namespace
#define PIFFT_DECL_PART(k) extern "C" const PassKernel* pifft_pass_table_##k(int* n);
PIFFT_DECL_PART(0)
PIFFT_DECL_PART(1)
PIFFT_DECL_PART(2)
PIFFT_DECL_PART(3)
PIFFT_DECL_PART(4)
PIFFT_DECL_PART(5)
PIFFT_DECL_PART(6)
PIFFT_DECL_PART(7)
namespace {
static_assert(PIFFT_NPART == 8, "update the part list");

const std::vector<PassKernel>& pass_kernels() {
    static const std::vector<PassKernel> all = [] {
        std::vector<PassKernel> v;
        const PassKernel* (*parts[])(int*) = {pifft_pass_table_0, pifft_pass_table_1, pifft_pass_table_2,
                                               pifft_pass_table_3, pifft_pass_table_4, pifft_pass_table_5,
                                               pifft_pass_table_6, pifft_pass_table_7};
        for (auto f : parts) {
            int n = 0;
            const PassKernel* t = f(&n);
            v.insert(v.end(), t, t + n);
        }
        return v;
    }();
    return all;
}

// every instance find_pass has returned in this process (pifft_instance_found):
// the planner probes instances to choose between plans, so the instances a
// plan depends on are those it found, launched or not (tests/test_instances.py)
std::atomic<unsigned char>* found_log() {
    static std::atomic<unsigned char>* f = new std::atomic<unsigned char>[pass_kernels().size()]();
    return f;
}

const PassKernel* find_pass(int prec, int R, int C, int mode, int nts = 0, int lp = 0, int vpt = 16) {
    const auto& all = pass_kernels();
    for (size_t i = 0; i < all.size(); i++) {
        const PassKernel& k = all[i];
        if (k.prec == prec && k.R == R && k.C == C && k.mode == mode && k.nts == nts && k.lp == lp && k.vpt == vpt) {
            found_log()[i].store(1, std::memory_order_relaxed);  // (plans may be built on several host threads)
            return &k;
        }
    }
    return nullptr;
}

// ---------------------------------------------------------------------------
// plan
// ---------------------------------------------------------------------------
enum { STEP_TREE = 1, STEP_PASS = 2, STEP_INTERLEAVE = 3, STEP_TREE_PASS = 4 };
enum { BUF_IN = 0, BUF_OUT = 1, BUF_W = 2, BUF_TA = 3, NBUF = 4 };

struct Step {
    int kind = 0;
    const void* fn = nullptr;
    const PassKernel* pk = nullptr;  // STEP_PASS / STEP_TREE_PASS: the instance
    dim3 grid, block;
    size_t lds = 0;
    int src = -1, dst = -2;  // -1 / -2: the chain element's input / output buffer
    uint64_t src_off = 0, dst_off = 0;  // elements
    PassArgs pa{};
    int nts = 0;  // STEP_PASS / STEP_TREE_PASS: the instance's streaming form
    TreeArgs ta{};
    uint64_t il_total = 0;
    uint32_t il_log_n = 0, il_log_p = 0;
    uint64_t bytes = 0;
};

}  // namespace

struct pifft_plan {
    uint64_t n = 0, m = 0;
    uint32_t P = 1, q0 = 0, nq = 1, batch = 1;
    int prec = 64, device = 0, flags = 0;
    int lp = 0, log_n = 0, log_m = 0;
    size_t esz = 16;
    bool natural = true;
    bool bitrev = false;  // PIFFT_OUT_BITREV
    bool ilv = false;     // the last pass stores natural order itself (PassArgs::ilv_log)
    bool wil = false;     // worker-interleaved layout (PassArgs::wil, MODE | 8 passes)
    bool separate_tree = false;  // PIFFT_SEPARATE_TREE: never fuse the tree into a pass
    std::vector<Step> steps;
    int tree_steps = 0, npasses = 0;
    bool fused_tree = false;  // tree evaluated inside the first pass (STEP_TREE_PASS)
    std::vector<Step> tree_only;  // the tree stage alone, for pifft_tree_device
    std::vector<hipEvent_t> prof_ev;  // pifft_profile_*: per recorded execution, a start and a stop per timed launch
#ifdef PIFFT_WG_CLOCK
    unsigned long long* dbg_clk = nullptr;  // pifft_debug_wg_clock: the clocked launch's words (diagnostics build)
#endif
    int prof_steps = 0, prof_used = 0, prof_mode = 0;
    int radix[8] = {0}, lines[8] = {0}, vpt[8] = {0};
    void* buf[NBUF] = {nullptr};
    size_t bytes_w = 0, bytes_ta = 0;
    void* d_tw = nullptr;
    size_t tw_bytes = 0;
    hipStream_t stream = nullptr;
    std::vector<hipEvent_t> ev;  // 2 per launch: its start and stop (launch_steps)
    hipEvent_t sev[3] = {nullptr, nullptr, nullptr};  // stage markers: start, end of stage 1, end of stage 2
    void* d_hin = nullptr;   // pifft_execute's staging copies
    void* d_hout = nullptr;
    void* d_gather = nullptr;  // pifft_allgather: every worker's slices on this plan's device
    std::vector<char> host_tmp;
    std::vector<int> peer_on;  // devices this plan's device has peer access to (pifft_allgather)
    std::vector<hipStream_t> gst;  // pifft_allgather: one copy stream per source plan
    std::vector<hipEvent_t> gdone;  // ... and its completion event
    hipEvent_t gev[2] = {nullptr, nullptr};  // gather start / end on `stream`
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (dev < 0) return;  // dry-run plans touch no device
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// Host twiddle tables, appended to one blob (offsets 256-B aligned).
struct TableBuilder {
    std::vector<char> blob;
    size_t esz;
    bool size_only = false;  // a dry run: the blob's layout and size only (no memory, no values)
    size_t sized = 0;        // the blob's size in a size_only run
    explicit TableBuilder(size_t e) : esz(e) {}
    size_t size() const { return size_only ? sized : blob.size(); }
    void grow_to(size_t bytes) {
        if (size_only) sized = bytes;
        else blob.resize(bytes);
    }
    size_t align() {
        size_t off = (size() + 255) & ~(size_t)255;
        grow_to(off);
        return off;
    }
    void put(double re, double im) {
        size_t o = blob.size();
        blob.resize(o + esz);
        if (esz == 16) {
            double v[2] = {re, im};
            memcpy(&blob[o], v, 16);
        } else {
            float v[2] = {(float)re, (float)im};
            memcpy(&blob[o], v, 8);
        }
    }
    // w_L^(e*stride), e < count, accurate (long double) -- the Stockham tables
    size_t roots(uint64_t L, uint64_t count, uint64_t stride) {
        size_t off = align();
        if (size_only) {
            grow_to(off + count * esz);
            return off;
        }
        const long double two_pi = 6.283185307179586476925286766559005768L;
        for (uint64_t e = 0; e < count; e++) {
            const uint64_t x = (e * stride) % L;
            const long double ang = two_pi * ((long double)x / (long double)L);
            put((double)cosl(ang), (double)(-sinl(ang)));
        }
        return off;
    }
    // omega(N,k) with the reference's own formula (CPU.c:644-651), packed by
    // tree level (TreeTw::direct): level t < levels holds omega(N, k 2^t),
    // k < N >> (t+1), at N - (N >> t) + k (level 0 = every k < N/2)
    size_t reference_omega_levels(uint64_t N, int levels) {
        size_t off = align();
        if (size_only) {
            grow_to(off + (N - (N >> (levels > 0 ? levels : 1))) * esz);
            return off;
        }
        // gcc -O1 and up folds the reference's cos()/sin() pair into one glibc
        // sincos() call; glibc's sincos and its separate cos/sin disagree in
        // the last fp64 bit for ~1e-3 of the angles (43 of 2^15 at N=2^16).
        // The reference build the fixtures pin (-O2) is the sincos one, so the
        // table is built the same way (clang keeps the pair separate).
        for (uint64_t k = 0; k < N / 2; k++) {
            double s, c;
            sincos(2.0 * M_PI / (double)N * (double)k, &s, &c);
            put(c, -s);
        }
        // the higher levels: byte copies of level-0 entries k 2^t
        blob.resize(off + (N - (N >> (levels > 0 ? levels : 1))) * esz);
        for (int t = 1; t < levels; t++) {
            const uint64_t base = N - (N >> t);
            for (uint64_t k = 0; k < (N >> (t + 1)); k++)
                memcpy(&blob[off + (base + k) * esz], &blob[off + (k << t) * esz], esz);
        }
        return off;
    }
};

struct TwoLevel {
    size_t lo = 0, hi = 0;
    uint32_t h = 0;
};

TwoLevel two_level(TableBuilder& tb, uint64_t L) {
    TwoLevel t;
    const int logl = ilog2u(L);
    t.h = (uint32_t)((logl + 1) / 2);
    t.lo = tb.roots(L, 1ull << t.h, 1);
    t.hi = tb.roots(L, (L >> t.h) ? (L >> t.h) : 1, 1ull << t.h);
    return t;
}

// slice-major -> natural order: k_interleave_tile (LDS tile of all P slices,
// P <= 2048) from P = 2^5 at fp64 and P = 2 at fp32, else k_interleave (one
// thread per output element, any P); profiles/r02_interleave_ab.log
bool interleave_tiled(int prec, int lp, uint64_t n) {
    const int lo = env_int(prec == 64 ? "PIFFT_INTERLEAVE_TILE_MIN64" : "PIFFT_INTERLEAVE_TILE_MIN32", prec == 64 ? 5 : 1);
    return lo > 0 && lp >= lo && lp <= 11 && n >= (uint64_t)IL_TILE;
}
const void* interleave_fn(int prec, int lp, uint64_t n) {
    if (interleave_tiled(prec, lp, n))
        return prec == 64 ? (const void*)&k_interleave_tile<double> : (const void*)&k_interleave_tile<float>;
    return prec == 64 ? (const void*)&k_interleave<double> : (const void*)&k_interleave<float>;
}
uint64_t interleave_threads(uint64_t total, int lp, int prec, uint64_t n) {
    return interleave_tiled(prec, lp, n) ? (total / IL_TILE) * 256 : total;
}

struct PassChoice {
    int R, C, mode, nts;
    int vpt = 16;
};

// Tile = R x C elements per workgroup (C adjacent lines of an R-point sub-FFT).
// Default tile 8192 (fp64) / 16384 (fp32): 128 KiB of data in registers, one
// component (64 KiB) in LDS at a time -> two workgroups per CU; at R = 512 the
// lines give 256-B contiguous row segments (the HBM-efficient width measured
// by tools/probe_bw.hip).
int tile_elems(int prec) {
    return env_int(prec == 64 ? "PIFFT_TILE64" : "PIFFT_TILE32", 8192);
}

int pick_lines(int prec, int R, uint64_t ntrans_lines_cap, uint64_t total_lines, const char* env_c, int mode,
               int strided_tile = 0) {
    int C = env_int(env_c, 0);
    // single pass: lines are whole contiguous transforms, no segment-width
    // constraint -> small tiles (measured best: C = 4096/R, i.e. C=1 at 4096)
    int tile = mode == 0   ? env_int(prec == 64 ? "PIFFT_SINGLE_TILE64" : "PIFFT_SINGLE_TILE32", 4096)
               : mode == 1 ? env_int(prec == 64 ? "PIFFT_FIRST_TILE64" : "PIFFT_FIRST_TILE32", tile_elems(prec))
                           : tile_elems(prec);
    if (strided_tile && (mode == 1 || mode == 2)) tile = strided_tile;  // (the packed VPT-32 fp32 tile)
    // fp64 strided passes of R <= 256, not the fused tree pass (mode 3): a
    // 4096-value tile.  At 8192 (R = 256, C = 32, 512 threads) the kernel
    // spills 20 B/lane at its 128-VGPR budget; at C = 16 it runs 256 threads
    // at 138 VGPRs, 3 workgroups per CU.  Measured on MI355X
    // (profiles/r02_smallr_tile.log): 2^22 -7 %, 2^23 -12 %, 2^24 -4 %, the
    // 2^28 worker of 8 -1.5 %; the fused pass itself loses at C = 16 (156
    // VGPRs), so it keeps the 8192 tile
    if (prec == 64 && (mode == 1 || mode == 2) && R <= 256) tile = env_int("PIFFT_SMALLR_TILE64", 4096);
    if (mode == 3) mode = 1;  // the fused first pass: the first-pass tile, mode-1 line rules
    if (C <= 0) C = tile / R;
    if (C < 1) C = 1;
    if (C > 64) C = 64;
    if (R <= 8) C = 64;
    while (C > 1 && (uint64_t)C > ntrans_lines_cap && R > 8) C /= 2;
    // fill the chip: at least ~2 workgroups per CU (small transforms)
    const uint64_t min_wg = (uint64_t)env_int("PIFFT_MIN_WORKGROUPS", 512);
    // strided passes are instantiated for C >= 4 (and fp64 C = 2 at R = 512-2048, PIFFT_STRIDED_CMIN=2)
    const int cmin = mode == 0 ? 1 : env_int("PIFFT_STRIDED_CMIN", 4);
    while (C > cmin && R > 8 && total_lines / (uint64_t)C < min_wg) C /= 2;
    while (C > cmin && !find_pass(prec, R, C, mode)) C /= 2;
    return C;
}

// non-temporal streaming when a pass moves more than the Infinity Cache holds,
// and for 16-64 MiB passes (measured on MI355X, profiles/r02_nt_sweep.log:
// fp64 2^20 P=1 26 -> 24 us, P=8 44 -> 41 us, fp32 4096 x 1024 16 -> 13 us,
// the 2^21-point worker of 8 95 -> 84 us; but 8-16 MiB and 128-256 MiB passes
// lose 5-40 %)
int pick_nts(uint64_t pass_bytes) {
    const int force = env_int("PIFFT_NT", -1);
    if (force >= 0) return force ? 1 : 0;
    return (pass_bytes > (256ull << 20) || (pass_bytes > (16ull << 20) && pass_bytes <= (64ull << 20))) ? 1 : 0;
}

// HBM rate of a pass side, by the contiguous bytes per row segment (TB/s).
// Measured on MI355X with tools/probe_bw.hip (strided tile copies) and the
// pass kernels themselves (profiles/r01_tune_*.log); contiguous ~5.6.
double seg_rate(double seg_bytes) {
    if (seg_bytes >= 1024) return 5.6;
    if (seg_bytes >= 512) return 5.5;
    if (seg_bytes >= 256) return 5.3;
    if (seg_bytes >= 128) return 4.2;
    if (seg_bytes >= 64) return 2.6;
    return 1.5;
}

// Whole-pass HBM rate (TB/s, both sides) by the pass's position in a plan and
// its strided row-segment width, for HBM-bound plans without a fused tree
// (round 3).  Measured on MI355X (profiles/r03_fp64_radix_order.log,
// r03_fp32_radix_order.log; fp64 2^28 / 2^29, fp32 packed 2^28): a 256-B pass
// runs 5.9 / 5.6 / 5.25 TB/s first / in the middle / last, a 128-B one 5.0 /
// 4.8 / 4.8 -- the last pass's strided stores into the caller's unpadded
// output are slow at either width, so the narrow pass costs least there.
// fp64 2^28: 512-512-1024 4.72 ms vs 1024-512-512 4.82 (same box); fp32 2^28
// 2.47 vs 2.60 ms; fp64 2^29 9.41 vs 9.65 ms.  Same for both precisions.
double pass_rate(double seg_bytes, bool first, bool last) {
    if (seg_bytes >= 256) return first ? 5.9 : last ? 5.25 : 5.6;
    if (seg_bytes >= 128) return first ? 5.0 : 4.8;
    return seg_rate(seg_bytes);
}

// Local FFT of length M as passes.  A single LDS/register-resident pass when M
// fits (M <= 2^14); otherwise k Stockham passes with balanced radices, k and
// the radix order chosen by a bandwidth model: each pass moves its bytes at
// the rate of its narrowest strided side (C*esz-byte row segments).
// heavy_first: the first pass also evaluates the tree (reads P leaves per
// input, P = 2^lp), so its read side dominates.
// fp32 strided passes at 32 values per thread, packed (k_pass VPT 32): a
// 16384-value tile on 512 threads, two workgroups per CU -- the bytes and
// row-segment widths of the fp64 8192-value tile, so fp32 2^28 runs in three
// passes (1024-512-512 at C = 16/32/32) instead of four 128-point ones.
// Measured on MI355X (profiles/r03_fp32_packed_vpt32.log): fp32 2^28 3.36 ->
// 2.67 ms, 2^30 13.7 -> 11.6 ms; 2^26 (512 MiB per side) 0.63 -> 0.65 ms.
// The rule: data beyond 1 GiB per side, no fused tree pass (no packed MODE 3
// instances).  PIFFT_VPT32: -1 this rule, 0 never, 1 whenever instantiated.
bool use_vpt32(int prec, uint64_t M, uint64_t ntrans, int heavy_lp) {
    const int force = env_int("PIFFT_VPT32", -1);
    if (prec != 32 || heavy_lp || force == 0) return false;
    return force == 1 || ntrans * M * 8 >= (1ull << 30);
}

// pos_ok: the position-aware pass rates may price this plan (not for the
// worker-interleaved layout, whose passes move rows of all workers: there the
// narrow pass last measured 1-14 % slower, profiles/r03_pos_model_shapes.log)
// single_max: the longest one-pass local FFT (log2; default 14, PIFFT_SINGLE_MAX_LOG)
int plan_passes(uint64_t M, int prec, uint64_t ntrans, std::vector<PassChoice>& out, int heavy_lp = 0,
                bool allow_v32 = true, bool pos_ok = true, int single_max = -1) {
    out.clear();
    if (M <= 1) return 0;
    const int logm = ilog2u(M);
    const size_t esz = prec == 64 ? 16 : 8;
    if (single_max < 0) single_max = env_int("PIFFT_SINGLE_MAX_LOG", 14);
    const bool v32 = allow_v32 && M > (1ull << single_max) && use_vpt32(prec, M, ntrans, heavy_lp);
    const int stile = v32 ? 16384 : 0;
    const int nts = pick_nts(2 * ntrans * M * esz);
    if (logm <= single_max) {
        const int R = (int)M;
        const int C = pick_lines(prec, R, ntrans, ntrans, prec == 64 ? "PIFFT_SINGLE_C64" : "PIFFT_SINGLE_C32", 0);
        if (!find_pass(prec, R, C, 0, nts)) return fail("no pass kernel for R=%d C=%d", R, C);
        // tuning: 8 values per thread (radix-8 stages, twice the waves per
        // sub-FFT) -- measured slower than 16 at every batch size
        // (profiles/r02_vpt_sweep.log), so only on request and if instantiated
        const int vpt = env_int("PIFFT_SINGLE_VPT", 16);
        if (vpt != 16 && find_pass(prec, R, C, 0, nts, 0, vpt)) {
            out.push_back({R, C, 0, nts, vpt});
            return 0;
        }
        out.push_back({R, C, 0, nts});
        return 0;
    }
    // tuning: explicit log2 radices, e.g. PIFFT_RADIX_LOGS=10,10,8 (must sum to log2 M)
    bool explicit_radices = false;
    if (const char* rl = tuning_on() ? getenv("PIFFT_RADIX_LOGS") : nullptr) {
        std::vector<int> logs;
        for (const char* c = rl; *c;) {
            char* end = nullptr;
            const long v = strtol(c, &end, 10);
            if (end == c) break;
            logs.push_back((int)v);
            c = *end ? end + 1 : end;
        }
        int sum = 0;
        for (int l : logs) sum += l;
        if (sum == logm && logs.size() > 1) {
            for (size_t p = 0; p < logs.size(); p++) {
                const int R = 1 << logs[p], mode = p == 0 ? 1 : 2;
                const int C = pick_lines(prec, R, M >> logs[p], ntrans * (M >> logs[p]),
                                         prec == 64 ? "PIFFT_COL_C64" : "PIFFT_COL_C32",
                                         (p == 0 && heavy_lp) ? 3 : mode, stile);
                if (!find_pass(prec, R, C, mode, nts)) return fail("no pass kernel R=%d C=%d", R, C);
                out.push_back({R, C, mode, nts});
            }
            explicit_radices = true;
        }
    }
    const int rmax_log = env_int(prec == 64 ? "PIFFT_COL_RMAX_LOG64" : "PIFFT_COL_RMAX_LOG32", 10);
    const int kmin = (logm + rmax_log - 1) / rmax_log;
    const int kmax = env_int("PIFFT_PASSES", 0) > 0 ? env_int("PIFFT_PASSES", 0) : kmin + 1;
    double best = 1e300;
    // data that stays in the 256 MiB Infinity Cache is not bound by HBM row
    // segments: fewest passes there
    const bool resident = 2 * ntrans * M * esz <= (256ull << 20);
    const int klast = resident && env_int("PIFFT_PASSES", 0) <= 0 ? kmin : kmax;
    for (int k = env_int("PIFFT_PASSES", 0) > 0 ? kmax : kmin; k <= klast && !explicit_radices; k++) {
        if (logm < 4 * k) break;  // every radix >= 16
        const int base = logm / k, extra = logm % k;
        const int force_order = env_int("PIFFT_ORDER", -1);  // tuning: 0 or 1 only
        for (int order = 0; order < 2; order++) {  // 0: larger radices first, 1: smaller first
            if (force_order >= 0 && order != force_order) continue;
            // a fused tree+first pass runs best with the larger radix (R = 512,
            // C = 16) first: measured 1-3 % over the model's pick at P = 4, 8.
            // Not when that radix leaves the P-fold leaf reads narrower than
            // 256-B segments (R = 1024, C = 8 at fp64): then the model picks
            // between both orders (config 5, 2^29 per worker: 512-1024-1024
            // 19.7 ms vs 256-128-128-128 21.3 ms, profiles/r01_tune_c5.log).
            // fp64 only: the fp32 tile gives R = 1024 128-B segments too, but
            // the other order there loses the fused kernel (no instance)
            if (force_order < 0 && heavy_lp > 0 && order == 1) {
                const int R0 = 1 << (base + (extra > 0 ? 1 : 0));
                const int C0 = pick_lines(prec, R0, M >> ilog2u((uint64_t)R0), ntrans * (M >> ilog2u((uint64_t)R0)),
                                          prec == 64 ? "PIFFT_COL_C64" : "PIFFT_COL_C32", 3);
                if (prec != 64 || (size_t)C0 * esz >= 256) continue;  // fp32: measured cases only
            }
            std::vector<PassChoice> cand;
            double cost = 0.0;
            bool ok = true;
            // the position rates were measured on passes of >= 128-B segments:
            // a candidate with a narrower pass keeps the segment-width model
            bool pos = pos_ok && !resident && !heavy_lp && env_int("PIFFT_POS_MODEL", 1);
            for (int p = 0; p < k && pos; p++) {
                const int bits = order ? base + (p >= k - extra ? 1 : 0) : base + (p < extra ? 1 : 0);
                const int C = pick_lines(prec, 1 << bits, M >> bits, ntrans * (M >> bits),
                                         prec == 64 ? "PIFFT_COL_C64" : "PIFFT_COL_C32", p == 0 ? 1 : 2, stile);
                pos = (size_t)C * esz >= 128;
            }
            for (int p = 0; p < k && ok; p++) {
                const int bits = order ? base + (p >= k - extra ? 1 : 0) : base + (p < extra ? 1 : 0);
                const int R = 1 << bits;
                const int mode = p == 0 ? 1 : 2;
                const int C = pick_lines(prec, R, M >> bits, ntrans * (M >> bits),
                                         prec == 64 ? "PIFFT_COL_C64" : "PIFFT_COL_C32",
                                         (p == 0 && heavy_lp) ? 3 : mode, stile);
                if (!find_pass(prec, R, C, mode, nts)) { ok = false; break; }
                const double rs = seg_rate((double)C * esz);           // strided side
                const double side = (double)ntrans * M * esz * 1e-12;  // TB per side
                const double reads = (p == 0 && heavy_lp) ? side * (1 << heavy_lp) : side;
                if (pos)
                    cost += 2 * side / pass_rate((double)C * esz, p == 0, p == k - 1);
                else
                    cost += reads / rs + side / (mode == 1 ? 5.6 : rs);
                cand.push_back({R, C, mode, nts});
            }
            if (ok && cost < best) {
                best = cost;
                out = cand;
            }
        }
    }
    if (out.empty()) return fail("no pass decomposition for M=2^%d", logm);
    // the packed VPT-32 passes for the 16384-value tile (every strided pass
    // must have its instance, else the plan is redone at the 8192 tile)
    if (v32) {
        for (auto& pc : out) {
            if (pc.mode != 1 && pc.mode != 2) continue;
            if (!find_pass(prec, pc.R, pc.C, pc.mode, pc.nts, 0, 32))
                return plan_passes(M, prec, ntrans, out, heavy_lp, false, pos_ok);
            pc.vpt = 32;
        }
    }
    // The fused tree pass of a small one-worker slice at 8 values per thread
    // (radix-8 stages, twice the waves per workgroup) when it has R <= 512
    // points and at most 128 workgroups: a latency-bound launch on a fraction
    // of the CUs, whose P leaf loads and tree per value then spread over twice
    // the threads.  Measured on MI355X (profiles/r04d_fused_vpt8.log): fp64
    // local 2^15-2^18 +4.5-31 % (config 2's slice 14.05 -> 12.66 us), fp32
    // +0.6-4 %; R = 1024 -2-3 %, 256 workgroups ties.  PIFFT_FUSED_VPT: the
    // values per thread instead (tuning).
    if (heavy_lp && !out.empty() && out[0].mode == 1) {
        PassChoice& pc = out[0];
        const uint64_t wgs = (ntrans * (M / (uint64_t)pc.R) + pc.C - 1) / (uint64_t)pc.C;
        const int fvpt = env_int("PIFFT_FUSED_VPT", (pc.R <= 512 && wgs <= 128) ? 8 : 16);
        if (fvpt != pc.vpt && find_pass(prec, pc.R, pc.C, 3, pc.nts, heavy_lp, fvpt)) pc.vpt = fvpt;
    }
    // The last strided pass of a small fp64 plan (R <= 512, <= 256
    // workgroups) at 8 values per thread too: measured on MI355X
    // (profiles/r04k_slice.log, r04k_shapes.log) config 2's one-GPU slice
    // 12.7 -> 12.2 us (+3.8 %), fp64 slices of local 2^16-2^19 +1.6-5 %, P = 1
    // 2^16-2^18 +5-6 %; 4 values per thread +2.6 % (slice).  PIFFT_LAST_VPT:
    // the values per thread instead (tuning, below).
    if (prec == 64 && out.size() > 1 && out.back().mode == 2 && out.back().vpt == 16) {
        PassChoice& pc = out.back();
        const uint64_t wgs = (ntrans * (M / (uint64_t)pc.R) + pc.C - 1) / (uint64_t)pc.C;
        if (pc.R <= 512 && wgs <= 256 && find_pass(prec, pc.R, pc.C, 2, pc.nts, 0, 8)) pc.vpt = 8;
    }
    // tuning: lines per workgroup (its write side's segment width) and values
    // per thread of the last pass
    const int last_c = env_int("PIFFT_LAST_C", 0), last_vpt = env_int("PIFFT_LAST_VPT", 0);
    if ((last_c > 0 || last_vpt > 0) && out.size() > 1) {
        PassChoice& b = out.back();
        const int c = last_c > 0 ? last_c : b.C, v = last_vpt > 0 ? last_vpt : b.vpt;
        if (find_pass(prec, b.R, c, b.mode, b.nts, 0, v)) {
            b.C = c;
            b.vpt = v;
        }
    }
    return 0;
}

void release(pifft_plan* p) {
    if (!p) return;
    DeviceGuard g(p->device);
    for (int b = BUF_W; b < NBUF; b++)
        if (p->buf[b]) (void)hipFree(p->buf[b]);
    if (p->d_tw) (void)hipFree(p->d_tw);
    if (p->d_hin) (void)hipFree(p->d_hin);
    if (p->d_hout) (void)hipFree(p->d_hout);
    if (p->d_gather) (void)hipFree(p->d_gather);
    for (auto st : p->gst) (void)hipStreamDestroy(st);
    for (auto e : p->gdone) (void)hipEventDestroy(e);
    for (auto e : p->gev)
        if (e) (void)hipEventDestroy(e);
    for (auto e : p->ev) (void)hipEventDestroy(e);
    for (auto e : p->sev)
        if (e) (void)hipEventDestroy(e);
    for (auto e : p->prof_ev) (void)hipEventDestroy(e);
    if (p->stream) (void)hipStreamDestroy(p->stream);
    delete p;
}

struct Elem {
    std::vector<Step> steps;
};

// dry: plan only (pifft_plan_dry_run) -- no device, no allocation
int build_plan(pifft_plan* p, bool dry = false) {
    const size_t esz = p->esz;
    const uint64_t ntrans = (uint64_t)p->batch * p->nq;  // local transforms
    std::vector<PassChoice> passes;
    // One worker per plan: the tree is fused into the first pass, which reads
    // the input once.  (Several workers per plan re-reading all P leaves in
    // each worker's fused pass measured no consistent win, profiles/
    // r02_fuse_all.log; removed in round 4.)
    // All P <= 16 workers of a natural-order plan on this GPU, with a
    // multi-pass local FFT: the worker-interleaved layout (PassArgs::wil).
    // The tree's one launch writes z_q[i] at i P + q, every pass reads and
    // writes rows holding all workers' values side by side, and the last pass
    // stores worker q at slot bitrev(q) -- the natural-order result, without
    // an interleave launch or scattered 16-B stores.  PIFFT_WORKER_IL=0: the
    // slice-major layout (+ interleave launch or natural-order store).
    const bool wil_ok = p->natural && p->P > 1 && p->nq == p->P && p->lp <= 4 && env_int("PIFFT_WORKER_IL", 1);
    const bool may_fuse = p->P > 1 && p->nq == 1 && p->lp <= 4 && !p->separate_tree && env_int("PIFFT_FUSE_TREE", 1);
    if (plan_passes(p->m, p->prec, ntrans, passes, may_fuse ? p->lp : 0, true, !wil_ok)) return -1;
    // the same radices, every pass a worker-interleaved MODE 2 (| 8) pass at
    // the C of a MODE 2 pass whose lines run over all workers
    auto to_wil = [&](std::vector<PassChoice>& w) -> bool {
        bool ok = true;
        for (auto& pc : w) {
            const uint64_t lines = p->m / (uint64_t)pc.R;
            pc.C = pick_lines(p->prec, pc.R, lines << p->lp, ntrans * lines,
                              p->prec == 64 ? "PIFFT_COL_C64" : "PIFFT_COL_C32", 2);
            pc.mode = 2 | 8;
            pc.vpt = 16;
            // tuning: at least this many lines per workgroup (e.g. P, so a
            // row holds every worker's value), if instantiated
            // (default P: 8 workers at C = 8 instead of 4 -- C2 35 -> 32 us,
            // fp32 2^20 P = 8 25 -> 24 us, 2^28 P = 8 unchanged at C = 16;
            // profiles/r03_worker_interleaved.log)
            const int cmin = env_int("PIFFT_WIL_CMIN", (int)p->P);
            if (cmin > pc.C && find_pass(p->prec, pc.R, cmin, pc.mode, pc.nts)) pc.C = cmin;
            ok = ok && find_pass(p->prec, pc.R, pc.C, pc.mode, pc.nts) != nullptr;
            // config-2-sized plans (<= 32 MiB of data): 8 values per thread
            // where instantiated (config 2 29.9 -> 29.0 us, profiles/
            // r04d_wil_vpt8_c2.log); PIFFT_WIL_VPT: instead (tuning)
            const bool small = (uint64_t)p->batch * p->n * esz <= (32ull << 20);
            const int wvpt = env_int("PIFFT_WIL_VPT", small ? 8 : 16);
            if (wvpt != pc.vpt && find_pass(p->prec, pc.R, pc.C, pc.mode, pc.nts, 0, wvpt)) pc.vpt = wvpt;
        }
        return ok;
    };
    if (wil_ok && passes.size() > 1) {
        std::vector<PassChoice> w = passes;
        if (to_wil(w)) {
            passes = w;
            p->wil = true;
        }
    }
    // A single transform whose local FFT is one pass (M <= 2^14) would run
    // tree + pass + interleave launches.  From M = 2^11 up the
    // worker-interleaved plan with every worker's tree fused into its first
    // pass (MODE 11 below: the first radix, then an M / R1-point pass) does
    // it in two, kept only where that fused plan exists (round 5,
    // profiles/r05w_small_wil.log: fp64 2^15 P = 2 22 -> 13 us, 2^16 P = 4
    // 23 -> 11, 2^17 P = 8 25 -> 12; fp32 2^17 P = 8 21 -> 9, 2^18 P = 16
    // 25 -> 13; 9-30 % at the other sizes).  PIFFT_WIL_SINGLE=0: off.
    // And a transform that fits one tile (P M <= 8192 values, from 1024: the
    // reference's own GPU sweep, cuda/run-experiments:16) runs every worker's
    // tree and its whole M-point FFT in ONE launch: the fused pass at J = 1 (C
    // = P lines of R = M points) storing natural order (PIFFT_WIL_ONE_LAUNCH=0:
    // off).  Batched, one workgroup per transform: 1.2-2.8x faster than tree +
    // pass (profiles/r05bo_batched_one_launch_ab.log; PIFFT_WIL_ONE_BATCH=0: off);
    // and batched two-pass plans 11-40 % (r05bt_batched_two_pass_ab.log;
    // PIFFT_WIL_SINGLE_BATCH=0: off).
    // The two-pass plan from M = 2^11 (fp64 2^14 P = 8 11 -> 10 us, fp32 8 vs
    // 11, fp32 2^15 P = 16 12 vs 14: profiles/r05za_small_plan_edges.log).
    // (PIFFT_WIL_ONE_MAX: the largest one-launch transform, values -- 16384
    // measured slower; the instances exist only where they compile spill-free.
    // PIFFT_WIL_SINGLE_MIN_LOG: the two-pass plan's smallest M, log2.  Tuning.)
    const uint64_t pm = (uint64_t)p->P * p->m;
    int nts0 = pick_nts(2 * ntrans * p->m * esz);
    // (fp64 P = 2 at M = 4096 spills at 16 values per thread: 8, 1024 threads,
    // batched only -- 64 transforms 21 -> 13 us, one 10 -> 12: profiles/r05v8_*)
    const int vpt0 = find_pass(p->prec, (int)p->m, (int)p->P, 11, 0, p->lp) ? 16 : p->batch >= 64 ? 8 : 0;
    if (nts0 && !find_pass(p->prec, (int)p->m, (int)p->P, 11, nts0, p->lp, vpt0)) nts0 = 0;  // (nt forms not instantiated)
    // (P = 32 too, one launch only: two threads per position, each evaluating
    // the tree pruned to half the workers)
    const bool wil_ok5 = p->natural && p->P > 1 && p->nq == p->P && p->lp == 5 && env_int("PIFFT_WORKER_IL", 1);
    const bool one_ok = (wil_ok || wil_ok5) && passes.size() == 1 && pm >= 1024 &&
                        pm <= (uint64_t)env_int("PIFFT_WIL_ONE_MAX", 8192) && env_int("PIFFT_WIL_ONE_LAUNCH", 1) &&
                        find_pass(p->prec, (int)p->m, (int)p->P, 11, nts0, p->lp, vpt0);
    const bool wil_single = (wil_ok || one_ok) && passes.size() == 1 && env_int("PIFFT_WIL_SINGLE", 1) &&
                            (((p->batch == 1 || env_int("PIFFT_WIL_SINGLE_BATCH", 1)) &&
                              p->m >= (1ull << env_int("PIFFT_WIL_SINGLE_MIN_LOG", 11))) ||
                             (one_ok && (p->batch == 1 || env_int("PIFFT_WIL_ONE_BATCH", 1))));
    if (wil_single) p->wil = true;
    // The worker-interleaved plan with its tree fused into the first pass
    // (MODE 11, k_pass wil_tree_to_lds): a tile of J adjacent line indices x
    // all P workers loads each position's P leaves once (J esz-byte leaf
    // rows) and evaluates every worker's tree there, so the tree launch (N
    // read + N written) and the first pass's re-read of its output are gone.
    // The first radix is what that tile leaves (8192 / (J P)), the rest of
    // the local FFT is planned as usual.  J by measurement (round 5,
    // profiles/r05m_wil_fuse_j.log, the separate tree launch in brackets):
    //   fp64, J = 8: config 2 (2^20 P = 8) 26 us (29), 2^20 P = 4 23 (31),
    //     P = 2 25 (31), 2^24 P = 8 310 (381), 2^26 P = 4 1.18 ms (1.50),
    //     2^28 P = 8 4.98 ms (6.31), P = 16 5.84 (6.13); but P = 16 below
    //     256 MiB ties or loses (2^20: 28-45 vs 26 us) -> separate there;
    //     J = 16 (256-B leaf rows, first radix 64 at P = 8) loses on the
    //     remaining passes it leaves (a 1024 / 2048 pass at 8 lines);
    //   fp32: J = 8 up to 32 MiB (2^20 P = 8 20 vs 24 us), J = 16 up to
    //     1 GiB (2^24 P = 8 165 vs 208 us); 2^28 P = 8 keeps the separate tree
    //     (3.26 vs 3.39-3.51 ms: its remaining passes at 8-B values get
    //     128-B rows).
    // Two refinements for P <= 8 (round 5, profiles/r05s_*, r05t_*, r05u_*;
    // every output checked against the default plan's):
    //   - where the 8192-value tile leaves fewer than 256 workgroups (<= 2^20
    //     values: 128), the tile is halved and J = 4, so every CU gets one:
    //     config 2 26 -> 23 us, fp64 2^20 P = 4 23 -> 21, P = 2 25 -> 23,
    //     2^19 P = 8 21 -> 18, 2^18 P = 8 16 -> 14; fp32 2^20 P = 2-8 -1 us;
    //   - where J = 8 leaves a remainder the rest of the plan splits in two
    //     passes (> 2048 points) and J = 4 leaves one pass: J = 4 (fp64 2^22
    //     P = 2 / 4 / 8: 68 / 65 / 64 -> 54 / 51 / 50 us); fp32 at P = 8 from a
    //     2048-point remainder on (2^21 27 -> 24 us, 2^22 51 -> 42).  (fp32 at
    //     P <= 4 keeps J = 8: its J = 4 remainder passes run at 4 lines, 32-B
    //     rows: 2^22 P = 4 50 -> 75 us.)
    // PIFFT_SEPARATE_TREE (CLI -u) or PIFFT_WIL_FUSE=0: the separate tree
    // launch; PIFFT_WIL_FUSE_J: J (then the tile stays 8192 unless
    // PIFFT_WIL_FUSE_TILE says otherwise), PIFFT_WIL_FUSE_TILE: the tile
    // (values), PIFFT_WIL_FUSE_VPT: values per thread (tuning, tests).
    uint32_t wil_fused_c = 0;
    if (wil_single && one_ok && !p->separate_tree && env_int("PIFFT_WIL_FUSE", 1)) {
        passes = {PassChoice{(int)p->m, (int)p->P, 11, nts0, vpt0}};
        wil_fused_c = p->P;
    }
    if (p->wil && !wil_fused_c && !p->separate_tree && env_int("PIFFT_WIL_FUSE", 1)) {
        const uint64_t data = (uint64_t)p->batch * p->n * esz;
        const int jdef = p->prec == 64 ? ((p->lp <= 3 || data >= (256ull << 20)) ? 8 : 0)
                                       : (data <= (32ull << 20) ? 8 : data <= (1ull << 30) ? 16 : 0);
        int J = jdef, tile1 = tile_elems(p->prec);
        if (jdef == 8 && p->lp <= 3) {
            const uint64_t rest8 = p->m / (uint64_t)(tile1 / (8 << p->lp)), rest4 = rest8 / 2;
            if ((uint64_t)p->batch * p->n / (uint64_t)tile1 < 256) {
                tile1 /= 2;
                J = 4;
            } else if (rest8 > (p->prec == 64 ? 2048u : 1024u) && rest4 <= 2048 && (p->prec == 64 || p->lp == 3)) {
                J = 4;
            }
        } else if (jdef == 8 && p->lp == 4) {
            // fp32 P = 16: J = 4 where it leaves a remainder of at most 1024
            // points (2^21: 41 -> 26 us; at 2048 its 4-line pass loses, 2^22
            // 52 -> 90, r05u_wil_fuse_remainder.log)
            const uint64_t rest8 = p->m / (uint64_t)(tile1 / (8 << p->lp));
            if (rest8 > 1024 && rest8 / 2 <= 1024) J = 4;
        } else if (jdef == 0 && p->lp == 4 && p->prec == 64 && data >= (32ull << 20) && data <= (64ull << 20)) {
            J = 2;  // fp64 P = 16 at 32-64 MiB: fused at J = 2 (2^21 43 -> 37 us, 2^22 70 -> 65; 2^23 loses)
        }
        const int jenv = env_int("PIFFT_WIL_FUSE_J", -1);
        if (jenv >= 0) {
            J = jenv;
            tile1 = tile_elems(p->prec);
        }
        tile1 = env_int("PIFFT_WIL_FUSE_TILE", tile1);
        const int C1 = J > 0 ? J << p->lp : 0;
        const int R1 = C1 > 0 ? tile1 / C1 : 0;
        const int vpt1 = env_int("PIFFT_WIL_FUSE_VPT", 16);
        const int nts1 = pick_nts(2 * ntrans * p->m * esz);
        std::vector<PassChoice> rest;
        const uint64_t m2 = R1 > 0 ? p->m / (uint64_t)R1 : 0;
        bool ok = R1 >= 16 && (uint64_t)R1 < p->m && m2 >= (uint64_t)J && find_pass(p->prec, R1, C1, 11, nts1, p->lp, vpt1) &&
                  plan_passes(m2, p->prec, ntrans * (uint64_t)R1, rest, 0, false, false) == 0;
        // (worker-interleaved passes exist up to R = 2048: a longer single
        // remainder becomes two balanced passes)
        if (ok && rest.size() == 1 && rest[0].R > 2048) {
            const int l = ilog2u(m2);
            rest = {PassChoice{1 << ((l + 1) / 2), 0, 2, rest[0].nts}, PassChoice{1 << (l / 2), 0, 2, rest[0].nts}};
        }
        if (ok && to_wil(rest)) {
            passes.clear();
            passes.push_back({R1, C1, 11, nts1, vpt1});
            for (const auto& pc : rest) passes.push_back(pc);
            wil_fused_c = (uint32_t)C1;
        }
    }
    if (wil_single && !wil_fused_c) {
        // no fused plan: the single pass -- except P = 16 at fp64 (no fused
        // pass below 256 MiB, above), where the worker-interleaved two-pass
        // plan after its tree launch still saves the interleave launch (2^16
        // 16 -> 15 us, 2^17 21 -> 16, 2^18 30 -> 19; r05w_small_wil.log)
        std::vector<PassChoice> w;
        p->wil = p->lp == 4 && p->batch == 1 && p->m >= 4096 && plan_passes(p->m, p->prec, ntrans, w, 0, false, false, ilog2u(p->m) - 1) == 0 &&
                 w.size() == 2 && to_wil(w);
        if (p->wil) passes = w;
    }
    if (p->bitrev && !passes.empty()) {
        // the last pass stores in bit-reversed order: its MODE | 4 twin, at
        // the planned C or the widest instantiated one below it
        PassChoice& l = passes.back();
        const int bm = l.mode, cmin = bm == 0 ? 1 : 4;
        if (l.vpt == 8 && !find_pass(p->prec, l.R, l.C, bm | 4, l.nts, 0, 8)) l.vpt = 16;  // (no VPT-8 twin)
        int C = l.C;
        while (C > cmin && !find_pass(p->prec, l.R, C, bm | 4, l.nts, 0, l.vpt)) C /= 2;
        if (!find_pass(p->prec, l.R, C, bm | 4, l.nts, 0, l.vpt))
            return fail("no bit-reversed pass kernel R=%d C=%d mode=%d", l.R, l.C, bm);
        l.C = C;
        l.mode = bm | 4;
    }

    // All P workers on this plan, natural order, and an output small enough to
    // stay in L2 / the Infinity Cache: the last pass stores each worker's bins
    // at their natural positions bitrev(q) + P k itself (plain stores; the P
    // workers' tiles of a line block back to back on one XCD) instead of a
    // slice-major store plus an interleave launch.  Measured on MI355X
    // (profiles/r02_ilv_store.log, wall per transform): fp64 2^18-2^22 P=2-16
    // 1-22 % faster, fp32 2^20 P=8 7 %, batched single-pass plans (4096 x
    // 4096 fp32 P=4, 1024 x 2^12 fp64 P=4) 13-16 %; 2^23 fp64 and 2^22 fp32
    // (32 MiB) single transforms up to 5 % slower, few tiles (2^16: 8) 12 %.
    // PIFFT_ILV: -1 this rule, 0 never, 1 always (where it applies).
    {
        const int force = env_int("PIFFT_ILV", -1);
        const bool ok = p->natural && p->P > 1 && p->nq == p->P && !passes.empty() && !p->wil;
        bool on = ok && force == 1;
        if (ok && force < 0) {
            const PassChoice& l = passes.back();
            const uint64_t tiles = (ntrans * (p->m / (uint64_t)l.R) + l.C - 1) / (uint64_t)l.C;
            const uint64_t cap_mib = passes.size() == 1 ? (uint64_t)env_int("PIFFT_ILV_SINGLE_MAX_MIB", 128)
                                     : p->prec == 64    ? (uint64_t)env_int("PIFFT_ILV_MAX_MIB64", 64)
                                                        : (uint64_t)env_int("PIFFT_ILV_MAX_MIB32", 16);
            on = tiles >= (uint64_t)env_int("PIFFT_ILV_MIN_TILES", 256) &&
                 (uint64_t)p->batch * p->n * esz <= (cap_mib << 20);
        }
        p->ilv = on;
    }
    if (p->ilv) passes.back().nts = 0;
    TableBuilder tb(esz);
    tb.size_only = dry;
    // --- tree tables (w_N) ---
    const bool need_tree = p->P > 1;
    size_t tree_direct = 0;
    TwoLevel tree2;
    bool tree_is_direct = false;
    // The worker-interleaved plan's one tree launch (k_tree_wil) feeds its
    // passes only -- its output is never observed, and the plan's result
    // matches the oracle within tolerance either way -- so from 2^21 values
    // up it takes the factored two-level twiddles (one small-table lookup per
    // level and thread) instead of the reference-formula table, whose
    // N (1 - 1/P) entries it otherwise reads beside the data (C2: 1.44x its
    // algorithmic bytes, profiles/r05b_traffic_n2^20_f64_b1_P8_q8.json).
    // Measured on MI355X (profiles/r05g_wil_tree.log): fp64 2^21 P = 8
    // 46 -> 42 us, 2^22 P = 16 80 -> 70 us; but config 2 itself (fp64 2^20,
    // P = 8: 512 workgroups, one round, latency-bound) 29 -> 31 us -- there
    // the extra dependent fp64 products sit on the critical path -- and 2^18
    // ties.  The stand-alone tree (pifft_tree_device) keeps the reference
    // table and stays bitwise.  PIFFT_WIL_TREE_DIRECT=1: the reference table
    // at every size (tuning, tests); PIFFT_WIL_TREE_MIN_LOG: the threshold.
    bool wil_factored = false;
    if (need_tree) {
        const int direct_max = env_int("PIFFT_TREE_DIRECT_MAX_LOG", 22);
        if (p->log_n <= direct_max) {
            tree_is_direct = true;
            tree_direct = tb.reference_omega_levels(p->n, p->lp);
            // (and at P = 32, whose one-launch pass evaluates 16 workers' tree
            // per thread: 80 dependent table lookups each, against 5: 2^10
            // 12 -> 8 us, fp32 11 -> 6; P = 16 ties, profiles/r05p32b_*)
            wil_factored = p->wil && env_int("PIFFT_WIL_TREE_DIRECT", 0) == 0 &&
                           ((uint64_t)p->batch * p->n >= (1ull << env_int("PIFFT_WIL_TREE_MIN_LOG", 21)) || p->lp == 5);
            if (wil_factored) tree2 = two_level(tb, p->n);
        } else {
            tree2 = two_level(tb, p->n);
        }
    }
    // --- pass tables ---
    std::vector<size_t> tw_r(passes.size());
    for (size_t i = 0; i < passes.size(); i++) {
        size_t found = (size_t)-1;
        for (size_t j = 0; j < i; j++)
            if (passes[j].R == passes[i].R) found = tw_r[j];
        tw_r[i] = (found != (size_t)-1) ? found : tb.roots(passes[i].R, passes[i].R, 1);
    }
    TwoLevel pass2;
    if (passes.size() > 1) pass2 = two_level(tb, p->m);  // (every worker-interleaved plan has >= 2 passes)
    tb.align();
    p->tw_bytes = tb.size() ? tb.size() : 256;
    if (!dry) {
        HIPCHK(hipMalloc(&p->d_tw, p->tw_bytes));
        if (!tb.blob.empty()) HIPCHK(hipMemcpy(p->d_tw, tb.blob.data(), tb.blob.size(), hipMemcpyHostToDevice));
    }
    auto twp = [&](size_t off) { return (const void*)((const char*)p->d_tw + off); };
    TreeTw ttw{};
    if (need_tree) {
        ttw.direct = tree_is_direct ? twp(tree_direct) : nullptr;
        ttw.lo = tree_is_direct ? nullptr : twp(tree2.lo);
        ttw.hi = tree_is_direct ? nullptr : twp(tree2.hi);
        ttw.h = tree2.h;
        ttw.log_n = (uint32_t)p->log_n;
    }
    // One worker on this plan, a multi-pass local FFT and log2 P <= 4: fuse the
    // tree into the first pass (its P leaves per input instead of a separate
    // tree launch that writes, and a pass that re-reads, the N/P segment).
    const PassKernel* fused = nullptr;
    if (may_fuse && passes.size() > 1)
        fused = find_pass(p->prec, passes[0].R, passes[0].C, 3, passes[0].nts, p->lp, passes[0].vpt);
    if (wil_fused_c) fused = find_pass(p->prec, passes[0].R, passes[0].C, 11, passes[0].nts, p->lp, passes[0].vpt);
    p->fused_tree = fused != nullptr;

    // the worker-interleaved plan's tree twiddles (its k_tree_wil launch or
    // its fused first pass): factored from 2^21 values up (wil_factored)
    TreeTw wtw = ttw;
    if (wil_factored) {
        wtw.direct = nullptr;
        wtw.lo = twp(tree2.lo);
        wtw.hi = twp(tree2.hi);
        wtw.h = tree2.h;
    }

    // --- chain: [tree] [passes] [interleave] ---
    std::vector<Elem> chain;
    const uint64_t M = p->m;
    if (need_tree) {
        Elem e;
        // ceil(log2 P / 4) launches of up to 4 levels each; in place over
        // one position-space buffer between launches (see k_tree)
        static const void* tk64[5] = {nullptr, (const void*)&k_tree<double, 1>, (const void*)&k_tree<double, 2>,
                                      (const void*)&k_tree<double, 3>, (const void*)&k_tree<double, 4>};
        static const void* tk32[5] = {nullptr, (const void*)&k_tree<float, 1>, (const void*)&k_tree<float, 2>,
                                      (const void*)&k_tree<float, 3>, (const void*)&k_tree<float, 4>};
        const int nl = (p->lp + 3) / 4;
        // number of level-t blocks (P >> t workers each) holding a requested worker
        auto blocks_needed = [&](int t) -> uint64_t {
            const uint64_t w = (uint64_t)p->P >> t;
            return ((uint64_t)p->q0 + p->nq - 1) / w - (uint64_t)p->q0 / w + 1;
        };
        int t0 = 0;
        for (int l = 0; l < nl; l++) {
            const int L = (p->lp - t0 + (nl - l) - 1) / (nl - l);  // spread levels evenly
            const bool first = (l == 0), last = (l == nl - 1);
            Step s;
            s.kind = STEP_TREE;
            s.fn = p->prec == 64 ? tk64[L] : tk32[L];
            s.src = first ? -1 : BUF_TA;  // -1: chain input
            s.dst = last ? -2 : BUF_TA;   // -2: chain output (slice-major)
            s.ta.tw = ttw;
            s.ta.in_bstride = p->n;
            s.ta.out_bstride = last ? (uint64_t)p->nq * M : p->n;
            s.ta.out_shift = last ? -(int64_t)((uint64_t)p->q0 * M) : 0;
            s.ta.total = (uint64_t)p->batch * (p->n >> L);
            s.ta.log_n = (uint32_t)p->log_n;
            s.ta.log_p = (uint32_t)p->lp;
            s.ta.t0 = (uint32_t)t0;
            s.ta.q0 = p->q0;
            s.ta.nq = p->nq;
            s.block = dim3(256);
            s.grid = dim3(stride_grid(s.ta.total / (uint64_t)std::max(1, env_int("PIFFT_TREE_GRID_DIV", 1))));
            s.bytes = (uint64_t)p->batch * esz *
                      (blocks_needed(t0) * (p->n >> t0) + blocks_needed(t0 + L) * (p->n >> (t0 + L)));
            e.steps.push_back(s);
            t0 += L;
        }
        if (nl > 1) p->bytes_ta = (size_t)p->batch * p->n * esz;
        // the stand-alone tree (pifft_tree_device) reads d_in and writes d_seg
        // (slice-major, always)
        for (Step t : e.steps) {
            if (t.src == -1) t.src = BUF_IN;
            if (t.dst == -2) t.dst = BUF_OUT;
            p->tree_only.push_back(t);
        }
        if (p->wil && p->lp <= 4) {  // one launch over all workers: the passes' interleaved layout
            static const void* tw64[5] = {nullptr, (const void*)&k_tree_wil<double, 1>, (const void*)&k_tree_wil<double, 2>,
                                          (const void*)&k_tree_wil<double, 3>, (const void*)&k_tree_wil<double, 4>};
            static const void* tw32[5] = {nullptr, (const void*)&k_tree_wil<float, 1>, (const void*)&k_tree_wil<float, 2>,
                                          (const void*)&k_tree_wil<float, 3>, (const void*)&k_tree_wil<float, 4>};
            Step& t = e.steps.back();
            t.fn = p->prec == 64 ? tw64[p->lp] : tw32[p->lp];
            t.ta.tw = wtw;
            t.ta.out_bstride = p->n;
            t.lds = (size_t)tree_wil_pad(256u << p->lp) * esz;
            if (t.lds > 65536 && !dry) (void)hipFuncSetAttribute(t.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)t.lds);
        }
        if (!fused) {
            p->tree_steps = (int)e.steps.size();
            chain.push_back(e);
        }
    }
    uint64_t ns = 1;
    p->npasses = (int)passes.size();
    for (size_t i = 0; i < passes.size(); i++) {
        const bool fuse_here = (i == 0 && fused);
        const bool last_pass = i + 1 == passes.size() && passes.size() > 1;
        // tuning: the last pass's streaming form (0 plain, 1 nt both, 2 nt loads, 3 nt stores)
        int nt_override = last_pass && passes[i].mode == 2 ? env_int("PIFFT_LAST_NT", -1) : -1;
        // (and the first pass's, 0 plain / 1 nt both, of a plan without a fused tree; round 6,
        // profiles/r06y3_*: the default stays)
        if (i == 0 && !fuse_here && passes.size() > 1 && passes[i].mode == 1)
            nt_override = env_int("PIFFT_FIRST_NT", -1);
        const PassKernel* k = fuse_here ? fused
                                        : find_pass(p->prec, passes[i].R, passes[i].C, passes[i].mode,
                                                    nt_override >= 0 ? nt_override : passes[i].nts, 0, passes[i].vpt);
        if (!k) return fail("no pass kernel R=%d C=%d", passes[i].R, passes[i].C);
        Step s;
        s.kind = fuse_here ? STEP_TREE_PASS : STEP_PASS;
        s.fn = k->fn;
        s.pk = k;
        s.nts = k->nts;
        const int logr = ilog2u((uint64_t)k->R);
        s.pa.tw_r = twp(tw_r[i]);
        s.pa.tw_lo = passes.size() > 1 ? twp(pass2.lo) : nullptr;
        s.pa.tw_hi = passes.size() > 1 ? twp(pass2.hi) : nullptr;
        s.pa.tw_h = pass2.h;
        s.pa.in_bstride = (i == 0 && (!need_tree || fuse_here)) ? p->n : M;
        if (fuse_here) {
            s.pa.tree = p->wil ? wtw : ttw;
            s.pa.worker = p->q0;
            s.pa.log_nq = (uint32_t)ilog2u(p->nq);
        }
        s.pa.out_bstride = M;
        s.pa.nlines = ntrans * (M >> logr);
        s.pa.log_lb = (uint32_t)(p->log_m - logr);
        s.pa.log_ns = (uint32_t)ilog2u(ns);
        s.pa.tw_shift = (uint32_t)(p->log_m - ilog2u(ns) - logr);
        s.pa.log_xg = (uint32_t)env_int((passes[i].mode & 3) == 0 ? "PIFFT_XCD_GROUP_SINGLE" : "PIFFT_XCD_GROUP",
                                        (passes[i].mode & 3) == 0 ? 0 : 2);
        if (last_pass) s.pa.log_xg = (uint32_t)env_int("PIFFT_LAST_XCD_GROUP", (int)s.pa.log_xg);
        if (p->wil) {
            s.pa.wil = (uint32_t)p->lp;
            s.pa.wbrev = (i + 1 == passes.size()) ? 1u : 0u;  // the last pass: natural order
            s.pa.in_bstride = s.pa.out_bstride = p->n;          // a transform's P interleaved workers
        }
        if (p->ilv && i + 1 == passes.size()) {
            s.pa.ilv_log = (uint32_t)p->lp;
            s.pa.out_bstride = p->n;
            s.pa.log_xg = std::max<uint32_t>(s.pa.log_xg, (uint32_t)env_int("PIFFT_ILV_XCD_GROUP", p->lp));
        }
        s.block = dim3((unsigned)k->nt);
        const uint64_t wgs = (s.pa.nlines + (uint64_t)k->C - 1) / (uint64_t)k->C;
        if (wgs * (uint64_t)k->nt >= (1ull << 32)) return fail("transform too large for one launch (%llu work-items)",
                                                             (unsigned long long)(wgs * k->nt));
        s.grid = dim3((unsigned)wgs);
        s.lds = (size_t)k->lds_bytes;
        // (a one-worker fused pass reads every leaf of its worker's transform:
        // N per worker; the all-worker one, MODE 11, each leaf once)
        s.bytes = (!fuse_here || p->wil) ? 2 * ntrans * M * esz : (uint64_t)p->batch * p->nq * (p->n + M) * esz;
        if (s.lds > 65536 && !dry)
            (void)hipFuncSetAttribute(k->fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)s.lds);
        if (i < 8) {
            p->radix[i] = k->R;
            p->lines[i] = k->C;
            p->vpt[i] = k->vpt;
        }
        ns *= (uint64_t)k->R;
        Elem e;
        e.steps.push_back(s);
        chain.push_back(e);
    }
    if (p->natural && p->P > 1 && !p->ilv && !p->wil) {
        Step s;
        s.kind = STEP_INTERLEAVE;
        s.fn = interleave_fn(p->prec, p->lp, p->n);
        s.il_total = (uint64_t)p->batch * p->n;
        s.il_log_n = (uint32_t)p->log_n;
        s.il_log_p = (uint32_t)p->lp;
        s.block = dim3(256);
        s.grid = dim3(stride_grid(interleave_threads(s.il_total, p->lp, p->prec, p->n)));
        s.bytes = 2 * s.il_total * esz;
        Elem e;
        e.steps.push_back(s);
        chain.push_back(e);
    }
    if (chain.empty()) return fail("empty plan");
    // destinations, backwards: last -> OUT, then W, OUT, W, ...
    std::vector<int> dst(chain.size());
    for (size_t i = chain.size(); i-- > 0;) dst[i] = ((chain.size() - 1 - i) % 2 == 0) ? BUF_OUT : BUF_W;
    bool need_w = false;
    for (size_t i = 0; i < chain.size(); i++) {
        const int src = (i == 0) ? BUF_IN : dst[i - 1];
        if (dst[i] == BUF_W || src == BUF_W) need_w = true;
        for (auto& s : chain[i].steps) {
            if (s.src == -1) s.src = src;
            if (s.dst == -2) s.dst = dst[i];
            p->steps.push_back(s);
        }
    }
    if (p->steps.size() > 4096) return fail("plan too large (%zu launches)", p->steps.size());
    // Padded workspace rows (PassArgs::in_pad / out_pad): where one k_pass
    // writes W and a later pass (BM 2) reads it, W's rows are spread by
    // w_pad elements each, so their offsets no longer coincide with the
    // caller's output rows that the same passes read or write.  Measured on
    // MI355X over fresh (W, output) allocation pairs (tools/probe_wpad.py,
    // profiles/r02_wpad.log): C4 fp64 2^28 4.88 -> 4.73 ms mean (worst 5.03
    // -> 4.82), fp32 2^28 3.22 -> 3.19 ms, with 16 KiB + 256 B per row;
    // 1 MiB + 256 B ties at fp64 and loses 4 % at fp32.  Only for W >= 2 GiB:
    // at 512 MiB (fp64 2^25, the worker of 8 at 2^28) padding cost 1.5-2.5 %,
    // at 1 GiB it ties, at 2 GiB (the worker of 2 at 2^28, of 8 at 2^30) it
    // gains ~0.5 % (profiles/r02_wpad.log, tools/gpu_wpad_shapes.sh).
    uint64_t w_tr = M;  // elements per transform in W
    const uint64_t w_pad = (uint64_t)env_int("PIFFT_W_PAD", (int)((16384 + 256) / esz));
    const uint64_t w_min = (uint64_t)env_int("PIFFT_W_PAD_MIN_MIB", 2048) << 20;
    if (w_pad && !p->wil && (uint64_t)p->batch * p->nq * M * esz >= w_min) {
        for (size_t i = 0; i + 1 < p->steps.size(); i++) {
            Step& a = p->steps[i];
            Step& b = p->steps[i + 1];
            if (a.dst != b.src || a.dst != BUF_W || (a.kind != STEP_PASS && a.kind != STEP_TREE_PASS) ||
                b.kind != STEP_PASS || b.pa.log_ns == 0 || a.pa.ilv_log)
                continue;
            const uint64_t rows = M >> b.pa.log_lb;  // the reading pass's radix
            const uint64_t tr = M + rows * w_pad;
            const uint32_t logr_a = (uint32_t)(p->log_m - a.pa.log_lb);  // the writing pass's radix
            a.pa.out_pad = b.pa.in_pad = (uint32_t)w_pad;
            a.pa.out_pad_log = b.pa.log_lb - logr_a;
            a.pa.out_bstride = b.pa.in_bstride = tr;
            w_tr = std::max(w_tr, tr);
        }
    }
    p->bytes_w = need_w ? (size_t)p->batch * p->nq * w_tr * esz : 0;
    if (dry) return 0;
    // tuning knob (tools/probe_place.py): hipExtMallocWithFlags flags for the
    // ping-pong workspace, e.g. 4 = hipDeviceMallocContiguous
    const int w_flags = env_int("PIFFT_W_MALLOC_FLAGS", 0);
    if (p->bytes_w)
        HIPCHK(w_flags ? hipExtMallocWithFlags(&p->buf[BUF_W], p->bytes_w, (unsigned)w_flags)
                       : hipMalloc(&p->buf[BUF_W], p->bytes_w));
    if (p->bytes_ta) HIPCHK(hipMalloc(&p->buf[BUF_TA], p->bytes_ta));
    HIPCHK(hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking));
    p->ev.resize(2 * p->steps.size());
    for (auto& e : p->ev) HIPCHK(hipEventCreateWithFlags(&e, kTimingEventFlags));
    for (auto& e : p->sev) HIPCHK(hipEventCreateWithFlags(&e, kTimingEventFlags));
    return 0;
}

int create(pifft_plan** out, uint64_t n, uint32_t workers, uint32_t first, uint32_t count,
           uint32_t batch, int prec, int device, int flags, bool dry = false) {
    if (!out) return fail("plan pointer is NULL");
    *out = nullptr;
    if (n < 2 || !is_pow2(n)) return fail("Invalid input size (should be 2^i for i>0)");
    if (workers == 0 || !is_pow2(workers)) return fail("Invalid number of procs (should be 2^i for i>0)");
    if (workers > n) return fail("More processors than inputs!");
    if (count == 0 || !is_pow2(count) || first % count != 0 || (uint64_t)first + count > workers)
        return fail("invalid worker range [%u, %u) of %u", first, first + count, workers);
    if (batch == 0) return fail("batch must be >= 1");
    if (prec != PIFFT_F32 && prec != PIFFT_F64) return fail("prec must be PIFFT_F32 or PIFFT_F64");
    const int order = flags & ~PIFFT_SEPARATE_TREE;
    if (order != PIFFT_OUT_NATURAL && order != PIFFT_OUT_SLICES && order != PIFFT_OUT_BITREV)
        return fail("unknown flags %d", flags);
    if (order == PIFFT_OUT_NATURAL && count != workers)
        return fail("natural-order output needs all workers on one plan (use PIFFT_OUT_SLICES)");
    if (!dry) {
        int ndev = 0;
        if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail("no HIP device available");
        if (device < 0 || device >= ndev) return fail("device %d out of range (%d devices)", device, ndev);
    }
    pifft_plan* p = new pifft_plan;
    p->n = n;
    p->P = workers;
    p->q0 = first;
    p->nq = count;
    p->batch = batch;
    p->prec = prec;
    p->device = device;
    p->flags = flags;
    p->natural = (order == PIFFT_OUT_NATURAL);
    p->bitrev = (order == PIFFT_OUT_BITREV);
    p->separate_tree = (flags & PIFFT_SEPARATE_TREE) != 0;
    p->esz = prec == PIFFT_F64 ? 16 : 8;
    p->lp = ilog2u(workers);
    p->log_n = ilog2u(n);
    p->log_m = p->log_n - p->lp;
    p->m = n >> p->lp;
    if (dry) p->device = -1;
    DeviceGuard g(dry ? -1 : device);
    if (build_plan(p, dry)) {
        std::string keep = g_err;
        release(p);
        g_err = keep;
        return -1;
    }
    *out = p;
    return 0;
}

// One launch.  With events (e0, e1): hipExtLaunchKernel binds them to the
// kernel's own dispatch (its start and end timestamps, what rocprofv3 reports
// as the kernel's duration) -- no marker packet between launches.  Marker
// events (hipEventRecord before every launch) cost ~4 us of GPU time each and
// made the per-launch means of the 10-50 us configs longer than their steps
// (round-2 verdict); kernel-bound events add nothing to the stream.
int launch_step(pifft_plan* p, const Step& s, const void* d_in, void* d_out, hipStream_t st,
                hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr) {
    void* base[NBUF] = {const_cast<void*>(d_in), d_out, p->buf[BUF_W], p->buf[BUF_TA]};
    const char* src = (const char*)base[s.src] + s.src_off * p->esz;
    char* dst = (char*)base[s.dst] + s.dst_off * p->esz;
    auto go = [&](void** args, size_t lds) {
        return (e0 || e1) ? hipExtLaunchKernel(s.fn, s.grid, s.block, args, lds, st, e0, e1, 0)
                          : hipLaunchKernel(s.fn, s.grid, s.block, args, lds, st);
    };
    hipError_t e = hipSuccess;
    switch (s.kind) {
        case STEP_PASS:
        case STEP_TREE_PASS: {
            PassArgs a = s.pa;
            a.in = src;
            a.out = dst;
#ifdef PIFFT_WG_CLOCK
            a.wg_clock = p->dbg_clk;
#endif
            void* args[] = {&a};
            e = go(args, s.lds);
            break;
        }
        case STEP_TREE: {
            TreeArgs a = s.ta;
            a.in = src;
            a.out = dst;
            void* args[] = {&a};
            e = go(args, s.lds);
            break;
        }
        case STEP_INTERLEAVE: {
            const void* in = src;
            void* o = dst;
            uint64_t total = s.il_total;
            uint32_t ln = s.il_log_n, lpp = s.il_log_p;
            void* args[] = {&in, &o, &total, &ln, &lpp};
            e = go(args, 0);
            break;
        }
        default:
            return fail("bad step kind %d", s.kind);
    }
    if (e != hipSuccess) return fail("kernel launch failed: %s", hipGetErrorString(e));
    return 0;
}

// every launch of the plan; ev (or NULL): 2 events per launch, its start and stop
int launch_steps(pifft_plan* p, const void* d_in, void* d_out, hipStream_t st, hipEvent_t* ev) {
    for (size_t i = 0; i < p->steps.size(); i++)
        if (launch_step(p, p->steps[i], d_in, d_out, st, ev ? ev[2 * i] : nullptr, ev ? ev[2 * i + 1] : nullptr))
            return -1;
    return 0;
}

// per-launch durations of one recorded execution (ev as launch_steps)
int read_launch_ms(size_t ns, hipEvent_t* ev, std::vector<float>& ms) {
    ms.assign(ns, 0.0f);
    if (!ns) return 0;
    HIPCHK(hipEventSynchronize(ev[2 * ns - 1]));
    for (size_t i = 0; i < ns; i++) HIPCHK(hipEventElapsedTime(&ms[i], ev[2 * i], ev[2 * i + 1]));
    return 0;
}

int check_buffers(const pifft_plan* p, const void* d_in, void* d_out) {
    if (!p) return fail("plan is NULL");
    if (!d_in || !d_out) return fail("NULL device buffer");
    if (d_in == d_out) return fail("in-place execution is not supported (d_in == d_out)");
    return 0;
}

uint64_t out_elems(const pifft_plan* p) { return (uint64_t)p->batch * p->nq * p->m; }

// run every step with kernel-bound events, wait, per-launch durations
int run_timed(pifft_plan* p, const void* d_in, void* d_out, hipStream_t st, std::vector<float>& ms) {
    if (launch_steps(p, d_in, d_out, st, p->ev.data())) return -1;
    return read_launch_ms(p->steps.size(), p->ev.data(), ms);
}

bool stage1_step(const Step& s) { return s.kind == STEP_TREE || s.kind == STEP_TREE_PASS; }

void stage_split(const pifft_plan* p, const std::vector<float>& ms, double* s1, double* s2) {
    double a = 0, b = 0;
    for (size_t i = 0; i < ms.size(); i++) (stage1_step(p->steps[i]) ? a : b) += ms[i];
    if (s1) *s1 = a;
    if (s2) *s2 = b;
}

// One execution timed like the reference's two stage timers (tm_funnel,
// tm_tube: wall clock around each whole stage, CPU.c:414-481): a marker
// event before the stage's first launch and after its last, so the gaps and
// launch latency between kernels count.  (The stage-1 launches -- the tree,
// or the tree fused into the first pass -- lead every plan.)
// An empty stage (P = 1: no tree, as the reference's funnel loop that never
// runs; M = 1: no local FFT) gets no marker of its own and reads 0.
size_t stage1_launches(const pifft_plan* p) {
    size_t n1 = 0;
    while (n1 < p->steps.size() && stage1_step(p->steps[n1])) n1++;
    return n1;
}
int launch_stage_marked(pifft_plan* p, const void* d_in, void* d_out) {
    const size_t n1 = stage1_launches(p), ns = p->steps.size();
    HIPCHK(hipEventRecord(p->sev[0], p->stream));
    for (size_t i = 0; i < ns; i++) {
        if (i == n1 && n1 > 0) HIPCHK(hipEventRecord(p->sev[1], p->stream));
        if (launch_step(p, p->steps[i], d_in, d_out, p->stream)) return -1;
    }
    HIPCHK(hipEventRecord(p->sev[2], p->stream));
    return 0;
}
int read_stage_marked(pifft_plan* p, double* s1, double* s2) {
    const size_t n1 = stage1_launches(p), ns = p->steps.size();
    float a = 0.0f, b = 0.0f;
    HIPCHK(hipEventSynchronize(p->sev[2]));
    if (n1 == 0)
        HIPCHK(hipEventElapsedTime(&b, p->sev[0], p->sev[2]));
    else if (n1 == ns)
        HIPCHK(hipEventElapsedTime(&a, p->sev[0], p->sev[2]));
    else {
        HIPCHK(hipEventElapsedTime(&a, p->sev[0], p->sev[1]));
        HIPCHK(hipEventElapsedTime(&b, p->sev[1], p->sev[2]));
    }
    *s1 = a;
    *s2 = b;
    return 0;
}

// device result of a plan holding only some workers (slice-major) -> their
// natural-order host positions (natural-order and bit-reversed plans copy
// straight into host_out, pifft_execute_group)
void scatter_to_host(const pifft_plan* p, const char* res, char* host_out) {
    const size_t esz = p->esz;
    const uint64_t M = p->m;
    // a plan holding only some workers: its bins go to their stride-P
    // natural-order positions (other positions untouched, CPU.c:496-499).
    // host_out is a plain C buffer (a double _Complex / float _Complex array is
    // only 8- / 4-byte aligned): element-sized memcpy, which the compiler
    // lowers to plain moves without assuming cx<T>'s 16- / 8-byte alignment
    for (uint32_t bt = 0; bt < p->batch; bt++) {
        for (uint32_t q = p->q0; q < p->q0 + p->nq; q++) {
            const uint64_t r = bitrev(q, p->lp);
            const char* s = res + ((uint64_t)bt * p->nq * M + (uint64_t)(q - p->q0) * M) * esz;
            char* d = host_out + ((uint64_t)bt * p->n + r) * esz;
            const uint64_t dstride = (uint64_t)p->P * esz;
            if (esz == 16)
                for (uint64_t k = 0; k < M; k++) memcpy(d + k * dstride, s + k * 16, 16);
            else
                for (uint64_t k = 0; k < M; k++) memcpy(d + k * dstride, s + k * 8, 8);
        }
    }
}

int ensure_host_staging(pifft_plan* p) {
    if (!p->d_hin) HIPCHK(hipMalloc(&p->d_hin, (size_t)p->batch * p->n * p->esz));
    if (!p->d_hout) HIPCHK(hipMalloc(&p->d_hout, (size_t)out_elems(p) * p->esz));
    return 0;
}

int launch_interleave(const void* d_slices, void* d_out, uint64_t n, uint32_t workers, uint32_t batch, int prec,
                      hipStream_t st) {
    if (prec != PIFFT_F64 && prec != PIFFT_F32) return fail("bad precision");
    uint64_t total = (uint64_t)batch * n;
    const int lp = ilog2u(workers);
    uint32_t ln = (uint32_t)ilog2u(n), lpp = (uint32_t)lp;
    const void* in = d_slices;
    void* o = d_out;
    void* args[] = {&in, &o, &total, &ln, &lpp};
    HIPCHK(hipLaunchKernel(interleave_fn(prec, lp, n), dim3(stride_grid(interleave_threads(total, lp, prec, n))),
                           dim3(256), args, 0, st));
    return 0;
}

// The plans' worker ranges cover [0, P) exactly once, every plan slice-major
// (PIFFT_OUT_SLICES) with the same n, P, batch and precision.
int check_cover(pifft_plan* const* plans, int np, bool quiet) {
    if (!plans || np <= 0) return quiet ? -1 : fail("no plans");
    std::vector<int> order;
    for (int i = 0; i < np; i++) {
        const pifft_plan* p = plans[i];
        if (!p) return quiet ? -1 : fail("plan %d is NULL", i);
        if (p->n != plans[0]->n || p->P != plans[0]->P || p->batch != plans[0]->batch || p->prec != plans[0]->prec)
            return quiet ? -1 : fail("plans of a gather must share n, workers, batch and precision");
        if (p->natural || p->bitrev)
            return quiet ? -1 : fail("plan %d: a gather needs slice-major plans (PIFFT_OUT_SLICES)", i);
        order.push_back(i);
    }
    std::sort(order.begin(), order.end(), [&](int a, int b) { return plans[a]->q0 < plans[b]->q0; });
    uint64_t next = 0;
    for (int i : order) {
        if (plans[i]->q0 != next) break;
        next += plans[i]->nq;
    }
    if (next != plans[0]->P)
        return quiet ? -1 : fail("the plans' worker ranges must cover workers [0, %u) exactly once", plans[0]->P);
    return 0;
}

// peer access from plan d's device to `src_dev` (xGMI loads/copies without a
// host bounce); a pair that cannot peer still copies, staged by the runtime
int enable_peer(pifft_plan* d, int src_dev) {
    if (fault_at("enable_peer"))
        return fail("hipDeviceEnablePeerAccess(%d -> %d): injected fault (PIFFT_FAULT=enable_peer)", d->device, src_dev);
    if (src_dev == d->device) return 0;
    for (int e : d->peer_on)
        if (e == src_dev) return 0;
    int can = 0;
    HIPCHK(hipDeviceCanAccessPeer(&can, d->device, src_dev));
    if (can) {
        const hipError_t e = hipDeviceEnablePeerAccess(src_dev, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
            return fail("hipDeviceEnablePeerAccess(%d -> %d): %s", d->device, src_dev, hipGetErrorString(e));
        (void)hipGetLastError();  // clear a sticky "already enabled"
    }
    d->peer_on.push_back(src_dev);
    return 0;
}

// The optional final exchange: on every destination j with
// d_natural[j] != NULL, copy each plan's slices into the plan-owned gather
// buffer of j's device (hipMemcpyPeerAsync over xGMI, one copy stream per
// source so the links run concurrently), then interleave them into natural
// order (k_interleave).  Synchronous; *ms = the slowest destination's time.
int gather_group(pifft_plan* const* plans, int np, const void* const* d_slices, void* const* d_natural, double* ms) {
    if (check_cover(plans, np, false)) return -1;
    if (!d_slices || !d_natural) return fail("NULL buffer list");
    for (int i = 0; i < np; i++)
        if (!d_slices[i]) return fail("d_slices[%d] is NULL", i);
    const pifft_plan* p0 = plans[0];
    const uint64_t N = p0->n, M = p0->m;
    const size_t esz = p0->esz;
    // every destination is written (interleave) while other destinations'
    // copy streams may still read the sources: no destination may overlap
    // any source buffer (or another destination)
    auto overlap = [](const void* a, size_t na, const void* b, size_t nb) {
        const char *x = (const char*)a, *y = (const char*)b;
        return x < y + nb && y < x + na;
    };
    const size_t nat_bytes = (size_t)p0->batch * N * esz;
    for (int j = 0; j < np; j++) {
        if (!d_natural[j]) continue;
        for (int i = 0; i < np; i++) {
            const size_t sb = (size_t)out_elems(plans[i]) * esz;
            if (overlap(d_natural[j], nat_bytes, d_slices[i], sb))
                return fail("d_natural[%d] overlaps d_slices[%d]: destinations must be distinct from every source", j, i);
            if (i < j && d_natural[i] && overlap(d_natural[j], nat_bytes, d_natural[i], nat_bytes))
                return fail("d_natural[%d] overlaps d_natural[%d]", j, i);
        }
    }
    // the copy schedule (pifft_gather.h; its multi-device logic is unit-tested on the CPU)
    std::vector<GatherSrc> srcs;
    std::vector<bool> has_dst;
    for (int i = 0; i < np; i++) {
        srcs.push_back({plans[i]->device, plans[i]->q0, plans[i]->nq});
        has_dst.push_back(d_natural[i] != nullptr);
    }
    const GatherSchedule gs = gather_schedule(srcs, has_dst, N, M, p0->batch);
    // one destination's copies + interleave, enqueued (no host wait)
    auto enqueue = [&](int j) -> int {
        pifft_plan* d = plans[j];
        DeviceGuard g(d->device);
        if (!d->d_gather) HIPCHK(hipMalloc(&d->d_gather, (size_t)d->batch * N * esz));
        for (const auto& pr : gs.peer)
            if (pr.first == d->device && enable_peer(d, pr.second)) return -1;
        while ((int)d->gst.size() < gs.streams) {
            hipStream_t st;
            hipEvent_t ev;
            HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            d->gst.push_back(st);
            HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            d->gdone.push_back(ev);
        }
        for (auto& e : d->gev)
            if (!e) HIPCHK(hipEventCreate(&e));
        HIPCHK(hipEventRecord(d->gev[0], d->stream));
        for (int i = 0; i < gs.streams; i++) HIPCHK(hipStreamWaitEvent(d->gst[i], d->gev[0], 0));
        for (const GatherCopy& c : gs.copies) {
            if (c.dst != j) continue;
            const pifft_plan* s = plans[c.src];
            if (fault_at("peer_copy"))
                return fail("hipMemcpyPeerAsync(%d <- %d): injected fault (PIFFT_FAULT=peer_copy)", d->device,
                            s->device);
            HIPCHK(hipMemcpyPeerAsync((char*)d->d_gather + c.dst_off * esz, d->device,
                                      (const char*)d_slices[c.src] + c.src_off * esz, s->device, c.elems * esz,
                                      d->gst[c.stream]));
        }
        for (int i = 0; i < gs.streams; i++) {
            HIPCHK(hipEventRecord(d->gdone[i], d->gst[i]));
            HIPCHK(hipStreamWaitEvent(d->stream, d->gdone[i], 0));
        }
        if (launch_interleave(d->d_gather, d_natural[j], N, d->P, d->batch, d->prec, d->stream)) return -1;
        HIPCHK(hipEventRecord(d->gev[1], d->stream));
        return 0;
    };
    for (int j = 0; j < np; j++) {
        if (!d_natural[j] || !enqueue(j)) continue;
        // a failure part-way: wait for what was already enqueued (copies
        // still reading the caller's slices, or writing a gather buffer)
        // before returning, so the caller may reuse its buffers and the plans
        // stay usable; the first error's message is kept
        const std::string msg = g_err;
        for (int k = 0; k <= j; k++) {
            if (!d_natural[k]) continue;
            DeviceGuard g(plans[k]->device);
            for (auto st : plans[k]->gst) (void)hipStreamSynchronize(st);
            (void)hipStreamSynchronize(plans[k]->stream);
        }
        (void)hipGetLastError();
        g_err = msg;
        return -1;
    }
    double worst = 0.0;
    for (int j = 0; j < np; j++) {
        if (!d_natural[j]) continue;
        pifft_plan* d = plans[j];
        DeviceGuard g(d->device);
        HIPCHK(hipEventSynchronize(d->gev[1]));
        float t = 0.0f;
        HIPCHK(hipEventElapsedTime(&t, d->gev[0], d->gev[1]));
        worst = std::max(worst, (double)t);
    }
    if (ms) *ms = worst;
    return 0;
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

const char* pifft_last_error(void) { return g_err.c_str(); }

int pifft_abi_version(void) { return PIFFT_ABI_VERSION; }

int pifft_gpu_count(void) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        fail("hipGetDeviceCount: %s", hipGetErrorString(e));
        return -1;
    }
    return n;
}

int pifft_plan_create(pifft_plan** plan, uint64_t n, uint32_t workers, uint32_t batch, int prec) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    return create(plan, n, workers, 0, workers, batch, prec, dev, PIFFT_OUT_NATURAL);
}

int pifft_plan_create_slices(pifft_plan** plan, uint64_t n, uint32_t workers, uint32_t first,
                             uint32_t count, uint32_t batch, int prec, int device, int flags) {
    return create(plan, n, workers, first, count, batch, prec, device, flags);
}

void pifft_plan_destroy(pifft_plan* plan) { release(plan); }

int pifft_plan_dry_run(uint64_t n, uint32_t workers, uint32_t first, uint32_t count, uint32_t batch, int prec,
                       int flags, pifft_plan_info* info) {
    if (!info) return fail("info is NULL");
    pifft_plan* p = nullptr;
    if (create(&p, n, workers, first, count, batch, prec, -1, flags, true)) return -1;
    const int rc = pifft_plan_get_info(p, info);
    release(p);
    return rc;
}

int pifft_instance_count(void) { return (int)pass_kernels().size(); }

int pifft_instance_desc(int i, int32_t* desc) {
    if (!desc) return fail("desc is NULL");
    if (i < 0 || i >= (int)pass_kernels().size()) return fail("instance %d out of range", i);
    const PassKernel& k = pass_kernels()[(size_t)i];
    const int32_t d[7] = {k.prec, k.R, k.C, k.mode, k.nts, k.lp, k.vpt};
    memcpy(desc, d, sizeof d);
    return 0;
}

int pifft_instance_found(int i) {
    if (i < 0 || i >= (int)pass_kernels().size()) return fail("instance %d out of range", i);
    return found_log()[(size_t)i].load(std::memory_order_relaxed);
}

int pifft_plan_dry_run_instances(uint64_t n, uint32_t workers, uint32_t first, uint32_t count, uint32_t batch,
                                 int prec, int flags, int32_t* ids, int max_ids) {
    if (!ids && max_ids > 0) return fail("ids is NULL");
    pifft_plan* p = nullptr;
    if (create(&p, n, workers, first, count, batch, prec, -1, flags, true)) return -1;
    const int nl = (int)p->steps.size();
    const PassKernel* base = pass_kernels().data();
    for (int i = 0; i < nl && i < max_ids; i++) {
        const PassKernel* k = p->steps[(size_t)i].pk;
        ids[i] = k ? (int32_t)(k - base) : -1;
    }
    release(p);
    return nl;
}

int pifft_plan_get_info(const pifft_plan* p, pifft_plan_info* info) {
    if (!p || !info) return fail("NULL argument");
    memset(info, 0, sizeof *info);
    info->n = p->n;
    info->workers = p->P;
    info->first_worker = p->q0;
    info->num_workers = p->nq;
    info->batch = p->batch;
    info->prec = p->prec;
    info->device = p->device;
    info->flags = p->flags;
    info->local_n = p->m;
    info->in_elems = (uint64_t)p->batch * p->n;
    info->out_elems = out_elems(p);
    info->workspace_bytes = p->bytes_w + p->bytes_ta + p->tw_bytes;
    info->layout = (p->wil ? 1 : 0) | (p->ilv ? 2 : 0);
    info->num_launches = (int)p->steps.size();
    info->num_passes = p->npasses;
    info->tree_launches = p->tree_steps;
    for (int i = 0; i < 8; i++) {
        info->radix[i] = p->radix[i];
        info->lines[i] = p->lines[i];
        info->vpt[i] = p->vpt[i];
    }
    std::vector<const void*> fns;
    for (size_t i = 0; i < p->steps.size() && i < PIFFT_MAX_LAUNCH_INFO; i++) {
        info->launch_bytes[i] = p->steps[i].bytes;
        info->launch_kind[i] = p->steps[i].kind;
        size_t f = 0;
        while (f < fns.size() && fns[f] != p->steps[i].fn) f++;
        if (f == fns.size()) fns.push_back(p->steps[i].fn);
        info->launch_fn[i] = (int32_t)f;
        info->launch_mode[i] = p->steps[i].pk ? p->steps[i].pk->mode : 0;
    }
    return 0;
}

int pifft_plan_kernel_name(const pifft_plan* p, int launch, char* buf, size_t len) {
    if (!p || !buf || len == 0) return fail("NULL argument");
    if (launch < 0 || launch >= (int)p->steps.size()) return fail("launch %d out of range", launch);
    DeviceGuard g(p->device);
    const char* mangled = hipKernelNameRefByPtr(p->steps[(size_t)launch].fn, nullptr);
    if (!mangled) return fail("no kernel name for launch %d", launch);
    int st = 0;
    char* dem = abi::__cxa_demangle(mangled, nullptr, nullptr, &st);
    snprintf(buf, len, "%s", (st == 0 && dem) ? dem : mangled);
    free(dem);
    return 0;
}

// the launch an execution of a PIFFT_PROFILE_SAMPLED run times (or -1):
// odd executions time one launch each, round robin, so every timed dispatch
// follows an untimed one (a timed dispatch delays the next one by ~9 us and
// would isolate it)
int sampled_launch(int k, size_t ns) { return (k & 1) ? (int)(((size_t)k >> 1) % ns) : -1; }

int pifft_execute_device(pifft_plan* p, const void* d_in, void* d_out, void* stream) {
    if (check_buffers(p, d_in, d_out)) return -1;
    DeviceGuard g(p->device);
    hipStream_t st = (hipStream_t)stream;  // NULL = the default stream
    const size_t ns = p->steps.size();
    if (p->prof_used >= p->prof_steps) return launch_steps(p, d_in, d_out, st, nullptr);
    const int k = p->prof_used++;
    if (p->prof_mode == PIFFT_PROFILE_ALL) return launch_steps(p, d_in, d_out, st, &p->prof_ev[(size_t)k * 2 * ns]);
    const int li = sampled_launch(k, ns);
    for (size_t i = 0; i < ns; i++) {
        hipEvent_t* e = (int)i == li ? &p->prof_ev[(size_t)k * 2] : nullptr;
        if (launch_step(p, p->steps[i], d_in, d_out, st, e ? e[0] : nullptr, e ? e[1] : nullptr)) return -1;
    }
    return 0;
}

int pifft_launch_loop(pifft_plan* p, const int* launches, int nlaunches, int reps, const void* d_in, void* d_out,
                      void* stream, float* mean_ms) {
    if (check_buffers(p, d_in, d_out)) return -1;
    if (!launches || nlaunches < 1 || reps < 1 || !mean_ms) return fail("bad arguments");
    for (int j = 0; j < nlaunches; j++)
        if (launches[j] < 0 || (size_t)launches[j] >= p->steps.size())
            return fail("launch %d out of range (plan has %zu)", launches[j], p->steps.size());
    DeviceGuard g(p->device);
    hipStream_t st = (hipStream_t)stream;
    auto rounds = [&](int r) -> int {
        for (int k = 0; k < r; k++)
            for (int j = 0; j < nlaunches; j++)
                if (launch_step(p, p->steps[(size_t)launches[j]], d_in, d_out, st)) return -1;
        return 0;
    };
    // the plan's own event pair, as markers around the loop (p->ev holds >= 2)
    if (rounds(2)) return -1;
    HIPCHK(hipEventRecord(p->ev[0], st));
    if (rounds(reps)) return -1;
    HIPCHK(hipEventRecord(p->ev[1], st));
    if (launch_steps(p, d_in, d_out, st, nullptr)) return -1;  // d_out = the plan's result again
    HIPCHK(hipEventSynchronize(p->ev[1]));
    float ms = 0.0f;
    HIPCHK(hipEventElapsedTime(&ms, p->ev[0], p->ev[1]));
    HIPCHK(hipStreamSynchronize(st));
    *mean_ms = ms / (float)((size_t)reps * (size_t)nlaunches);
    return 0;
}

#ifdef PIFFT_WG_CLOCK
// Diagnostics build only (-DPIFFT_WG_CLOCK, tools/wg_clock.py; not in
// include/pifft.h): `warm` full executions, then launches 0 .. launch-1 as
// usual and `launch` with every workgroup recording its entry and
// stores-done wall clock, hardware id and per-stage stamps
// (PIFFT_WGC_WORDS words per workgroup, PassArgs::wg_clock) into
// host[0 .. min(PIFFT_WGC_WORDS grid, max_words)).  Returns the workgroup count (or -1);
// *wall_hz = the wall clock's rate.  Synchronous.
int pifft_debug_wg_clock(pifft_plan* p, int launch, const void* d_in, void* d_out, void* stream, int warm,
                         unsigned long long* host, size_t max_words, unsigned long long* wall_hz) {
    if (check_buffers(p, d_in, d_out)) return -1;
    if (launch < 0 || (size_t)launch >= p->steps.size()) return fail("launch %d out of range", launch);
    const Step& s = p->steps[(size_t)launch];
    if (s.kind != STEP_PASS && s.kind != STEP_TREE_PASS) return fail("launch %d is not a pass", launch);
    DeviceGuard g(p->device);
    hipStream_t st = (hipStream_t)stream;
    const size_t nwg = (size_t)s.grid.x * s.grid.y * s.grid.z, words = PIFFT_WGC_WORDS * nwg;
    unsigned long long* clk = nullptr;
    HIPCHK(hipMalloc(&clk, words * sizeof(unsigned long long)));
    HIPCHK(hipMemset(clk, 0, words * sizeof(unsigned long long)));  // (stamps a pass does not reach stay 0)
    int rc = 0;
    for (int k = 0; k < warm && rc == 0; k++) rc = launch_steps(p, d_in, d_out, st, nullptr);
    for (int i = 0; i < launch && rc == 0; i++) rc = launch_step(p, p->steps[(size_t)i], d_in, d_out, st);
    if (rc == 0) {
        p->dbg_clk = clk;
        rc = launch_step(p, s, d_in, d_out, st);
        p->dbg_clk = nullptr;
    }
    if (rc == 0 && hipStreamSynchronize(st) != hipSuccess) rc = fail("hipStreamSynchronize failed");
    if (rc == 0 && hipMemcpy(host, clk, std::min(words, max_words) * sizeof(unsigned long long),
                             hipMemcpyDeviceToHost) != hipSuccess)
        rc = fail("hipMemcpy failed");
    int khz = 0;
    if (rc == 0 && hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, p->device) != hipSuccess)
        rc = fail("no wall clock rate");
    (void)hipFree(clk);
    if (rc) return -1;
    *wall_hz = (unsigned long long)khz * 1000ull;
    return (int)nwg;
}
#endif

int pifft_plan_tune_workspace(pifft_plan* p, const void* d_in, void* d_out, void* stream, int tries,
                              float* best_ms) {
    if (check_buffers(p, d_in, d_out)) return -1;
    if (tries < 1) return fail("tries must be >= 1");
    DeviceGuard g(p->device);
    hipStream_t st = (hipStream_t)stream;
    if (!p->buf[BUF_W] || tries == 1) {  // nothing to place
        if (best_ms) *best_ms = 0.0f;
        return 0;
    }
    hipEvent_t e[2];
    HIPCHK(hipEventCreateWithFlags(&e[0], kTimingEventFlags));
    if (hipEventCreateWithFlags(&e[1], kTimingEventFlags) != hipSuccess) {
        (void)hipEventDestroy(e[0]);
        return fail("hipEventCreate failed");
    }
    // mean of 3 executions after one warm-up, with the plan's current workspace
    auto timed = [&](float& ms) -> int {
        if (launch_steps(p, d_in, d_out, st, nullptr)) return -1;
        HIPCHK(hipEventRecord(e[0], st));
        for (int r = 0; r < 3; r++)
            if (launch_steps(p, d_in, d_out, st, nullptr)) return -1;
        HIPCHK(hipEventRecord(e[1], st));
        HIPCHK(hipEventSynchronize(e[1]));
        HIPCHK(hipEventElapsedTime(&ms, e[0], e[1]));
        ms /= 3.0f;
        return 0;
    };
    int rc = 0;
    float best = 0.0f;
    if (timed(best)) rc = -1;
    // every losing workspace stays allocated until the end, so each try lands
    // somewhere new (a freed range would come straight back from hipMalloc)
    std::vector<void*> losers;
    for (int t = 1; t < tries && rc == 0; t++) {
        void* keep = p->buf[BUF_W];
        void* fresh = nullptr;
        // the losers stay allocated until the end: try only while the device
        // keeps room for another workspace and 4 GiB beyond this one (other
        // processes on the GPU, e.g. bench.py's same-device rehearsal ranks,
        // allocate concurrently)
        size_t mfree = 0, mtotal = 0;
        if (hipMemGetInfo(&mfree, &mtotal) != hipSuccess || mfree < 2 * p->bytes_w + (4ull << 30)) {
            (void)hipGetLastError();
            break;
        }
        if (hipMalloc(&fresh, p->bytes_w) != hipSuccess) {
            (void)hipGetLastError();
            break;  // no room for another workspace: keep the best so far
        }
        p->buf[BUF_W] = fresh;
        float ms = 0.0f;
        if (timed(ms)) {
            rc = -1;
            p->buf[BUF_W] = keep;
            losers.push_back(fresh);
        } else if (ms < best) {
            best = ms;
            losers.push_back(keep);
        } else {
            p->buf[BUF_W] = keep;
            losers.push_back(fresh);
        }
    }
    (void)hipStreamSynchronize(st);
    for (void* w : losers) (void)hipFree(w);
    (void)hipEventDestroy(e[0]);
    (void)hipEventDestroy(e[1]);
    if (best_ms) *best_ms = best;
    return rc;
}

int pifft_profile_start(pifft_plan* p, int steps, int mode) {
    if (!p || steps < 0) return fail("bad arguments");
    if (mode != PIFFT_PROFILE_ALL && mode != PIFFT_PROFILE_SAMPLED) return fail("unknown profile mode %d", mode);
    DeviceGuard g(p->device);
    const size_t need = (size_t)steps * 2 * (mode == PIFFT_PROFILE_ALL ? p->steps.size() : 1);
    while (p->prof_ev.size() < need) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, kTimingEventFlags));
        p->prof_ev.push_back(e);
    }
    p->prof_steps = steps;
    p->prof_used = 0;
    p->prof_mode = mode;
    return 0;
}

int pifft_profile_read(pifft_plan* p, float* launch_ms_sum, int* launch_samples, int max_launches) {
    if (!p) return fail("plan is NULL");
    DeviceGuard g(p->device);
    const size_t ns = p->steps.size();
    const int used = p->prof_used;
    p->prof_steps = p->prof_used = 0;  // profiling stops, also on an error below
    std::vector<float> sum(ns, 0.0f), ms;
    std::vector<int> cnt(ns, 0);
    for (int k = 0; k < used; k++) {
        // each execution's own events: the executions may have run on different streams
        if (p->prof_mode == PIFFT_PROFILE_ALL) {
            if (read_launch_ms(ns, &p->prof_ev[(size_t)k * 2 * ns], ms)) return -1;
            for (size_t i = 0; i < ns; i++) sum[i] += ms[i], cnt[i]++;
        } else {
            const int li = sampled_launch(k, ns);
            if (li < 0) continue;
            hipEvent_t* e = &p->prof_ev[(size_t)k * 2];
            float t = 0.0f;
            HIPCHK(hipEventSynchronize(e[1]));
            HIPCHK(hipEventElapsedTime(&t, e[0], e[1]));
            sum[(size_t)li] += t;
            cnt[(size_t)li]++;
        }
    }
    for (int i = 0; i < max_launches && i < (int)ns; i++) {
        if (launch_ms_sum) launch_ms_sum[i] = sum[(size_t)i];
        if (launch_samples) launch_samples[i] = cnt[(size_t)i];
    }
    return used;
}

int pifft_execute_device_timed(pifft_plan* p, const void* d_in, void* d_out, void* stream,
                               float* launch_ms, int max_launches) {
    if (check_buffers(p, d_in, d_out)) return -1;
    DeviceGuard g(p->device);
    hipStream_t st = (hipStream_t)stream;  // NULL = the default stream
    std::vector<float> ms;
    if (run_timed(p, d_in, d_out, st, ms)) return -1;
    // (fence-free timing events: the output is complete and visible once the
    // stream itself has drained)
    HIPCHK(hipStreamSynchronize(st));
    if (launch_ms)
        for (int i = 0; i < max_launches && i < (int)ms.size(); i++) launch_ms[i] = ms[i];
    return 0;
}

int pifft_execute(pifft_plan* p, const void* host_in, void* host_out, double* ms1, double* ms2) {
    return pifft_execute_group(&p, 1, host_in, host_out, ms1, ms2);
}

int pifft_execute_group(pifft_plan** plans, int np, const void* host_in, void* host_out,
                        double* ms1, double* ms2) {
    if (!plans || np <= 0) return fail("no plans");
    if (!host_in) return fail("host_in is NULL");
    for (int i = 0; i < np; i++) {
        if (!plans[i]) return fail("plan %d is NULL", i);
        if (plans[i]->n != plans[0]->n || plans[i]->batch != plans[0]->batch ||
            plans[i]->prec != plans[0]->prec)
            return fail("plans of a group must share n, batch and precision");
    }
    // stage the input on every device (outside the timed region, like the
    // reference's per-worker memcpy of the whole input, CPU.c:407): one copy
    // over PCIe to the first plan's device, then a broadcast device to device
    // (hipMemcpyPeerAsync over xGMI, all destinations concurrently) instead
    // of one PCIe copy per GPU
    const size_t in_bytes = (size_t)plans[0]->batch * plans[0]->n * plans[0]->esz;
    {
        pifft_plan* p0 = plans[0];
        DeviceGuard g(p0->device);
        if (ensure_host_staging(p0)) return -1;
        HIPCHK(hipMemcpyAsync(p0->d_hin, host_in, in_bytes, hipMemcpyHostToDevice, p0->stream));
        HIPCHK(hipStreamSynchronize(p0->stream));
    }
    // (a failure part-way waits for the broadcast copies already enqueued --
    // they read plans[0]'s staging buffer, which the next call overwrites)
    auto broadcast = [&](int i) -> int {
        pifft_plan* p = plans[i];
        DeviceGuard g(p->device);
        if (ensure_host_staging(p)) return -1;
        if (enable_peer(p, plans[0]->device)) return -1;
        if (fault_at("broadcast"))
            return fail("hipMemcpyPeerAsync(%d <- %d): injected fault (PIFFT_FAULT=broadcast)", p->device,
                        plans[0]->device);
        HIPCHK(hipMemcpyPeerAsync(p->d_hin, p->device, plans[0]->d_hin, plans[0]->device, in_bytes, p->stream));
        return 0;
    };
    for (int i = 1; i < np; i++) {
        if (!broadcast(i)) continue;
        const std::string msg = g_err;
        for (int k = 1; k < i; k++) {
            DeviceGuard g(plans[k]->device);
            (void)hipStreamSynchronize(plans[k]->stream);
        }
        (void)hipGetLastError();
        g_err = msg;
        return -1;
    }
    for (int i = 1; i < np; i++) {
        DeviceGuard g(plans[i]->device);
        HIPCHK(hipStreamSynchronize(plans[i]->stream));
    }
    // launch all GPUs, then wait for all (stage markers: wall time per stage)
    for (int i = 0; i < np; i++) {
        pifft_plan* p = plans[i];
        DeviceGuard g(p->device);
        if (launch_stage_marked(p, p->d_hin, p->d_hout)) return -1;
    }
    double t1 = 0, t2 = 0;
    for (int i = 0; i < np; i++) {
        pifft_plan* p = plans[i];
        DeviceGuard g(p->device);
        double a, b;
        if (read_stage_marked(p, &a, &b)) return -1;
        // the timing events skip the system-scope fence: the stream itself is
        // waited for before anything reads the result on the host
        HIPCHK(hipStreamSynchronize(p->stream));
        if (a + b > t1 + t2) {  // the slowest GPU sets the job's time
            t1 = a;
            t2 = b;
        }
    }
    if (ms1) *ms1 = t1;
    if (ms2) *ms2 = t2;
    if (host_out) {
        if (np > 1 && check_cover(plans, np, true) == 0) {
            // the whole transform over several plans: gather on the first
            // plan's device (pifft_allgather) into a result buffer held for
            // this call only -- not the input staging copy, which
            // pifft_execute_group_kernel_times re-runs the plans on, and not
            // a persistent one (it would add N to the first device's
            // footprint for the plan's life) -- and copy back once
            pifft_plan* p = plans[0];
            const size_t nat_bytes = (size_t)p->batch * p->n * p->esz;
            void* d_nat = nullptr;
            {
                DeviceGuard g(p->device);
                HIPCHK(hipMalloc(&d_nat, nat_bytes));
            }
            std::vector<const void*> sl(np);
            std::vector<void*> nat(np, nullptr);
            for (int i = 0; i < np; i++) sl[i] = plans[i]->d_hout;
            nat[0] = d_nat;
            int rc = gather_group(plans, np, sl.data(), nat.data(), nullptr);
            DeviceGuard g(p->device);
            if (rc == 0) {
                const hipError_t e = hipMemcpy(host_out, d_nat, nat_bytes, hipMemcpyDeviceToHost);
                if (e != hipSuccess) rc = fail("hipMemcpy of the gathered result: %s", hipGetErrorString(e));
            }
            (void)hipFree(d_nat);  // (synchronizes: no gather copy still writes it)
            return rc;
        }
        for (int i = 0; i < np; i++) {
            pifft_plan* p = plans[i];
            DeviceGuard g(p->device);
            // natural order, and the reference's scratch order (whole segments),
            // land in host_out as they are: straight device-to-host copies (no
            // host-side staging copy: that single-threaded 4 GiB memcpy was half
            // of a 2^28 fp64 call, profiles/r02_host_boundary.log)
            if (p->natural) {
                HIPCHK(hipMemcpy(host_out, p->d_hout, (size_t)p->batch * p->n * p->esz, hipMemcpyDeviceToHost));
                continue;
            }
            if (p->bitrev) {
                const uint64_t M = p->m;
                for (uint32_t bt = 0; bt < p->batch; bt++)
                    HIPCHK(hipMemcpy((char*)host_out + ((uint64_t)bt * p->n + (uint64_t)p->q0 * M) * p->esz,
                                     (const char*)p->d_hout + (uint64_t)bt * p->nq * M * p->esz,
                                     (size_t)p->nq * M * p->esz, hipMemcpyDeviceToHost));
                continue;
            }
            const size_t bytes = (size_t)out_elems(p) * p->esz;
            p->host_tmp.resize(bytes);
            HIPCHK(hipMemcpy(p->host_tmp.data(), p->d_hout, bytes, hipMemcpyDeviceToHost));
            scatter_to_host(p, p->host_tmp.data(), (char*)host_out);
        }
    }
    return 0;
}

int pifft_execute_group_kernel_times(pifft_plan** plans, int np, double* ms1, double* ms2) {
    if (!plans || np <= 0) return fail("no plans");
    for (int i = 0; i < np; i++) {
        if (!plans[i]) return fail("plan %d is NULL", i);
        if (!plans[i]->d_hin || !plans[i]->d_hout) return fail("plan %d: no staged input (call pifft_execute_group first)", i);
    }
    for (int i = 0; i < np; i++) {
        pifft_plan* p = plans[i];
        DeviceGuard g(p->device);
        if (launch_steps(p, p->d_hin, p->d_hout, p->stream, p->ev.data())) return -1;
    }
    double t1 = 0, t2 = 0;
    for (int i = 0; i < np; i++) {
        pifft_plan* p = plans[i];
        DeviceGuard g(p->device);
        std::vector<float> ms;
        if (read_launch_ms(p->steps.size(), p->ev.data(), ms)) return -1;
        HIPCHK(hipStreamSynchronize(p->stream));
        double a, b;
        stage_split(p, ms, &a, &b);
        if (a + b > t1 + t2) {
            t1 = a;
            t2 = b;
        }
    }
    if (ms1) *ms1 = t1;
    if (ms2) *ms2 = t2;
    return 0;
}

int pifft_generate_device(void* d_x, uint64_t count, uint64_t n, uint64_t seed, uint64_t first,
                          int prec, void* stream) {
    if (!d_x) return fail("NULL buffer");
    if (prec != PIFFT_F32 && prec != PIFFT_F64) return fail("bad precision");
    if (count == 0) return 0;
    const double scale = sqrt((double)n);
    const dim3 blk(256), grd(stride_grid(count));
    hipStream_t st = (hipStream_t)stream;
    if (prec == PIFFT_F64)
        hipLaunchKernelGGL(k_generate<double>, grd, blk, 0, st, (cx<double>*)d_x, count, scale, seed, first);
    else
        hipLaunchKernelGGL(k_generate<float>, grd, blk, 0, st, (cx<float>*)d_x, count, scale, seed, first);
    HIPCHK(hipGetLastError());
    return 0;
}

int pifft_interleave_device(const void* d_slices, void* d_out, uint64_t n, uint32_t workers,
                            uint32_t batch, int prec, void* stream) {
    if (!d_slices || !d_out || d_slices == d_out) return fail("bad buffers");
    if (n < 2 || !is_pow2(n) || !workers || !is_pow2(workers) || workers > n) return fail("bad n/workers");
    return launch_interleave(d_slices, d_out, n, workers, batch, prec, (hipStream_t)stream);
}

int pifft_allgather(pifft_plan* const* plans, int nplans, const void* const* d_slices, void* const* d_natural,
                    double* ms) {
    return gather_group(plans, nplans, d_slices, d_natural, ms);
}

int pifft_tree_device(pifft_plan* p, const void* d_in, void* d_seg, void* stream) {
    if (check_buffers(p, d_in, d_seg)) return -1;
    DeviceGuard g(p->device);
    hipStream_t st = (hipStream_t)stream;  // NULL = the default stream
    if (p->tree_only.empty()) {  // P == 1: the segment is the input
        HIPCHK(hipMemcpyAsync(d_seg, d_in, (size_t)p->batch * p->n * p->esz, hipMemcpyDeviceToDevice, st));
        return 0;
    }
    for (const Step& s : p->tree_only)
        if (launch_step(p, s, d_in, d_seg, st)) return -1;
    return 0;
}

}  // extern "C"
