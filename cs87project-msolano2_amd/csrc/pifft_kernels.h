// cs87project-msolano2_amd/csrc/pifft_kernels.h
//
// Hand-written gfx950 (CDNA4) kernels of the MI355X-native pi-FFT.  Device code
// only; the host planner and the C-ABI live in pifft.hip.
//
// The reference computes, per worker q of P, a radix-2 DIF "tree" of log2 P
// half-butterfly stages (CPU.c:419-448) followed by a radix-2 DIF FFT of its
// N/P segment (the "cylinder", CPU.c:463-478), one butterfly per loop step with
// a libm twiddle each (CPU.c:540-576, 644-651).  Here:
//
//  * k_tree   -- the tree stage, one thread per segment element: it loads the P
//               inputs x[i + m*N/P] and evaluates the reference's radix-2 tree
//               in registers in the reference's operation order (add/sub/mul of
//               CPU.c:584-627, no FMA), keeping only the branches that lead to
//               the requested workers.  With the host-built omega(N,k) table
//               (CPU.c:644-651 formula) its output is bit-identical to the
//               reference's post-tree segment.
//               Up to 4 levels per launch; log2 P > 4 takes ceil(log2 P / 4)
//               launches, in place over the reference's scratch layout.
//  * k_pass   -- one Stockham pass of the local N/P-point FFT: each workgroup
//               stages C adjacent "lines" (sub-FFTs of length R, elements
//               strided by M/R in HBM) in LDS, applies the inter-pass twiddle,
//               runs the R-point FFT as radix-16 (plus one radix-2/4/8) stages
//               with twiddles from a table, and writes the lines in Stockham
//               (auto-sort) order.  Loads/stores are 16 B per lane for fp64 and
//               coalesced across the C adjacent lines.
//  * k_interleave -- slice-major worker outputs -> natural order.
//  * k_generate   -- the synthetic splitmix64 input.
//
// Compile with -ffp-contract=off: the tree's bitwise parity with the
// reference depends on every product and sum being rounded separately.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace pifft {

template <typename T>
struct alignas(2 * sizeof(T)) cx {
    T re, im;
};

template <typename T>
__device__ __forceinline__ cx<T> cadd(cx<T> a, cx<T> b) {
    return {a.re + b.re, a.im + b.im};
}
template <typename T>
__device__ __forceinline__ cx<T> csub(cx<T> a, cx<T> b) {
    return {a.re - b.re, a.im - b.im};
}
// CPU.c:620-627 order: re = ar*br - ai*bi, im = ar*bi + ai*br
template <typename T>
__device__ __forceinline__ cx<T> cmul(cx<T> a, cx<T> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
// a * (-i)
template <typename T>
__device__ __forceinline__ cx<T> mul_negi(cx<T> a) {
    return {a.im, -a.re};
}

constexpr int ilog2c(uint64_t x) { return x <= 1 ? 0 : 1 + ilog2c(x >> 1); }

// ---------------------------------------------------------------------------
// Small forward DFTs in registers (natural order in and out), omega = e^{-2 pi i/q}
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void dft4(cx<T>& a0, cx<T>& a1, cx<T>& a2, cx<T>& a3) {
    cx<T> t0 = cadd(a0, a2), t1 = csub(a0, a2);
    cx<T> t2 = cadd(a1, a3), t3 = mul_negi(csub(a1, a3));
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    a1 = cadd(t1, t3);
    a3 = csub(t1, t3);
}

template <typename T>
__device__ __forceinline__ void dft8(cx<T>* v) {
    const T s = (T)0.70710678118654752440084436210484903928L;
    cx<T> e0 = v[0], e1 = v[2], e2 = v[4], e3 = v[6];
    cx<T> o0 = v[1], o1 = v[3], o2 = v[5], o3 = v[7];
    dft4(e0, e1, e2, e3);
    dft4(o0, o1, o2, o3);
    o1 = {(o1.re + o1.im) * s, (o1.im - o1.re) * s};   // * w8^1 = (s, -s)
    o2 = mul_negi(o2);                                 // * w8^2 = -i
    o3 = {(o3.im - o3.re) * s, -((o3.re + o3.im) * s)}; // * w8^3 = (-s, -s)
    v[0] = cadd(e0, o0);
    v[4] = csub(e0, o0);
    v[1] = cadd(e1, o1);
    v[5] = csub(e1, o1);
    v[2] = cadd(e2, o2);
    v[6] = csub(e2, o2);
    v[3] = cadd(e3, o3);
    v[7] = csub(e3, o3);
}

template <typename T>
__device__ __forceinline__ void dft16(cx<T>* v) {
    const T c1 = (T)0.92387953251128675612818318939678828682L;  // cos(pi/8)
    const T s1 = (T)0.38268343236508977172845998403039886676L;  // sin(pi/8)
    const T s = (T)0.70710678118654752440084436210484903928L;
    // n = 4 n1 + n2, k = k1 + 4 k2.  Column DFT4s over n1.
#pragma unroll
    for (int n2 = 0; n2 < 4; n2++) dft4(v[n2], v[4 + n2], v[8 + n2], v[12 + n2]);
    // v[4 k1 + n2] *= w16^(n2 k1)
    const cx<T> w1 = {c1, -s1}, w2 = {s, -s}, w3 = {s1, -c1}, w6 = {-s, -s}, w9 = {-c1, s1};
    v[5] = cmul(v[5], w1);
    v[6] = cmul(v[6], w2);
    v[7] = cmul(v[7], w3);
    v[9] = cmul(v[9], w2);
    v[10] = mul_negi(v[10]);
    v[11] = cmul(v[11], w6);
    v[13] = cmul(v[13], w3);
    v[14] = cmul(v[14], w6);
    v[15] = cmul(v[15], w9);
    // row DFT4s over n2
#pragma unroll
    for (int k1 = 0; k1 < 4; k1++) dft4(v[4 * k1], v[4 * k1 + 1], v[4 * k1 + 2], v[4 * k1 + 3]);
    // v[4 k1 + k2] = X[k1 + 4 k2]: transpose the 4x4 (register renaming)
    cx<T> t;
#define PIFFT_SWP(a, b) t = v[a], v[a] = v[b], v[b] = t
    PIFFT_SWP(1, 4);
    PIFFT_SWP(2, 8);
    PIFFT_SWP(3, 12);
    PIFFT_SWP(6, 9);
    PIFFT_SWP(7, 13);
    PIFFT_SWP(11, 14);
#undef PIFFT_SWP
}

template <int Q, typename T>
__device__ __forceinline__ void dft(cx<T>* v) {
    if constexpr (Q == 1) {
    } else if constexpr (Q == 2) {
        cx<T> a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    } else if constexpr (Q == 4) {
        dft4(v[0], v[1], v[2], v[3]);
    } else if constexpr (Q == 8) {
        dft8(v);
    } else {
        static_assert(Q == 16, "radix");
        dft16(v);
    }
}

// streamed data: each element is read once and written once per pass.  NTS
// selects non-temporal (nt) loads/stores for it -- a win when a pass streams
// more than the 256 MiB Infinity Cache holds, a loss when the data would
// otherwise stay resident there (measured).
#ifndef PIFFT_NT_LOADS
#define PIFFT_NT_LOADS 1  // build-time switches for A/B variants (tools/mkvariant.sh)
#endif
#ifndef PIFFT_NT_STORES
#define PIFFT_NT_STORES 1
#endif
// NTS (k_pass template argument): 0 plain; 1 nt loads and stores
constexpr bool nt_loads(int nt) { return nt == 1; }
constexpr bool nt_stores(int nt) { return nt == 1; }
// PIFFT_VEC_NT: a complex value moves as ONE 8- or 16-byte vector access
// (1: both precisions, 2: fp32 only, 0: two scalar nt accesses, which the
// compiler merges -- for fp32 into loads that waited on each other).
// Measured on MI355X (profiles/r03_ab_kernel_forms.log): fp32 2^28 3.23 ->
// 3.04 ms with 2 (the same with 1); fp64 2^28 within the box's +-2 % spread
// either way, so fp64 keeps its round-2 code (2).
#ifndef PIFFT_VEC_NT
#define PIFFT_VEC_NT 2
#endif
template <typename T>
using vec2_t = T __attribute__((ext_vector_type(2)));
template <typename T>
constexpr bool vec_nt() {
    return PIFFT_VEC_NT == 1 || (PIFFT_VEC_NT == 2 && sizeof(T) == 4);
}
template <bool NTS, typename T>
__device__ __forceinline__ cx<T> ld_stream(const cx<T>* p) {
    if constexpr (NTS && PIFFT_NT_LOADS && vec_nt<T>()) {
        const vec2_t<T> r = __builtin_nontemporal_load(reinterpret_cast<const vec2_t<T>*>(p));
        return cx<T>{r.x, r.y};
    } else if constexpr (NTS && PIFFT_NT_LOADS) {
        cx<T> r;
        r.re = __builtin_nontemporal_load(&p->re);
        r.im = __builtin_nontemporal_load(&p->im);
        return r;
    } else {
        return *p;
    }
}
template <bool NTS, typename T>
__device__ __forceinline__ void st_stream(cx<T>* p, cx<T> v) {
    if constexpr (NTS && PIFFT_NT_STORES && vec_nt<T>()) {
        vec2_t<T> r;
        r.x = v.re;
        r.y = v.im;
        __builtin_nontemporal_store(r, reinterpret_cast<vec2_t<T>*>(p));
    } else if constexpr (NTS && PIFFT_NT_STORES) {
        __builtin_nontemporal_store(v.re, &p->re);
        __builtin_nontemporal_store(v.im, &p->im);
    } else {
        *p = v;
    }
}
// PIFFT_CLAMP_LOADS: a partial last tile's idle lanes load the last line again
// (unconditional loads, no per-load branch; 1: both precisions, 2: fp32 only)
// instead of skipping their loads (same measurements: fp32 only, 2)
#ifndef PIFFT_CLAMP_LOADS
#define PIFFT_CLAMP_LOADS 2
#endif
template <typename T>
constexpr bool clamp_loads() {
    return PIFFT_CLAMP_LOADS == 1 || (PIFFT_CLAMP_LOADS == 2 && sizeof(T) == 4);
}

// two-level twiddle: w_M^E = hi[E >> h] * lo[E & (2^h - 1)]
template <typename T>
__device__ __forceinline__ cx<T> tw2(const cx<T>* __restrict__ lo, const cx<T>* __restrict__ hi,
                                     uint32_t h, uint64_t E) {
    const cx<T> a = lo[E & ((1ull << h) - 1)];
    const cx<T> b = hi[E >> h];
    return cmul(b, a);
}

// w_NS^e = (cos 2 pi e/NS, -sin 2 pi e/NS), e < NS, evaluated at compile time
// (Taylor series on the first quadrant, then the quadrant's exact rotation)
template <int NS>
struct RootsOf {
    double re[NS], im[NS];
    constexpr RootsOf() : re(), im() {
        constexpr double two_pi = 6.283185307179586476925286766559;
        for (int e = 0; e < NS; e++) {
            const int quad = (4 * e) / NS, r = e - quad * (NS / 4);
            const double x = two_pi * r / NS;  // [0, pi/2)
            double c = 1, s = x, tc = 1, ts = x;
            for (int i = 1; i < 16; i++) {
                tc *= -x * x / ((2 * i - 1) * (2 * i));
                ts *= -x * x / ((2 * i) * (2 * i + 1));
                c += tc;
                s += ts;
            }
            const double cq = quad == 0 ? c : quad == 1 ? -s : quad == 2 ? -c : s;
            const double sq = quad == 0 ? s : quad == 1 ? c : quad == 2 ? -s : -c;
            re[e] = cq;
            im[e] = -sq;
        }
    }
};

// for (I = B; I < E; I += S) f(integral_constant<I>) -- compile-time indices
template <int B, int E, int S, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + S, E, S>(f);
    }
}

// ---------------------------------------------------------------------------
// Tree ("funnel") network, shared by k_tree and the fused first pass
// ---------------------------------------------------------------------------
struct TreeTw {
    // The reference formula omega(N, e) (CPU.c:644-651), packed by tree level:
    // level t's entries omega(N, k 2^t), k < N >> (t+1), sit contiguously at
    // N - (N >> t) + k, so a level's lookups i, i+1, ... read consecutive
    // entries (a single N/2 table read at e = k 2^t touches a whole line per
    // 2^-t of its entries); or null
    const void* direct;
    const void* lo;      // else two-level w_N
    const void* hi;
    uint32_t h;
    uint32_t log_n;
};

// omega(N, e), any e < N/2 (two-level table only)
template <typename T>
__device__ __forceinline__ cx<T> tree_tw(const TreeTw& tw, uint64_t e) {
    return tw2(static_cast<const cx<T>*>(tw.lo), static_cast<const cx<T>*>(tw.hi), tw.h, e);
}

// omega(N, k 2^t), k < N >> (t+1): the level-t twiddle of butterfly k
template <typename T>
__device__ __forceinline__ cx<T> tree_tw_lv(const TreeTw& tw, uint64_t k, uint32_t t) {
    if (tw.direct)
        return static_cast<const cx<T>*>(tw.direct)[(1ull << tw.log_n) - (1ull << (tw.log_n - t)) + k];
    return tree_tw<T>(tw, k << t);
}

// The twiddles tree_levels applies, fetched in one go before any of them is
// used (round 6): with the reference-formula table, level tl's H = V >> (tl+1)
// entries omega(N, (i + ml D) 2^t) (the same for every block of the level) at
// w[V - (V >> tl) + ml]; with the two-level table, the raw lo / hi entries of
// each level's base w_N^{i 2^t} at w[2 tl], w[2 tl + 1].  Issued right after
// the leaf loads, all levels' lookups are ONE round trip beside them; looked
// up inside tree_levels, each level's loads waited behind the previous level's
// arithmetic (the compiler does not hoist them: a dependent load round trip
// per level -- 3 of them at P = 8, ~2.9 us of config 2's 4.9-us load phase,
// profiles/r06b_wg_clock_*).  Same values, same operations: bitwise equal.
template <typename T, int L>
struct TreeTwRegs {
    cx<T> w[(1 << L) > 2 * L ? (1 << L) : 2 * L];
};
template <typename T, int L>
__device__ __forceinline__ void tree_tw_fetch(TreeTwRegs<T, L>& r, const TreeTw& tw, uint64_t i, uint32_t log_d,
                                              uint32_t t0) {
    constexpr int V = 1 << L;
    if (tw.direct) {
#pragma unroll
        for (int tl = 0; tl < L; tl++) {
#pragma unroll
            for (int ml = 0; ml < (V >> (tl + 1)); ml++)
                r.w[V - (V >> tl) + ml] = tree_tw_lv<T>(tw, i + ((uint64_t)ml << log_d), t0 + (uint32_t)tl);
        }
    } else {
        const cx<T>* lo = static_cast<const cx<T>*>(tw.lo);
        const cx<T>* hi = static_cast<const cx<T>*>(tw.hi);
#pragma unroll
        for (int tl = 0; tl < L; tl++) {
            const uint64_t E = i << (t0 + (uint32_t)tl);
            r.w[2 * tl] = lo[E & ((1ull << tw.h) - 1)];
            r.w[2 * tl + 1] = hi[E >> tw.h];
        }
    }
}

// Levels t0 .. t0+L-1 of the reference's radix-2 tree (CPU.c:419-448; level t
// is the butterfly of size N >> t) on the 2^L values a thread holds at
// positions base + i + m*2^log_d.  After the last of these levels v[m] lies
// in the block leading to workers [((blk0 << L) + m) << log_w, +2^log_w);
// only branches leading to workers [q0, q1) are evaluated (uniform branches,
// compile-time register indices).  Operation order = butterfly_left /
// butterfly_right (CPU.c:540-576): add, or (sub) * omega.
// With the reference-formula table (tw.direct, N <= 2^22) every twiddle is a
// table entry, so the output is bit-identical to the reference.  With the
// two-level table the twiddle of position i + ml D at level t factors as
// w_N^{i 2^t} * w_{2^(L-tl)}^{ml} (D 2^t / N = 2^(tl-L)): one table lookup
// per level and thread, times a compile-time root (the fused pass's
// tree_path_steps does the same), instead of one two-level lookup per
// butterfly.  PRE: the twiddles were fetched already (tree_tw_fetch, `pre`).
template <typename T, int L, bool PRE = false>
__device__ __forceinline__ void tree_levels(cx<T>* v, const TreeTw& tw, uint64_t i, uint32_t log_d, uint32_t t0,
                                            uint64_t blk0, uint32_t log_w, uint64_t q0, uint64_t q1,
                                            const TreeTwRegs<T, L>& pre = TreeTwRegs<T, L>{}) {
    constexpr int V = 1 << L;
    if (!tw.direct) {
        cx<T> base[L];
#pragma unroll
        for (int tl = 0; tl < L; tl++) {
            if constexpr (PRE) base[tl] = cmul(pre.w[2 * tl + 1], pre.w[2 * tl]);  // (= tw2)
            else base[tl] = tree_tw<T>(tw, i << (t0 + tl));
        }
        static_for<0, L, 1>([&](auto tlc) {
            constexpr int tl = decltype(tlc)::value;
            constexpr int BS = V >> tl, H = BS >> 1, NS = 1 << (L - tl);
            constexpr RootsOf<NS> roots{};
#pragma unroll
            for (int blk = 0; blk < (1 << tl); blk++) {
                const int lo = blk * BS;
                const uint64_t cl0 = (((blk0 << L) + lo) << log_w), cl1 = (((blk0 << L) + lo + H) << log_w);
                const uint64_t cr1 = (((blk0 << L) + lo + BS) << log_w);
                const bool needL = (cl0 < q1) && (cl1 > q0);
                const bool needR = (cl1 < q1) && (cr1 > q0);
#pragma unroll
                for (int ml = 0; ml < H; ml++) {
                    const cx<T> x0 = v[lo + ml], x1 = v[lo + ml + H];
                    if (needL) v[lo + ml] = cadd(x0, x1);
                    if (needR) {
                        const cx<T> s{(T)roots.re[ml], (T)roots.im[ml]};
                        v[lo + ml + H] = cmul(csub(x0, x1), ml ? cmul(base[tl], s) : base[tl]);
                    }
                }
            }
        });
        return;
    }
#pragma unroll
    for (int tl = 0; tl < L; tl++) {
        const int BS = V >> tl, H = BS >> 1;
        const uint32_t t = t0 + tl;
#pragma unroll
        for (int blk = 0; blk < (1 << tl); blk++) {
            const int lo = blk * BS;
            const uint64_t cl0 = (((blk0 << L) + lo) << log_w), cl1 = (((blk0 << L) + lo + H) << log_w);
            const uint64_t cr1 = (((blk0 << L) + lo + BS) << log_w);
            const bool needL = (cl0 < q1) && (cl1 > q0);
            const bool needR = (cl1 < q1) && (cr1 > q0);
#pragma unroll
            for (int ml = 0; ml < H; ml++) {
                const cx<T> x0 = v[lo + ml], x1 = v[lo + ml + H];
                if (needL) v[lo + ml] = cadd(x0, x1);                      // butterfly_left
                if (needR)  // butterfly_right: omega(N, b N/size), b = i + ml D
                    v[lo + ml + H] = cmul(csub(x0, x1), PRE ? pre.w[V - (V >> tl) + ml]
                                                            : tree_tw_lv<T>(tw, i + ((uint64_t)ml << log_d), t));
            }
        }
    }
}

// The tree for ONE worker q (the reference's run_thread view, CPU.c:419-448):
// v[m] = x[i + m M] (m < P); level t keeps the left half (add) or the right
// half ((sub) * omega(N, b 2^t)) as bit log2P-1-t of q says (CPU.c:429), the
// kept half compacted into v[0 .. P>>(t+1)).  One uniform branch per level.
template <typename T, int LP>
__device__ __forceinline__ cx<T> tree_path(cx<T>* v, const TreeTw& tw, uint64_t i, uint32_t log_m, uint32_t q) {
#pragma unroll
    for (int t = 0; t < LP; t++) {
        const int H = (1 << LP) >> (t + 1);
        if ((q >> (LP - 1 - t)) & 1) {
#pragma unroll
            for (int ml = 0; ml < H; ml++)
                v[ml] = cmul(csub(v[ml], v[ml + H]), tree_tw_lv<T>(tw, i + ((uint64_t)ml << log_m), t));
        } else {
#pragma unroll
            for (int ml = 0; ml < H; ml++) v[ml] = cadd(v[ml], v[ml + H]);
        }
    }
    return v[0];
}

// tree_path for a thread's k-th first-pass input z_q[zi], zi = zi0 + k M/Q
// (the fused first pass): its level-t twiddle w_N^{(zi + ml M) 2^t} is
// bt[t] = w_N^{zi0 2^t} times the compile-time constant w_{QP}^{(k + Q ml) 2^t}
// (N = P M), so a thread needs log2 P table lookups instead of up to 2P per
// input.  Not bitwise vs the reference (the standalone k_tree is); tolerance.
template <typename T, int LP, int Q, int K>
__device__ __forceinline__ cx<T> tree_path_steps(cx<T>* v, const cx<T>* bt, uint32_t q) {
    constexpr int NS = Q << LP;
    constexpr RootsOf<NS> roots{};
#pragma unroll
    for (int t = 0; t < LP; t++) {
        const int H = (1 << LP) >> (t + 1);
        if ((q >> (LP - 1 - t)) & 1) {
#pragma unroll
            for (int ml = 0; ml < H; ml++) {
                const int e = ((K + Q * ml) << t) & (NS - 1);
                const cx<T> s{(T)roots.re[e], (T)roots.im[e]};
                v[ml] = cmul(csub(v[ml], v[ml + H]), cmul(bt[t], s));
            }
        } else {
#pragma unroll
            for (int ml = 0; ml < H; ml++) v[ml] = cadd(v[ml], v[ml + H]);
        }
    }
    return v[0];
}

// ---------------------------------------------------------------------------
// Stockham pass
// ---------------------------------------------------------------------------
// One pass of the local FFT (Stockham auto-sort, natural order in and out):
// for each line j < M/R of each transform, v_r = in[j + r M/R] (r < R),
// v_r *= w_{Ns R}^{(j mod Ns) r}, V = DFT_R(v),
// out[(j/Ns) Ns R + (j mod Ns) + r' Ns] = V_r'.
// A workgroup owns C adjacent lines (C*16 B contiguous per row on both sides
// for fp64) and keeps them in registers, 16 values per thread; the R-point
// DFT is one radix-2/4/8/16 stage plus radix-16 stages, with the values
// exchanged through LDS between stages one component at a time (re, then im),
// so the LDS footprint is C*R*sizeof(T) and two workgroups fit per CU.
struct PassArgs {
    const void* in;
    void* out;
    const void* tw_r;   // w_R^e, e < R
    const void* tw_lo;  // two-level w_M
    const void* tw_hi;
    uint64_t in_bstride;  // elements between consecutive transforms (input)
    uint64_t out_bstride;
    uint64_t nlines;      // transforms * M/R
    uint32_t log_lb;      // log2(M/R): lines per transform == element stride of a line
    uint32_t log_ns;      // log2 Ns (product of the radices of the previous passes)
    uint32_t tw_h;        // bits of the low twiddle table
    uint32_t tw_shift;    // log2(M / (Ns R))
    // MODE 3 (tree fused into the first pass): worker q of P = 2^LP, leaves
    // x[i + m M], in_bstride = N
    TreeTw tree;
    uint32_t worker;      // first worker of the plan (q0)
    uint32_t log_nq;      // log2 workers in the plan: transform t of the launch is
                          // worker q0 + (t mod nq) of batch t / nq (0: one worker)
    // XCD-aware tile order: blocks b and b+8 run on one XCD (shared L2); with
    // log_xg = g > 0, 2^g consecutive tiles (adjacent line groups) are given
    // to blocks of one XCD.  Needs gridDim.x % (8 << g) == 0 (else identity).
    uint32_t log_xg;
    // Natural-order store of a plan holding all P = 2^ilv_log workers (its
    // last pass; 0: the usual slice-major store).  Local transform bt is worker
    // bt mod P of batch bt / P, and its bin k lands at bitrev(bt mod P) + P k
    // of that batch's N = out_bstride outputs -- the stride-P interleave done
    // by the store instead of a separate launch (small N only: 16-B pieces
    // P x 16 B apart, cheap while the output stays in L2 / the Infinity Cache)
    uint32_t ilv_log;
    // Padded workspace rows (the plan's ping-pong buffer W between two
    // passes; 0 elsewhere).  Element e of a W transform sits at
    // e + (e >> s) pad, s = log2 of the reading pass's row stride: the
    // reading pass (BM 2) steps its R rows by 2^log_lb + in_pad, the writing
    // pass adds (j >> out_pad_log) out_pad to every store of line j (its
    // outputs e >> s all equal j >> (s - log2 R): a Stockham pass's output
    // blocks Ns R never straddle the next pass's rows, Ns R <= M / R').
    // Unpadded, the rows of W and of the caller's output sit at the same
    // offsets, 8 MiB apart at 2^28 fp64, and the C4 passes 2 and 3 ran fast
    // or slow (pass 3 1.58 vs 1.70-1.86 ms) by how the two allocations
    // happened to line up (tools/probe_place.py, tools/probe_pair.hip).
    uint32_t in_pad, out_pad, out_pad_log;
    // Worker-interleaved layout (MODE | 8, all P <= 16 workers of a natural-
    // order plan on one GPU): worker q's element e of transform bt sits at
    // bt bstride + e 2^wil + q, and launch line L = (j << wil) + q within a
    // transform -- line j of every worker back to back, so a tile's rows hold
    // all workers' values side by side (row segments 2^wil times wider) and
    // the last pass, storing worker q at slot bitrev(q) (wbrev), writes the
    // natural-order result bitrev(q) + P k directly: no interleave launch and
    // no scattered 16-B stores.
    uint32_t wil, wbrev;
#ifdef PIFFT_WG_CLOCK
    // diagnostics build only (tools/wg_clock.py): PIFFT_WGC_WORDS words per
    // workgroup -- 0 wall clock at entry, 1 once its stores completed, 2 the
    // hardware id, and thread 0's wall clock at each step of the chain: 3 the
    // tile's inputs in registers (loads landed; MODE 11: the tree evaluated
    // and handed to the first stage), 3 + S stage S's inputs received (S =
    // 1 .. 3: after the exchange from stage S - 1), 7 the last stage's
    // outputs computed (before the stores)
    unsigned long long* wg_clock;
#endif
};

#ifdef PIFFT_WG_CLOCK
#define PIFFT_WGC_WORDS 8
// thread 0 stamps `slot` once its own outstanding loads / LDS reads have
// landed (s_waitcnt 0); scheduling barriers keep the stamp in program order
__device__ __forceinline__ void wgc_stamp(const PassArgs& a, int tid, int slot) {
    __builtin_amdgcn_sched_barrier(0);
    if (a.wg_clock && tid == 0) {
        __builtin_amdgcn_s_waitcnt(0);
        a.wg_clock[PIFFT_WGC_WORDS * blockIdx.x + slot] = wall_clock64();
    }
    __builtin_amdgcn_sched_barrier(0);
}
#define PIFFT_WGC(slot) wgc_stamp(a, tid, (slot))
#else
#define PIFFT_WGC(slot) ((void)0)
#endif

__device__ __forceinline__ uint64_t tile_of_block(uint32_t b, uint32_t log_xg, uint32_t nblocks) {
    if (log_xg == 0 || (nblocks & ((8u << log_xg) - 1))) return b;
    const uint32_t xcd = b & 7, slot = b >> 3, gmask = (1u << log_xg) - 1;
    return ((uint64_t)(slot >> log_xg) << (log_xg + 3)) + ((uint64_t)xcd << log_xg) + (slot & gmask);
}

// values held per thread (VPT, a k_pass template argument): 16 for both
// precisions (32 fp32 values -- the same bytes as 16 fp64 -- measured 160-200
// VGPRs with spills at 128; 8 -- radix-8 stages, twice the waves per sub-FFT --
// measured slower for every single-pass batch size, profiles/r02_vpt_sweep.log).
// VPT 16: radix-16 stages + one trailing radix 2/4/8/16 stage; VPT 8: radix-8
// stages + one trailing radix 2/4/8.
template <int R, int VPT = 16>
struct PassShape {
    static constexpr int Q = R >= VPT ? VPT : (R >= 16 ? 16 : R);  // values per thread
    static constexpr int B = Q >= 16 ? 16 : Q;                      // radix of the non-last stages
    static constexpr int LOGB = ilog2c(B);
    static constexpr int LOGR = ilog2c(R);
    static constexpr int NSTG = LOGB ? (LOGR + LOGB - 1) / LOGB : 1;   // radix-B stages + 1 trailing
    static constexpr int QL = 1 << (LOGR - LOGB * (NSTG - 1));        // trailing radix
};

template <int R, int C, int VPT = 16>
struct PassCfg {
    static constexpr int NT = C * R / PassShape<R, VPT>::Q;
#ifndef PIFFT_MIN_WG_PER_CU
#define PIFFT_MIN_WG_PER_CU 2
#endif
    // register budget: PIFFT_MIN_WG_PER_CU workgroups resident per CU, but
    // never under 128 VGPRs (4 waves/SIMD): 16 complex values + twiddles
    static constexpr int wpe = NT >= 256 ? (NT * PIFFT_MIN_WG_PER_CU) / 256 : 1;
    static constexpr int waves_per_eu = wpe > 4 ? 4 : wpe;
};

// LDS image of a workgroup's C lines during an exchange (one component, T
// scalars): element r of line c sits at c*ls + swz(r), swz(r) = (r XOR ((r >>
// xs) & xm) XOR ((c & cm) << cs)) + (ps ? r >> ps : 0) -- XOR swizzles of the
// low bits (by higher bits of r, or by the line) and/or one pad scalar per 2^ps.  The round-1 layout (lds_default: r + r/16, odd line
// stride) had 2-way bank conflicts on every exchange of the C4 first pass
// (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 0.40, profiles/r01_lds_pmc.txt).
// tools/lds_model.hip replays each pass instance's exchanges through the
// kernel's own thread maps (Stage::map) under the gfx950 banking rules
// (MI355X_MICROARCH.md, LDS) and picks, per instance, the layout with the
// fewest LDS-array cycles at no more LDS than the default: the generated
// LdsPick specializations in pifft_lds_layouts.inc.
struct LdsLayout {
    int ls, xs, xm, ps, cm, cs;  // (cm, cs): XOR of (c & cm) << cs, a per-line rotation of the banks
};
__host__ __device__ constexpr int lds_at(LdsLayout L, int c, int r) {
    return c * L.ls + (r ^ ((r >> L.xs) & L.xm) ^ ((c & L.cm) << L.cs)) + (L.ps ? (r >> L.ps) : 0);
}
template <int R>
constexpr LdsLayout lds_default() { return LdsLayout{R + R / 16 + 1, 4, 0, 4, 0, 0}; }
template <typename T, int R, int C, int BM, int VPT>
struct LdsPick {
    static constexpr LdsLayout value = lds_default<R>();
};
#ifndef PIFFT_LDS_DEFAULT_ONLY
#include "pifft_lds_layouts.inc"
#endif

// The stage maps (Stage) and LDS layout (LdsPick) a pass MODE uses: its
// low two bits, except MODE 11 (the all-worker tree fused into the first
// worker-interleaved pass), whose stages are those of a MODE 10 pass -- lanes
// across lines on both strided sides.
constexpr int stage_mode(int mode) { return ((mode & 3) == 3 && (mode & 8)) ? 2 : (mode & 3); }

// dynamic LDS bytes of a k_pass instance (0 for a single-stage sub-FFT; MODE
// 11 always exchanges: the tree's values reach the first stage through LDS)
template <typename T, int R, int C, int MODE, int VPT>
constexpr int pass_lds_bytes() {
    return (PassShape<R, VPT>::NSTG > 1 || MODE == 11)
               ? C * LdsPick<T, R, C, stage_mode(MODE), VPT>::value.ls * (int)sizeof(T)
               : 0;
}

// v[k] *= w^k (0 < k < q), w^k = w^(k - lowbit k) * w^(lowbit k), anchors
// a[i] = w^(2^i): chains of <= 3 products, each power applied when formed.
template <int q, typename T>
__device__ __forceinline__ void apply_powers(cx<T>* v, const cx<T>* anc) {
    cx<T> w[q];
#pragma unroll
    for (int k = 1; k < q; k++) {
        const int lb = k & -k;
        w[k] = (k == lb) ? anc[ilog2c(lb)] : cmul(w[k - lb], w[lb]);
        v[k] = cmul(v[k], w[k]);
    }
}

// Stage S of the R-point sub-FFT in a pass of mode MODE:
//   radix q (16, the last one 2/4/8/16), U = Q/q butterflies per thread,
//   NB = R/q butterflies per line, ns = 16^S (product of previous radices).
// Butterfly g = tid + u*NT maps to (line c, butterfly b) "c-fast" (lanes
// across lines: the strided side of a pass in HBM) or "b-fast" (lanes along
// a line: LDS stages and contiguous HBM sides).
template <int R, int C, int MODE, int S, int VPT>
struct Stage {
    using Sh = PassShape<R, VPT>;
    static constexpr int NT = PassCfg<R, C, VPT>::NT;
    static constexpr bool first = S == 0, last = S == Sh::NSTG - 1;
    static constexpr int q = last ? Sh::QL : Sh::B;
    static constexpr int U = Sh::Q / q;
    static constexpr int NB = R / q;
    static constexpr int ns = 1 << (Sh::LOGB * S);
    static constexpr bool cfast = first ? (MODE != 0) : (last ? (MODE == 2) : false);  // MODE 3 as MODE 1
#ifndef PIFFT_WAVE_PRIVATE
#define PIFFT_WAVE_PRIVATE 3  // bit 0: whole-line stages (a), bit 1: beta groups (b)
#endif
    // Wave-private exchanges (no workgroup barrier into this stage).
    // (a) b-fast stage after a b-fast radix-16 stage (one butterfly per
    //     thread) whose R/16 butterflies per line divide 64: every wave holds
    //     whole lines, and this stage keeps each wave on the same lines.
    static constexpr int NBP = R / 16;
    static constexpr bool whole_lines = (PIFFT_WAVE_PRIVATE & 1) && !first && !cfast && (S >= 2 || MODE == 0) &&
                                        Sh::Q == 16 && NBP <= 64 && 64 % NBP == 0 && NT % 64 == 0;
    static constexpr int LPW = whole_lines ? 64 / NBP : 1;  // lines per wave
    // (b) MODE 2, three stages, middle + (c-fast) last stage: last-stage
    //     butterflies beta + 16 m (m < 16) read exactly the outputs of the
    //     middle-stage butterflies beta + 16 k (k < QL).  A wave owns the same
    //     beta groups on all C lines in both stages (lanes across lines).
    static constexpr bool grouped = (PIFFT_WAVE_PRIVATE & 2) && MODE == 2 && Sh::NSTG == 3 && S >= 1 && Sh::Q == 16 &&
                                    64 % C == 0 && (64 / C) % Sh::QL == 0 && NT % 64 == 0;
    static constexpr int GPW = grouped ? 64 / (C * Sh::QL) : 1;  // beta groups per wave
    static constexpr bool wave_private = whole_lines || (grouped && last);
    // (c) Register exchange into the last stage: no LDS round trip.  The
    //     middle radix-16 stage leaves one butterfly per thread (lane l of a
    //     wave = butterfly l % NBP of line l / NBP, holding elements
    //     256 (l%NBP / 16) + l%16 + 16 k, k < 16).  A last radix 4 over
    //     NBP = 64 lanes (R = 1024) is then a 4x4 transpose of register
    //     quadruples across the wave's four 16-lane rows, a last radix 2 over
    //     NBP = 32 (R = 512) a 2x2 transpose of register pairs across row
    //     pairs: cross-lane v_permlane32_swap / v_permlane16_swap (CDNA4)
    //     instead of an LDS store + load per component.
    //     PIFFT_PERMLANE bit 0: radix 2 (R = 512), bit 1: radix 4 (R = 1024).
    //     Measured on MI355X (tools/gpu_round.sh perm): radix 2 in the fused
    //     tree pass ~0.5 % faster.  Radix 4 cost 2 spills and 5.5 % in round
    //     1's C4 first pass; since round 3 it compiles spill-free wherever
    //     the workgroup holds at most 4 lines or runs a plain first pass
    //     (fp32 instances drop 4-16 VGPRs with it), while the fp64 single
    //     passes at C = 8 / 16 and fused passes at C = 16 would spill 2-4
    //     VGPRs (round 5, every instance's gfx950 register metadata with and
    //     without it) -- so it is on there only (perm4_ok).  Config 1 +0.5-1 %
    //     (profiles/r04c_permlane4_c1.log), bitwise equal to the LDS path.
#ifndef PIFFT_PERMLANE
#define PIFFT_PERMLANE 3
#endif
    static constexpr bool perm4_ok = C <= 4 || MODE == 1;
    static constexpr bool perm = last && !first && !cfast && Sh::Q == 16 && NT % 64 == 0 && Sh::NSTG == 3 &&
                                 (((PIFFT_PERMLANE & 2) && q == 4 && NBP == 64 && perm4_ok) ||
                                  ((PIFFT_PERMLANE & 1) && q == 2 && NBP == 32));
    __host__ __device__ static __forceinline__ void map(int tid, int u, int& c, int& b) {
        if constexpr (perm) {
            const int lane = tid & 63;
            c = (tid >> 6) * (64 / NBP) + lane / NBP;
            b = lane % NBP + NBP * u;
        } else if constexpr (grouped) {
            const int w = tid >> 6, lane = tid & 63;
            c = lane % C;
            if constexpr (!last) {  // one butterfly per thread
                const int slot = lane / C;
                b = (w * GPW + slot / Sh::QL) + 16 * (slot % Sh::QL);
            } else {
                const int slot = (u * 64 + lane) / C;
                b = (w * GPW + slot % GPW) + 16 * (slot / GPW);
            }
        } else if constexpr (cfast) {
            const int g = tid + u * NT;
            c = g % C; b = g / C;
        } else if constexpr (whole_lines) {
            const int i = u * 64 + (tid & 63);
            c = (tid >> 6) * LPW + i / NB; b = i % NB;
        } else {
            const int g = tid + u * NT;
            c = g / NB; b = g % NB;
        }
    }
};

// The LDS hand-off between two stages: a workgroup barrier, or -- when each
// wave reads back only what it wrote itself -- a fence that keeps the
// compiler from moving the wave's LDS loads above its stores (a wave's LDS
// instructions complete in order).
template <bool WAVE>
__device__ __forceinline__ void lds_handoff() {
    if constexpr (WAVE) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    } else {
        __syncthreads();
    }
}

// swap halves across lanes (v_permlane16_swap: odd 16-lane rows of a with even
// rows of b; v_permlane32_swap: upper 32 lanes of a with lower 32 of b)
template <int W>
__device__ __forceinline__ void pl_swap(uint32_t& a, uint32_t& b) {
    if constexpr (W == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
        a = r[0];
        b = r[1];
    } else {
        static_assert(W == 32, "permlane width");
        const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
        a = r[0];
        b = r[1];
    }
}
template <int W, typename T>
__device__ __forceinline__ void pl_swap(cx<T>& a, cx<T>& b) {
    constexpr int ND = (int)(sizeof(cx<T>) / 4);
    uint32_t x[ND], y[ND];
    __builtin_memcpy(x, &a, sizeof a);
    __builtin_memcpy(y, &b, sizeof b);
#pragma unroll
    for (int d = 0; d < ND; d++) pl_swap<W>(x[d], y[d]);
    __builtin_memcpy(&a, x, sizeof a);
    __builtin_memcpy(&b, y, sizeof b);
}

// Stage twiddles fetched with the data (PIFFT_TW_PREFETCH): the anchors of
// every later stage's butterflies are loaded right after the tile's inputs
// are issued (all of w, w^2, w^4, w^8, or only w with the others formed by
// squaring when the stage runs) -- instead of 2-4 table loads at the start
// of each stage, each a
// dependent round trip on a workgroup's critical path.  That path is what
// bounds the latency-bound small launches (one or two workgroups per CU);
// the streaming passes hide it behind the other workgroup.
// 0: off; 1: single passes (MODE 0/4) only; 2: every pass; 3: single and
// first passes (MODE 0/1) of tiles built for at most 2 waves per SIMD (a
// budget of 256 VGPRs), every anchor w, w^2, w^4, w^8 fetched from the table
// (the values the stage would load itself: bitwise equal to 0; the 128-VGPR
// instances would spill 4-46 VGPRs).
// Measured on MI355X (profiles/r02_ab_twiddle_prefetch.log): no gain on the
// small launches (fp32 4096 x 512: 9 us either way; fp64 2^20: 24 us either
// way), fp64 8192 x 64 single passes 11 -> 15 us (registers), C4 +3 % at 2 --
// so off; round 6 (profiles/r06s_*): at 2, config 3's single pass 47 -> 45
// us and the first passes of C1 / C4 1-2 % faster, config 2's and C4's
// later passes 3-11 % slower (spills at 128 VGPRs) -- hence 3, the default
// since round 6 (profiles/r06t_*: outputs bitwise equal to 0 on 15 plans;
// config 3 +1.4 %, config 1 +0.9 %, fp64 4096 x 1024 +5.5 %, fp64 2^22 +1.2 %,
// configs 2 and 4 tie).
#ifndef PIFFT_DIAG_NO_XCHG
#define PIFFT_DIAG_NO_XCHG 0  // diagnostics: skip the LDS hand-offs between stages (timing only)
#endif
#ifndef PIFFT_TW_PREFETCH
#define PIFFT_TW_PREFETCH 3
#endif
template <int R, int C, int BM, int VPT>
constexpr bool tw_prefetch() {
    return PIFFT_TW_PREFETCH == 2 || (PIFFT_TW_PREFETCH == 1 && BM == 0) ||
           (PIFFT_TW_PREFETCH == 3 && (BM == 0 || BM == 1) && PassCfg<R, C, VPT>::waves_per_eu <= 2);
}
// anchors fetched per butterfly of a radix-q stage: all log2 q (3), or the
// base one, the others formed by squaring (1, 2)
template <int q>
constexpr int pre_anchors() { return PIFFT_TW_PREFETCH == 3 ? ilog2c(q) : 1; }
// anchors of stages 1 .. S-1
template <int R, int C, int BM, int VPT, int S>
constexpr int pre_offset() {
    if constexpr (S <= 1) return 0;
    else return pre_offset<R, C, BM, VPT, S - 1>() +
                Stage<R, C, BM, S - 1, VPT>::U * pre_anchors<Stage<R, C, BM, S - 1, VPT>::q>();
}
template <int R, int C, int BM, int VPT>
constexpr int pre_count() {
    return pre_offset<R, C, BM, VPT, PassShape<R, VPT>::NSTG>();
}

// Workgroups per CU a k_pass instance is built for: two (PIFFT_MIN_WG_PER_CU),
// one for the fused tree pass at P = 16 (its 16 leaves per input)
// (config 3's single pass built for 8 waves per SIMD -- 64 VGPRs, 8 of its 16
// workgroups per CU at once instead of 7 -- spills 18 B per lane and runs
// 70 % slower: round 4, profiles/r04f_c3_wpe8.log)
template <typename T, int R, int C, int MODE, int LP, int VPT>
constexpr int pass_waves_per_eu() {
    constexpr int w = PassCfg<R, C, VPT>::waves_per_eu;
    return ((MODE & 3) == 3 && LP >= 5) ? 1 : ((MODE & 3) == 3 && LP >= 4 && w > 2) ? 2 : w;
}
// The stage-twiddle prefetch of a k_pass instance: tw_prefetch, and (at 3)
// the one-worker fused tree pass (MODE 3) of 256-VGPR tiles as well -- round 6
// (profiles/r06y5_*): config 2's one-GPU slice +1.9 %, bitwise equal; the
// all-worker fused pass (MODE 11) measured 0.3 % slower with it, so not there.
template <typename T, int R, int C, int MODE, int LP, int VPT>
constexpr bool pass_tw_prefetch() {
    if constexpr (PIFFT_TW_PREFETCH == 3 && (MODE & 3) == 3 && !(MODE & 8) &&
                  pass_waves_per_eu<T, R, C, MODE, LP, VPT>() <= 2)
        return true;
    return tw_prefetch<R, C, MODE & 3, VPT>();
}

// MODE 11 = 3 | 8: the tree of ALL P = 2^LP workers fused into the first
// worker-interleaved pass (an all-worker natural-order plan, PassArgs::wil =
// LP).  The tile's C = J P launch lines are J adjacent line indices j times
// the P workers (L = (j << LP) + q), so its C R inputs z_q[j + r M/R] come from
// exactly J R P leaves x[j + r M/R + m M]: each position's P leaves are loaded
// once (J adjacent j per leaf row: J esz-byte segments, 256 B at the
// planner's J), the full radix-2 tree (tree_levels, every branch, the
// reference's operation order) gives every worker's value there, and one LDS
// transpose per component hands them to the pass's first stage (lanes across
// lines, as MODE 10).  Replaces the all-worker tree launch (k_tree_wil),
// which wrote the N tree values and had the first pass read them back.
template <typename T, int R, int C, int LP, int VPT, int NTS>
__device__ __forceinline__ void wil_tree_to_lds(const PassArgs& a, T* lds, cx<T>* v, int tid, uint64_t tile) {
    using C2 = cx<T>;
    using Sh = PassShape<R, VPT>;
    using St = Stage<R, C, 2, 0, VPT>;
    constexpr int P = 1 << LP, J = C / P;
    constexpr int NT = PassCfg<R, C, VPT>::NT;
    constexpr LdsLayout LL = LdsPick<T, R, C, 2, VPT>::value;
    const uint32_t log_lb = a.log_lb;
    const uint32_t lbi = log_lb + (uint32_t)LP;
    const uint32_t log_m = log_lb + (uint32_t)Sh::LOGR;  // leaf stride M
    const uint64_t line0 = tile * C;                    // (C divides a transform's lines: no partial tile)
    const uint64_t bt = line0 >> lbi;
    const uint64_t j0 = (line0 & ((1ull << lbi) - 1)) >> LP;
    const C2* __restrict__ x = static_cast<const C2*>(a.in) + bt * a.in_bstride;
    if constexpr (P > Sh::Q) {
        // P = 2 Q (32 workers at 16 values per thread): two threads per
        // position, thread half h evaluating the tree pruned to workers [h P/2,
        // (h + 1) P/2) (tree_levels' worker range: the reference's order on
        // the branches it keeps); h is uniform per wave from R = 64 on
        static_assert(P == 2 * Sh::Q && 2 * J * R == NT, "MODE 11, P = 2Q: two threads per position");
        constexpr int H = P / 2;
        const int p = tid % (J * R), h = tid / (J * R);
        const uint64_t i = j0 + (uint64_t)(p % J) + ((uint64_t)(p / J) << log_lb);
        C2 w[P];
#pragma unroll
        for (int m = 0; m < P; m++) w[m] = ld_stream<nt_loads(NTS)>(x + i + ((uint64_t)m << log_m));
        tree_levels<T, LP>(w, a.tree, i, log_m, 0, 0, 0, (uint64_t)(h * H), (uint64_t)(h * H + H));
        const int jl = p % J, r = p / J;
#pragma unroll
        for (int comp = 0; comp < 2; comp++) {
            if (comp) __syncthreads();
            if (h) {
#pragma unroll
                for (int m = 0; m < H; m++) lds[lds_at(LL, jl * P + H + m, r)] = comp ? w[H + m].im : w[H + m].re;
            } else {
#pragma unroll
                for (int m = 0; m < H; m++) lds[lds_at(LL, jl * P + m, r)] = comp ? w[m].im : w[m].re;
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < St::U; u++) {
                int c, b;
                St::map(tid, u, c, b);
#pragma unroll
                for (int k = 0; k < St::q; k++) {
                    const T y = lds[lds_at(LL, c, b + k * St::NB)];
                    if (comp) v[u * St::q + k].im = y; else v[u * St::q + k].re = y;
                }
            }
        }
        __syncthreads();
        return;
    } else {
    constexpr int PPT = Sh::Q / P;  // tree positions per thread
    static_assert(C % P == 0 && Sh::Q % P == 0 && PPT * P * NT == C * R, "MODE 11 tile: J P lines, Q / P positions");
    C2 w[PPT][P];
#pragma unroll
    for (int u = 0; u < PPT; u++) {  // every leaf load issued before any use
        const int p = tid + u * NT;  // position: J adjacent j (lanes), then r
        const uint64_t i = j0 + (uint64_t)(p % J) + ((uint64_t)(p / J) << log_lb);
#pragma unroll
        for (int m = 0; m < P; m++) w[u][m] = ld_stream<nt_loads(NTS)>(x + i + ((uint64_t)m << log_m));
    }
    // every level's twiddles in one round trip beside the leaves (where the
    // instance has the registers: <= 2 waves per SIMD, i.e. the latency-bound
    // small tiles; the 128-VGPR streaming instances would spill)
    constexpr bool PRE = pass_waves_per_eu<T, R, C, 11, LP, VPT>() <= 2;
    TreeTwRegs<T, LP> trw[PRE ? PPT : 1];
    if constexpr (PRE) {
#pragma unroll
        for (int u = 0; u < PPT; u++) {
            const int p = tid + u * NT;
            tree_tw_fetch<T, LP>(trw[u], a.tree, j0 + (uint64_t)(p % J) + ((uint64_t)(p / J) << log_lb), log_m, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int u = 0; u < PPT; u++) {
        const int p = tid + u * NT;
        const uint64_t i = j0 + (uint64_t)(p % J) + ((uint64_t)(p / J) << log_lb);
        tree_levels<T, LP, PRE>(w[u], a.tree, i, log_m, 0, 0, 0, 0, P, trw[PRE ? u : 0]);  // w[u][m] = z_m[i]
    }
#pragma unroll
    for (int comp = 0; comp < 2; comp++) {
        if (comp) __syncthreads();  // the first component's reads are done
#pragma unroll
        for (int u = 0; u < PPT; u++) {
            const int p = tid + u * NT, jl = p % J, r = p / J;
#pragma unroll
            for (int m = 0; m < P; m++) lds[lds_at(LL, jl * P + m, r)] = comp ? w[u][m].im : w[u][m].re;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < St::U; u++) {
            int c, b;
            St::map(tid, u, c, b);
#pragma unroll
            for (int k = 0; k < St::q; k++) {
                const T y = lds[lds_at(LL, c, b + k * St::NB)];
                if (comp) v[u * St::q + k].im = y; else v[u * St::q + k].re = y;
            }
        }
    }
    __syncthreads();  // every read done before the first stage's exchange writes LDS
    }
}

#ifndef PIFFT_SERIAL_BFLY
#define PIFFT_SERIAL_BFLY 1
#endif
template <typename T, int R, int C, int MODE, int NTS, int LP, int S, int VPT>
__device__ __forceinline__ void pass_stages(const PassArgs& a, T* lds, cx<T>* v, cx<T>* pre, int tid, uint64_t tile,
                                            cx<T>* twp) {
    using C2 = cx<T>;
    // MODE | 4: the same pass storing at bitrev_{log2 M}(natural position),
    // the reference's scratch order (PIFFT_OUT_BITREV; last pass only).  Each
    // line's R outputs still land in one contiguous R-element block; plain
    // (L2-merged) stores.  A compile-time variant: a run-time flag in the
    // store path cost 5-15 % on every pass (tools/ab.sh).
    constexpr int BM = MODE & 3;
    constexpr bool BREV = (MODE & 4) != 0;
    constexpr bool WIL = (MODE & 8) != 0;  // worker-interleaved layout (PassArgs::wil)
    constexpr int SM = stage_mode(MODE);   // the stage maps' mode (MODE 11: MODE 10's)
    using St = Stage<R, C, SM, S, VPT>;
    using Sh = PassShape<R, VPT>;
    constexpr int q = St::q, U = St::U, NB = St::NB, ns = St::ns;
    constexpr LdsLayout LL = LdsPick<T, R, C, SM, VPT>::value;
    // Several butterflies per thread (VPT 32): one after the other, each with
    // its own twiddles, loads and stores -- scheduling barriers keep the
    // compiler from interleaving their temporaries and hoisting their
    // addresses (two concurrent radix-16 DFTs spill at the 128-VGPR budget of
    // two workgroups per CU)
    constexpr bool serial = U > 1 && Sh::Q > 16 && PIFFT_SERIAL_BFLY;
    // (run-time even where the mode fixes them -- M/R = 1 for a single pass,
    // Ns = 1 for a first pass: compile-time values measured 2 % slower there)
    const uint32_t log_lb = a.log_lb;
    const uint32_t log_ns = a.log_ns;
    const uint64_t ns_mask = (1ull << log_ns) - 1;
    // lines per transform (= element stride of a line): 2^log_lb, or with the
    // worker-interleaved layout 2^(log_lb + wil) launch lines L = (j << wil) + q
    const uint32_t wil = WIL ? a.wil : 0u;
    const uint32_t lbi = log_lb + wil;
    const uint64_t lb_mask = (1ull << lbi) - 1;
    if constexpr (S > 0 && S <= 3) PIFFT_WGC(3 + S);

    // MODE 2: the inter-pass twiddle factors depend only on (line, b); their
    // two-level table entries are fetched with the data, not after it (a
    // second dependent round trip per workgroup otherwise)
    // With several butterflies per thread on the same line (c-fast map, NT a
    // multiple of C: c does not depend on u) the step factor w^{jm NB} is
    // shared: fetched once, for u = 0.
    constexpr bool share_anc = St::cfast && U > 1 && St::NT % C == 0;
    [[maybe_unused]] C2* tw_pre = twp;  // 4 U entries (k_pass: first_tw_count)
    if constexpr (St::first && BM == 2) {
        const C2* tlo = static_cast<const C2*>(a.tw_lo);
        const C2* thi = static_cast<const C2*>(a.tw_hi);
        const uint64_t hmask = (1ull << a.tw_h) - 1;
#pragma unroll
        for (int u = 0; u < U; u++) {
            int c, b;
            St::map(tid, u, c, b);
            const uint64_t jm = (((tile * C + c) & lb_mask) >> wil) & ns_mask;
            const uint64_t e0 = (jm * (uint64_t)NB) << a.tw_shift, e1 = (jm * (uint64_t)b) << a.tw_shift;
            if (!share_anc || u == 0) {
                tw_pre[4 * u + 0] = tlo[e0 & hmask];
                tw_pre[4 * u + 1] = thi[e0 >> a.tw_h];
            }
            tw_pre[4 * u + 2] = tlo[e1 & hmask];
            tw_pre[4 * u + 3] = thi[e1 >> a.tw_h];
        }
    }
    if constexpr (St::first && BM == 3 && WIL) {
        // ---- MODE 11: every worker's tree, then the first stage's inputs via LDS ----
        wil_tree_to_lds<T, R, C, LP, VPT, NTS>(a, lds, v, tid, tile);
    } else if constexpr (St::first) {
        // ---- inputs straight from HBM (all loads issued before any use) ----
        const C2* __restrict__ in = static_cast<const C2*>(a.in);
#pragma unroll
        for (int u = 0; u < U; u++) {
            int c, b;
            St::map(tid, u, c, b);
            // (clamp_loads: idle lanes of a partial last tile load the last
            // line again -- their results are never stored)
            constexpr bool CL = clamp_loads<T>();
            const bool ok = CL || tile * C + c < a.nlines;
            const uint64_t line = (!CL || tile * C + c < a.nlines) ? tile * C + c : a.nlines - 1;
            const uint64_t bt = line >> lbi, j = line & lb_mask;
            const uint32_t les = lbi;
            // MODE 3: transform bt is worker (bt mod nq) of batch bt / nq, and
            // the leaves come from that batch's input
            const uint64_t bin = BM == 3 ? (bt >> a.log_nq) : bt;
            const C2* src = in + bin * a.in_bstride + j + ((uint64_t)b << les);
            if constexpr (BM == 3) {
                static_assert(!WIL, "the fused tree pass is slice-major only");
                // z_q[zi] from the P leaves x[zi + m M] (M = 2^(log_lb + LOGR)),
                // G elements (G*P = 8 loads in flight) per round: no spills up
                // to P = 8 at 128 VGPRs.  Small tiles (<= 256 threads: a
                // register budget of >= 256 VGPRs, e.g. config 2's one-GPU
                // slice, 64 workgroups) keep more leaves in flight, so fewer
                // dependent rounds of loads
                constexpr int P = 1 << LP;
#ifndef PIFFT_TREE_LOADS
#define PIFFT_TREE_LOADS 8  // leaf loads in flight per thread and round
#endif
#ifndef PIFFT_TREE_LOADS_SMALL
#define PIFFT_TREE_LOADS_SMALL 16  // the same for tiles of <= 256 threads
#endif
                constexpr int TL = PassCfg<R, C, VPT>::NT <= 256 ? PIFFT_TREE_LOADS_SMALL : PIFFT_TREE_LOADS;
                constexpr int G0 = P >= TL ? 1 : TL / P;
                constexpr int G = G0 > q ? q : G0;  // (at most one round per value)
                static_assert(q % G == 0, "whole rounds of leaf loads");
                const uint32_t log_m = log_lb + Sh::LOGR;
                const uint32_t wq = a.worker + (uint32_t)(tile * C >> log_lb & ((1u << a.log_nq) - 1));
                const C2* lsrc = src;
                // this thread's base twiddles w_N^{zi0 2^t}, zi0 = its k = 0 input
                const uint64_t zi0 = j + ((uint64_t)b << log_lb);
                C2 bt[LP];
#pragma unroll
                for (int t = 0; t < LP; t++) bt[t] = tree_tw_lv<T>(a.tree, zi0, t);
                static_for<0, q, G>([&](auto k0c) {
                    constexpr int k0 = decltype(k0c)::value;
                    C2 w[G][P];
#pragma unroll
                    for (int g = 0; g < G; g++) {
                        const C2* leaf = lsrc + ((uint64_t)((k0 + g) * NB) << log_lb);
#pragma unroll
                        for (int m = 0; m < P; m++)
                            w[g][m] = ok ? ld_stream<nt_loads(NTS)>(leaf + ((uint64_t)m << log_m)) : C2{(T)0, (T)0};
                    }
                    static_for<0, G, 1>([&](auto gc) {
                        constexpr int g = decltype(gc)::value;
                        v[u * q + k0 + g] =
                            tree_path_steps<T, LP, q, k0 + g>(w[g], bt, wq);
                    });
                    __builtin_amdgcn_sched_barrier(0);  // next round's leaves after this one's trees
                });
            } else if constexpr (BM == 2) {
                // rows 2^les + in_pad apart (padded workspace, PassArgs::in_pad)
                const uint64_t rs = (1ull << les) + a.in_pad;
                const C2* row = in + bin * a.in_bstride + j + (uint64_t)b * rs;
#pragma unroll
                for (int k = 0; k < q; k++)
                    v[u * q + k] = ok ? ld_stream<nt_loads(NTS)>(row + (uint64_t)(k * NB) * rs) : C2{(T)0, (T)0};
            } else {
#pragma unroll
                for (int k = 0; k < q; k++)
                    v[u * q + k] = ok ? ld_stream<nt_loads(NTS)>(src + ((uint64_t)(k * NB) << les)) : C2{(T)0, (T)0};
            }
        }
    }
    if constexpr (St::first) PIFFT_WGC(3);
    if constexpr (St::first && pass_tw_prefetch<T, R, C, MODE, LP, VPT>()) {
        const C2* __restrict__ twr = static_cast<const C2*>(a.tw_r);
        static_for<1, Sh::NSTG, 1>([&](auto sc) {
            constexpr int S2 = decltype(sc)::value;
            using St2 = Stage<R, C, SM, S2, VPT>;  // (the stage maps' mode: MODE 11 uses MODE 10's)
#pragma unroll
            for (int u = 0; u < St2::U; u++) {
                int c, b;
                St2::map(tid, u, c, b);
                constexpr int NA = pre_anchors<St2::q>();
                const int e1 = (b & (St2::ns - 1)) * (R / (St2::ns * St2::q));
#pragma unroll
                for (int i = 0; i < NA; i++) pre[pre_offset<R, C, SM, VPT, S2>() + u * NA + i] = twr[e1 << i];
            }
        });
    }
    // ---- twiddles before the butterflies ----
    if constexpr (St::first && BM == 2) {
        // w_{Ns R}^{(j mod Ns) r}, r = b + k NB: the k-dependent factor
        // step^k now, the common factor w^{(j mod Ns) b} after the DFT
        C2 anc[4];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (!share_anc || u == 0) {
                const int uu = share_anc ? 0 : u;
                anc[0] = cmul(tw_pre[4 * uu + 1], tw_pre[4 * uu + 0]);  // = tw2(lo, hi, h, jm NB)
#pragma unroll
                for (int i = 1; (1 << i) < q; i++) anc[i] = cmul(anc[i - 1], anc[i - 1]);
            }
            apply_powers<q>(&v[u * q], anc);
            if constexpr (serial) {
                dft<q>(&v[u * q]);
                const C2 base = cmul(tw_pre[4 * u + 3], tw_pre[4 * u + 2]);  // = tw2(lo, hi, h, jm b)
#pragma unroll
                for (int k = 0; k < q; k++) v[u * q + k] = cmul(v[u * q + k], base);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    if constexpr (!St::first) {
        // w_{ns q}^{(b mod ns) k} = w_R^{(b mod ns) k R/(ns q)}
        const C2* __restrict__ twr = static_cast<const C2*>(a.tw_r);
#pragma unroll
        for (int u = 0; u < U; u++) {
            int c, b;
            St::map(tid, u, c, b);
            const int e1 = (b & (ns - 1)) * (R / (ns * q));
            C2 anc[4];
            if constexpr (pass_tw_prefetch<T, R, C, MODE, LP, VPT>()) {
                constexpr int NA = pre_anchors<q>();
#pragma unroll
                for (int i = 0; i < NA; i++) anc[i] = pre[pre_offset<R, C, SM, VPT, S>() + u * NA + i];
#pragma unroll
                for (int i = NA; (1 << i) < q; i++) anc[i] = cmul(anc[i - 1], anc[i - 1]);
            } else {
#pragma unroll
                for (int i = 0; (1 << i) < q; i++) anc[i] = twr[e1 << i];
            }
            apply_powers<q>(&v[u * q], anc);
        }
    }
    if constexpr (!(St::first && BM == 2 && serial)) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            dft<q>(&v[u * q]);
            if constexpr (serial) __builtin_amdgcn_sched_barrier(0);
        }
    }
    if constexpr (St::first && BM == 2 && !serial) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const C2 base = cmul(tw_pre[4 * u + 3], tw_pre[4 * u + 2]);  // = tw2(lo, hi, h, jm b)
#pragma unroll
            for (int k = 0; k < q; k++) v[u * q + k] = cmul(v[u * q + k], base);
        }
    }

    if constexpr (St::last) {
        PIFFT_WGC(7);
        // ---- outputs r' = b + k NB straight to HBM ----
        C2* __restrict__ out = static_cast<C2*>(a.out);
#pragma unroll
        for (int u = 0; u < U; u++) {
            int c, b;
            St::map(tid, u, c, b);
            const uint64_t line = tile * C + c;
            if (line < a.nlines) {
                const uint64_t bt = line >> lbi, lj = line & lb_mask;
                const uint64_t j = lj >> wil;  // the worker's own line
                const uint32_t lns = (uint32_t)log_ns;
                const uint64_t pos = ((j >> lns) << (lns + Sh::LOGR)) + (j & ((1ull << lns) - 1)) + ((uint64_t)b << lns);
                if constexpr (WIL) {
                    // worker q at slot q (or bitrev(q): the natural-order result)
                    const uint32_t wq = (uint32_t)(lj & ((1ull << wil) - 1));
                    const uint64_t slot = a.wbrev ? (uint64_t)(__builtin_bitreverse32(wq) >> (32 - wil)) : wq;
                    C2* dst = out + bt * a.out_bstride + (pos << wil) + slot;
                    const uint32_t ks = lns + wil;
#pragma unroll
                    for (int k = 0; k < q; k++) st_stream<nt_stores(NTS)>(dst + ((uint64_t)(k * NB) << ks), v[u * q + k]);
                } else if constexpr (!BREV) {
                    // (ilv_log = 0: dst = out + bt out_bstride + pos + k NB 2^lns)
                    const uint32_t il = a.ilv_log;
                    const uint64_t rq = il ? (uint64_t)(__builtin_bitreverse32((uint32_t)bt) >> (32 - il)) : 0;
                    // (out_pad: the line block's offset in a padded workspace)
                    const uint64_t pad = (j >> a.out_pad_log) * a.out_pad;
                    C2* dst = out + (bt >> il) * a.out_bstride + rq + (pos << il) + pad;
                    const uint32_t ks = lns + il;
#pragma unroll
                    for (int k = 0; k < q; k++) st_stream<nt_stores(NTS)>(dst + ((uint64_t)(k * NB) << ks), v[u * q + k]);
                    if constexpr (serial && PIFFT_SERIAL_BFLY >= 2) __builtin_amdgcn_sched_barrier(0);
                } else {
                    C2* dst = out + bt * a.out_bstride;
                    const uint32_t sh = 64 - (log_lb + Sh::LOGR);  // log2 M bits
#pragma unroll
                    for (int k = 0; k < q; k++) {
                        const uint64_t pk = pos + ((uint64_t)(k * NB) << lns);
                        dst[sh < 64 ? __builtin_bitreverse64(pk) >> sh : 0] = v[u * q + k];
                    }
                }
            }
        }
    } else if constexpr (Stage<R, C, SM, S + 1, VPT>::perm) {
        // ---- exchange with the last stage across lanes (Stage::perm) ----
        // quadruple g: row m, register 4g+j holds element 256 m + 16 (4g+j) + i;
        // afterwards it holds element 256 j + 16 (4g+m) + i (input j of
        // butterfly 64 g + 16 m + i)
        if constexpr (Stage<R, C, SM, S + 1, VPT>::q == 4) {
#pragma unroll
            for (int g = 0; g < 4; g++) {
                pl_swap<32>(v[4 * g + 0], v[4 * g + 2]);
                pl_swap<32>(v[4 * g + 1], v[4 * g + 3]);
                pl_swap<16>(v[4 * g + 0], v[4 * g + 1]);
                pl_swap<16>(v[4 * g + 2], v[4 * g + 3]);
            }
        } else {
#pragma unroll
            for (int g = 0; g < 8; g++) pl_swap<16>(v[2 * g], v[2 * g + 1]);
        }
        pass_stages<T, R, C, MODE, NTS, LP, S + 1, VPT>(a, lds, v, pre, tid, tile, twp);
    } else if constexpr (PIFFT_DIAG_NO_XCHG && MODE != 11) {
        // diagnostics build only (timing, WRONG results): no hand-off at all --
        // the upper bound of what any register exchange (DPP, ds_swizzle,
        // permlane) could save on this pass (round 6, profiles/sessions/gpu_r06w.sh)
        pass_stages<T, R, C, MODE, NTS, LP, S + 1, VPT>(a, lds, v, pre, tid, tile, twp);
    } else {
        // ---- exchange with stage S+1 through LDS, one component at a time ----
        using Nx = Stage<R, C, SM, S + 1, VPT>;
#pragma unroll
        for (int comp = 0; comp < 2; comp++) {
            // (the tile's first LDS store has no earlier reader to wait for;
            // MODE 11's first stage has just read its inputs from LDS and
            // waited for every thread's reads)
            if (S > 0 || comp > 0) lds_handoff<Nx::wave_private>();
            const int tidc = tid;
#pragma unroll
            for (int u = 0; u < U; u++) {
                int c, b;
                St::map(tidc, u, c, b);
                const int base = (b / ns) * ns * q + (b & (ns - 1));  // r' = base + k ns
#pragma unroll
                for (int k = 0; k < q; k++) lds[lds_at(LL, c, base + k * ns)] = comp ? v[u * q + k].im : v[u * q + k].re;
            }
            lds_handoff<Nx::wave_private>();
#pragma unroll
            for (int u = 0; u < Nx::U; u++) {
                int c, b;
                Nx::map(tidc, u, c, b);
#pragma unroll
                for (int k = 0; k < Nx::q; k++) {
                    const T x = lds[lds_at(LL, c, b + k * Nx::NB)];
                    if (comp) v[u * Nx::q + k].im = x; else v[u * Nx::q + k].re = x;
                }
            }
        }
        pass_stages<T, R, C, MODE, NTS, LP, S + 1, VPT>(a, lds, v, pre, tid, tile, twp);
    }
}

// ---------------------------------------------------------------------------
// fp32 at 32 values per thread, packed (VPT 32): a 16384-value tile on 512
// threads (two workgroups per CU), i.e. the bytes and row-segment widths of
// the fp64 8192-value tile.  Each thread's butterflies u = 2m and 2m + 1 of a
// stage travel together in one register pair per component (cx<f2>: .x the
// even butterfly, .y the odd one), so their arithmetic is v_pk_add_f32 /
// v_pk_mul_f32 on pairs -- the same operations in the same order as two
// scalar butterflies (bitwise equal), with the register state of ONE fp64
// butterfly instead of two interleaved fp32 ones (the scalar VPT-32 form wants
// 174 VGPRs in MODE 2 and spills at 128).  Loads, stores and LDS exchanges
// address each half with the VPT-32 Stage map of its own butterfly.
// ---------------------------------------------------------------------------
// Diagnostics builds only (timing, WRONG results; never the product): the
// packed fp32 passes without their twiddles (PIFFT_DIAG_NO_TW=1: no table
// loads, no twiddle products) or without their butterflies
// (PIFFT_DIAG_NO_DFT=1), to split a pass's time between its data movement,
// LDS exchanges, twiddles and arithmetic (round 6, profiles/sessions/gpu_r06g.sh).
#ifndef PIFFT_DIAG_NO_TW
#define PIFFT_DIAG_NO_TW 0
#endif
#ifndef PIFFT_DIAG_NO_DFT
#define PIFFT_DIAG_NO_DFT 0
#endif
template <int q, typename V>
__device__ __forceinline__ void dft_diag(V* v) {
    if constexpr (!PIFFT_DIAG_NO_DFT) dft<q>(v);
}
#ifndef PIFFT_PK_SERIAL
#define PIFFT_PK_SERIAL 0  // packed passes: a scheduling barrier after each butterfly pair (tuning A/B)
#endif
#ifndef PIFFT_PK_REMAT
#define PIFFT_PK_REMAT 1  // packed VPT-32 exchanges: LDS addresses recomputed per component
#endif
using f2 = float __attribute__((ext_vector_type(2)));

template <int H>
__device__ __forceinline__ void pk_put(cx<f2>& d, cx<float> s) {
    if constexpr (H) {
        d.re.y = s.re;
        d.im.y = s.im;
    } else {
        d.re.x = s.re;
        d.im.x = s.im;
    }
}
template <int H>
__device__ __forceinline__ cx<float> pk_get(const cx<f2>& d) {
    if constexpr (H) return cx<float>{d.re.y, d.im.y};
    else return cx<float>{d.re.x, d.im.x};
}
__device__ __forceinline__ cx<f2> pk_pair(cx<float> a, cx<float> b) {
    cx<f2> r;
    r.re = f2{a.re, b.re};
    r.im = f2{a.im, b.im};
    return r;
}

template <int R, int C, int MODE, int NTS, int S>
__device__ __forceinline__ void pass_stages_packed(const PassArgs& a, float* lds, cx<f2>* vp, int tid, uint64_t tile,
                                                   cx<float>* twp) {
    using C1 = cx<float>;
    using CP = cx<f2>;
    constexpr int VPT = 32;
    constexpr int BM = MODE & 3;
    static_assert(BM == 1 || BM == 2, "packed VPT-32 passes: strided first / later passes");
    static_assert((MODE & ~3) == 0 && (NTS == 0 || NTS == 1), "no bit-reversed or interleaved forms");
    using St = Stage<R, C, BM, S, VPT>;
    using Sh = PassShape<R, VPT>;
    constexpr int q = St::q, U = St::U, NB = St::NB, ns = St::ns;
    static_assert(U % 2 == 0, "butterflies go in pairs");
    constexpr LdsLayout LL = LdsPick<float, R, C, BM, VPT>::value;
    const uint32_t log_lb = a.log_lb, log_ns = a.log_ns;
    const uint64_t lb_mask = (1ull << log_lb) - 1, ns_mask = (1ull << log_ns) - 1;
    constexpr bool share_anc = St::cfast && U > 1 && St::NT % C == 0;

    if constexpr (St::first) {
        if constexpr (BM == 2 && !PIFFT_DIAG_NO_TW) {
            const C1* tlo = static_cast<const C1*>(a.tw_lo);
            const C1* thi = static_cast<const C1*>(a.tw_hi);
            const uint64_t hmask = (1ull << a.tw_h) - 1;
#pragma unroll
            for (int u = 0; u < U; u++) {
                int c, b;
                St::map(tid, u, c, b);
                const uint64_t jm = (tile * C + c) & lb_mask & ns_mask;
                const uint64_t e0 = (jm * (uint64_t)NB) << a.tw_shift, e1 = (jm * (uint64_t)b) << a.tw_shift;
                if (!share_anc || u == 0) {
                    twp[4 * u + 0] = tlo[e0 & hmask];
                    twp[4 * u + 1] = thi[e0 >> a.tw_h];
                }
                twp[4 * u + 2] = tlo[e1 & hmask];
                twp[4 * u + 3] = thi[e1 >> a.tw_h];
            }
        }
        // ---- inputs straight from HBM (all loads issued before any use) ----
        const C1* __restrict__ in = static_cast<const C1*>(a.in);
        static_for<0, U, 1>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            int c, b;
            St::map(tid, u, c, b);
            const uint64_t line = tile * C + c < a.nlines ? tile * C + c : a.nlines - 1;
            const uint64_t bt = line >> log_lb, j = line & lb_mask;
            const uint32_t les = log_lb;
            if constexpr (BM == 2) {
                const uint64_t rs = (1ull << les) + a.in_pad;
                const C1* row = in + bt * a.in_bstride + j + (uint64_t)b * rs;
#pragma unroll
                for (int k = 0; k < q; k++)
                    pk_put<u & 1>(vp[(u >> 1) * q + k], ld_stream<nt_loads(NTS)>(row + (uint64_t)(k * NB) * rs));
            } else {
                const C1* src = in + bt * a.in_bstride + j + ((uint64_t)b << les);
#pragma unroll
                for (int k = 0; k < q; k++)
                    pk_put<u & 1>(vp[(u >> 1) * q + k], ld_stream<nt_loads(NTS)>(src + ((uint64_t)(k * NB) << les)));
            }
        });
    }
    // ---- twiddles and butterflies, one packed pair of butterflies at a time ----
    if constexpr (St::first && BM == 2 && !PIFFT_DIAG_NO_TW) {
        C1 anc0[4], anc1[4];
        if constexpr (share_anc) {
            anc0[0] = cmul(twp[1], twp[0]);
#pragma unroll
            for (int i = 1; (1 << i) < q; i++) anc0[i] = cmul(anc0[i - 1], anc0[i - 1]);
        }
#pragma unroll
        for (int m = 0; m < U / 2; m++) {
            if constexpr (!share_anc) {
                anc0[0] = cmul(twp[4 * (2 * m) + 1], twp[4 * (2 * m) + 0]);
                anc1[0] = cmul(twp[4 * (2 * m + 1) + 1], twp[4 * (2 * m + 1) + 0]);
#pragma unroll
                for (int i = 1; (1 << i) < q; i++) {
                    anc0[i] = cmul(anc0[i - 1], anc0[i - 1]);
                    anc1[i] = cmul(anc1[i - 1], anc1[i - 1]);
                }
            }
            CP ap[4];
#pragma unroll
            for (int i = 0; (1 << i) < q; i++) ap[i] = pk_pair(anc0[i], share_anc ? anc0[i] : anc1[i]);
            apply_powers<q>(&vp[m * q], ap);
            dft_diag<q>(&vp[m * q]);
            if constexpr (PIFFT_PK_SERIAL) __builtin_amdgcn_sched_barrier(0);
            const CP base = pk_pair(cmul(twp[4 * (2 * m) + 3], twp[4 * (2 * m) + 2]),
                                    cmul(twp[4 * (2 * m + 1) + 3], twp[4 * (2 * m + 1) + 2]));
#pragma unroll
            for (int k = 0; k < q; k++) vp[m * q + k] = cmul(vp[m * q + k], base);
        }
    } else if constexpr (!St::first && !PIFFT_DIAG_NO_TW) {
        // w_{ns q}^{(b mod ns) k} = w_R^{(b mod ns) k R/(ns q)}, per butterfly
        const C1* __restrict__ twr = static_cast<const C1*>(a.tw_r);
#pragma unroll
        for (int m = 0; m < U / 2; m++) {
            int c0, b0, c1, b1;
            St::map(tid, 2 * m, c0, b0);
            St::map(tid, 2 * m + 1, c1, b1);
            const int e0 = (b0 & (ns - 1)) * (R / (ns * q)), e1 = (b1 & (ns - 1)) * (R / (ns * q));
            CP ap[4];
#pragma unroll
            for (int i = 0; (1 << i) < q; i++) ap[i] = pk_pair(twr[e0 << i], twr[e1 << i]);
            apply_powers<q>(&vp[m * q], ap);
            dft_diag<q>(&vp[m * q]);
            if constexpr (PIFFT_PK_SERIAL) __builtin_amdgcn_sched_barrier(0);
        }
    } else {
#pragma unroll
        for (int m = 0; m < U / 2; m++) {
            dft_diag<q>(&vp[m * q]);
            if constexpr (PIFFT_PK_SERIAL) __builtin_amdgcn_sched_barrier(0);
        }
    }

    if constexpr (St::last) {
        // ---- outputs r' = b + k NB straight to HBM ----
        C1* __restrict__ out = static_cast<C1*>(a.out);
        static_for<0, U, 1>([&](auto uc) {
            constexpr int u = decltype(uc)::value;
            int c, b;
            St::map(tid, u, c, b);
            const uint64_t line = tile * C + c;
            if (line < a.nlines) {
                const uint64_t bt = line >> log_lb, j = line & lb_mask;
                const uint32_t lns = (uint32_t)log_ns;
                const uint64_t pos = ((j >> lns) << (lns + Sh::LOGR)) + (j & ((1ull << lns) - 1)) + ((uint64_t)b << lns);
                const uint64_t pad = (j >> a.out_pad_log) * a.out_pad;
                C1* dst = out + bt * a.out_bstride + pos + pad;
#pragma unroll
                for (int k = 0; k < q; k++)
                    st_stream<nt_stores(NTS)>(dst + ((uint64_t)(k * NB) << lns), pk_get<u & 1>(vp[(u >> 1) * q + k]));
            }
        });
    } else {
        // ---- exchange with stage S+1 through LDS, one component at a time ----
        using Nx = Stage<R, C, BM, S + 1, VPT>;
        static_assert(Nx::U % 2 == 0, "butterflies go in pairs");
#pragma unroll
        for (int comp = 0; comp < 2; comp++) {
            if (S > 0 || comp > 0) __syncthreads();
            // the second component recomputes its LDS addresses from an opaque
            // copy of tid instead of keeping the first's 2 x 32 addresses live
            // beside the 64 data registers (they spilled 52 B per lane in the
            // 1024-point MODE 2 instance)
            int tidc = tid;
            if (PIFFT_PK_REMAT && comp) asm volatile("" : "+v"(tidc));
            static_for<0, U, 1>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                int c, b;
                St::map(tidc, u, c, b);
                const int base = (b / ns) * ns * q + (b & (ns - 1));  // r' = base + k ns
#pragma unroll
                for (int k = 0; k < q; k++) {
                    const C1 x = pk_get<u & 1>(vp[(u >> 1) * q + k]);
                    lds[lds_at(LL, c, base + k * ns)] = comp ? x.im : x.re;
                }
            });
            __syncthreads();
            static_for<0, Nx::U, 1>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                int c, b;
                Nx::map(tidc, u, c, b);
#pragma unroll
                for (int k = 0; k < Nx::q; k++) {
                    const float x = lds[lds_at(LL, c, b + k * Nx::NB)];
                    CP& d = vp[(u >> 1) * Nx::q + k];
                    if (comp) {
                        if constexpr (u & 1) d.im.y = x; else d.im.x = x;
                    } else {
                        if constexpr (u & 1) d.re.y = x; else d.re.x = x;
                    }
                }
            });
        }
        pass_stages_packed<R, C, MODE, NTS, S + 1>(a, lds, vp, tid, tile, twp);
    }
}

#ifndef PIFFT_PACK32
#define PIFFT_PACK32 1  // VPT-32 fp32 instances: the packed form (0: the scalar form, which spills)
#endif
// inter-pass twiddle entries fetched with a tile's first-stage loads (MODE 2)
template <int R, int C, int MODE, int VPT>
constexpr int first_tw_count() {
    return (MODE & 3) == 2 ? 4 * Stage<R, C, 2, 0, VPT>::U : 1;
}


// MODE 0: single pass (lines contiguous in and out, no inter-pass twiddle)
// MODE 1: first pass of several (lines strided in, contiguous out, no twiddle)
// MODE 2: later pass (strided in and out, inter-pass twiddle)
// MODE 3: first pass with the tree stage fused in (one worker, P = 2^LP):
//         each input v_r = z_q[j + r M/R] is evaluated from its P leaves
// MODE 4 / 6: MODE 0 / 2 storing in bit-reversed order (PIFFT_OUT_BITREV)
// NTS: non-temporal streaming of the data (nt_loads / nt_stores)
template <typename T, int R, int C, int MODE, int NTS, int LP, int VPT = 16>
__global__ __launch_bounds__((PassCfg<R, C, VPT>::NT), (pass_waves_per_eu<T, R, C, MODE, LP, VPT>()))
void k_pass(PassArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char pifft_smem[];
    constexpr int Q = PassShape<R, VPT>::Q;
    constexpr int TWN = first_tw_count<R, C, MODE, VPT>();
    cx<T> pre[pre_count<R, C, stage_mode(MODE), VPT>() > 0 ? pre_count<R, C, stage_mode(MODE), VPT>() : 1];
    // one tile per workgroup: a persistent tile loop (1, 2 or 4 resident
    // workgroups per CU walking the tiles) measured 1.4-1.7x slower at 2^28
    // fp64
    uint64_t tile = tile_of_block(blockIdx.x, a.log_xg, gridDim.x);
    T* lds = reinterpret_cast<T*>(pifft_smem);
    const int tid = (int)threadIdx.x;
#ifdef PIFFT_WG_CLOCK
    if (a.wg_clock && tid == 0) a.wg_clock[PIFFT_WGC_WORDS * blockIdx.x] = wall_clock64();
#endif
    if constexpr (VPT == 32 && std::is_same_v<T, float> && PIFFT_PACK32) {
        cx<f2> vp[PassShape<R, VPT>::Q / 2];
        cx<float> twp[TWN];
        pass_stages_packed<R, C, MODE, NTS, 0>(a, reinterpret_cast<float*>(pifft_smem), vp, tid, tile, twp);
        (void)pre;
        (void)lds;
    } else {
        if (a.ilv_log && a.log_lb >= (uint32_t)ilog2c(C)) {
            // natural-order store: the P workers' tiles of one line block run
            // back to back (and on one XCD, log_xg >= log2 P), so the P 16-B
            // pieces of each output line meet in one L2 before it is written
            const uint32_t il = a.ilv_log, ltt = a.log_lb - (uint32_t)ilog2c(C);  // 2^ltt tiles per transform
            const uint64_t q = tile & ((1ull << il) - 1), rest = tile >> il;
            tile = ((rest >> ltt) << (il + ltt)) + (q << ltt) + (rest & ((1ull << ltt) - 1));
        }
        cx<T> v[Q];
        cx<T> twp[TWN];
        pass_stages<T, R, C, MODE, NTS, LP, 0, VPT>(a, lds, v, pre, tid, tile, twp);
    }
#ifdef PIFFT_WG_CLOCK
    if (a.wg_clock) {
        __builtin_amdgcn_s_waitcnt(0);  // this thread's stores are done
        __syncthreads();
        if (tid == 0) {
            a.wg_clock[PIFFT_WGC_WORDS * blockIdx.x + 1] = wall_clock64();
            a.wg_clock[PIFFT_WGC_WORDS * blockIdx.x + 2] = __smid();
        }
    }
#endif
}

// ---------------------------------------------------------------------------
// Tree ("funnel") stage
// ---------------------------------------------------------------------------
// Levels t0 .. t0+L-1 of the reference's radix-2 tree (CPU.c:419-448, level t
// = butterflies of size N >> t) in "position space": the reference's scratch
// layout, where after all log2 P levels worker q's segment sits at
// [q N/P, (q+1) N/P).  A thread owns 2^L positions base + i + m*D
// (D = N >> (t0+L)), which only interact with each other in these levels, so
// one launch applies L levels in registers and writes the same positions back
// (in place).  Only branches leading to workers [q0, q0+nq) are evaluated and
// stored; the last launch writes slice-major (out_shift = -q0 N/P).
struct TreeArgs {
    const void* in;
    void* out;
    TreeTw tw;
    uint64_t in_bstride;    // N
    uint64_t out_bstride;   // N (position space) or nq * N/P (slice-major)
    int64_t out_shift;      // 0 or -q0 * N/P
    uint64_t total;         // transforms * (N >> L)
    uint32_t log_n, log_p, t0;
    uint32_t q0, nq;        // workers [q0, q0+nq)
};

template <typename T, int L>
__global__ __launch_bounds__(256) void k_tree(TreeArgs a) {
    using C2 = cx<T>;
    constexpr int V = 1 << L;
    // grid-stride: the work-item count of one launch must stay below 2^32
    for (uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < a.total;
         gid += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t log_g = a.log_n - L;            // threads per transform = 2^log_g
    const uint32_t log_d = a.log_n - a.t0 - L;     // D = stride between a thread's positions
    const uint64_t g = gid & ((1ull << log_g) - 1), bt = gid >> log_g;
    const uint64_t blk0 = g >> log_d, i = g & ((1ull << log_d) - 1);
    const uint64_t base = blk0 << (a.log_n - a.t0);
    const uint32_t log_w = a.log_p - a.t0 - L;     // workers below one level-(t0+L) block
    const uint64_t q0 = a.q0, q1 = (uint64_t)a.q0 + a.nq;
    const uint64_t w_lo = (blk0 << L) << log_w, w_hi = ((blk0 + 1) << L) << log_w;
    if (w_hi <= q0 || w_lo >= q1) continue;  // no requested worker below this group
    // no __restrict__ on src/dst: launches after the first of a multi-launch
    // tree (log2 P > 4) run in place (src == dst == the plan's tree buffer);
    // each thread reads and writes only its own 2^L positions
    const C2* src = static_cast<const C2*>(a.in) + bt * a.in_bstride + base + i;
    C2 v[V];
#pragma unroll
    for (int m = 0; m < V; m++) v[m] = src[(uint64_t)m << log_d];
    tree_levels<T, L>(v, a.tw, i, log_d, a.t0, blk0, log_w, q0, q1);
    C2* dst = static_cast<C2*>(a.out) + bt * a.out_bstride + (int64_t)(base + i) + a.out_shift;
#pragma unroll
    for (int m = 0; m < V; m++) {
        const uint64_t wm = ((blk0 << L) + m) << log_w;
        if (wm < q1 && wm + (1ull << log_w) > q0) dst[(uint64_t)m << log_d] = v[m];
    }
    }  // grid-stride
}

// The single launch of an all-worker tree (t0 = 0, all P = 2^L workers)
// writing the worker-interleaved layout of the passes (PassArgs::wil):
// z_q[i] at bt out_bstride + i P + q.  A block's 256 threads own 256
// consecutive i -- one contiguous run of 256 P outputs (M = N / P >= 256) --
// staged through LDS (one pad value per 8) so that every store instruction
// writes 64 consecutive values instead of 64 pieces P values apart.
// Dynamic LDS: 256 P (9/8) values.
__host__ __device__ constexpr uint32_t tree_wil_pad(uint32_t idx) { return idx + (idx >> 3); }
template <typename T, int L>
__global__ __launch_bounds__(256) void k_tree_wil(TreeArgs a) {
    using C2 = cx<T>;
    constexpr int V = 1 << L;
    extern __shared__ __attribute__((aligned(16))) unsigned char pifft_smem[];
    C2* stage = reinterpret_cast<C2*>(pifft_smem);
    const uint32_t log_d = a.log_n - L;  // 2^log_d = M threads per transform
    const uint64_t nblk = (a.total + 255) / 256;
    // (block-uniform loop: every thread of a block reaches the barriers)
    for (uint64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
        const uint64_t g0 = blk * 256, gid = g0 + threadIdx.x;
        const uint64_t g = gid < a.total ? gid : a.total - 1;
        const uint64_t bt = g >> log_d, i = g & ((1ull << log_d) - 1);
        const C2* src = static_cast<const C2*>(a.in) + bt * a.in_bstride + i;
        C2 v[V];
#pragma unroll
        for (int m = 0; m < V; m++) v[m] = src[(uint64_t)m << log_d];
        tree_levels<T, L>(v, a.tw, i, log_d, 0, 0, 0, 0, V);
        __syncthreads();  // the previous round's reads of `stage` are done
#pragma unroll
        for (int m = 0; m < V; m++) stage[tree_wil_pad(threadIdx.x * V + m)] = v[m];
        __syncthreads();
        const uint64_t b0 = g0 >> log_d, i0 = g0 & ((1ull << log_d) - 1);
        C2* dst = static_cast<C2*>(a.out) + b0 * a.out_bstride + (i0 << L);
        const uint64_t nvalid = (a.total - g0 < 256 ? a.total - g0 : 256) * V;
#pragma unroll
        for (int k = 0; k < V; k++) {
            const uint32_t idx = (uint32_t)k * 256 + threadIdx.x;
            if (idx < nvalid) dst[idx] = stage[tree_wil_pad(idx)];
        }
    }
}

// ---------------------------------------------------------------------------
// slice-major -> natural order: out[bt N + bitrev_P(q) + P k] = in[bt N + q M + k]
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_interleave(const cx<T>* __restrict__ in,
                                                    cx<T>* __restrict__ out, uint64_t total,
                                                    uint32_t log_n, uint32_t log_p) {
    const uint64_t n = 1ull << log_n;
    for (uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; gid < total;
         gid += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t bt = gid >> log_n, o = gid & (n - 1);
        const uint64_t k = o >> log_p;
        const uint32_t rr = (uint32_t)(o & ((1ull << log_p) - 1));
        const uint32_t q = log_p ? (__builtin_bitreverse32(rr) >> (32 - log_p)) : 0u;
        out[gid] = in[bt * n + ((uint64_t)q << (log_n - log_p)) + k];
    }
}

// The same through an LDS tile of all P slices x K = 2048/P consecutive k
// (P <= 2048): every slice is read in runs of K elements (>= 256 B for
// P <= 128 at fp64) and the tile's 2048 outputs out[P k + r] are one
// contiguous block -- instead of P different rows per wave instruction
// (k_interleave: 16-B pieces for P >= 64).  Measured on MI355X
// (profiles/r02_interleave_ab.log): fp64 2^28 P = 64 4.05 -> 1.55 ms, 2^24
// P = 256 0.34 -> 0.09 ms, fp32 2^24 P = 8 0.053 -> 0.044 ms; for fp64 P <= 16
// k_interleave is as fast or faster (2^28 P = 8: 1.52 vs 1.62 ms).
constexpr int IL_TILE = 2048;
template <typename T>
__global__ __launch_bounds__(256) void k_interleave_tile(const cx<T>* __restrict__ in, cx<T>* __restrict__ out,
                                                         uint64_t total, uint32_t log_n, uint32_t log_p) {
    __shared__ cx<T> tile[IL_TILE + IL_TILE / 16];
    const uint32_t log_k = 11 - log_p;  // K = 2048 / P
    const uint32_t log_m = log_n - log_p;
    const uint64_t ntiles = total >> 11;
    const uint32_t P = 1u << log_p;
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t e0 = t << 11;  // first output of the tile
        const uint64_t bt = e0 >> log_n, k0 = (e0 & ((1ull << log_n) - 1)) >> log_p;
        const cx<T>* src = in + (bt << log_n) + k0;
        __syncthreads();  // the previous tile's reads are done
#pragma unroll
        for (int i = 0; i < IL_TILE / 256; i++) {
            const uint32_t e = threadIdx.x + i * 256;
            const uint32_t q = e >> log_k, k = e & ((1u << log_k) - 1);
            const uint32_t r = log_p ? (__builtin_bitreverse32(q) >> (32 - log_p)) : 0u;
            const uint32_t o = (k << log_p) + r;  // natural position within the tile
            tile[o + (o >> 4)] = src[((uint64_t)q << log_m) + k];
        }
        __syncthreads();
        cx<T>* dst = out + e0;
#pragma unroll
        for (int i = 0; i < IL_TILE / 256; i++) {
            const uint32_t o = threadIdx.x + i * 256;
            dst[o] = tile[o + (o >> 4)];
        }
        (void)P;
    }
}

// ---------------------------------------------------------------------------
// synthetic input (bit-identical to oracle_generate_*)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t splitmix64(uint64_t seed, uint64_t draw) {
    uint64_t z = seed + (draw + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <typename T>
__global__ __launch_bounds__(256) void k_generate(cx<T>* __restrict__ x, uint64_t count,
                                                  double scale, uint64_t seed, uint64_t first) {
    for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < count;
         e += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t d = 2 * (first + e);
        const double ur = (double)(splitmix64(seed, d) >> 11) * 0x1.0p-53;
        const double ui = (double)(splitmix64(seed, d + 1) >> 11) * 0x1.0p-53;
        x[e] = cx<T>{(T)((2.0 * ur - 1.0) / scale), (T)((2.0 * ui - 1.0) / scale)};
    }
}

}  // namespace pifft
