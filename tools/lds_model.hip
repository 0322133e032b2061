// tools/lds_model.hip -- LDS bank-conflict model of the k_pass exchanges, and
// the per-instance layout search that generates
// cs87project-msolano2_amd/csrc/pifft_lds_layouts.inc.
//
// Host-only (runs here, no GPU).  Every LDS exchange of a pass instance is
// replayed through the kernel's own thread -> (line, element) maps
// (Stage::map, pifft_kernels.h) and the addressing of pass_stages: stage S
// writes element base + k ns of line c, stage S+1 reads b + k NB.  Each wave
// instruction is costed with the gfx950 LDS rules (MI355X_MICROARCH.md, LDS):
//   ds_write_b64: lane groups 4 x 16, bank = dword mod 32, 1 array cycle/group
//   ds_read_b64 : lane groups 2 x 32, bank = dword mod 64
//   ds_write_b32 / ds_read_b32: lane groups 2 x 32, bank = dword mod 32
// a group takes as many array cycles as the most distinct dwords on one bank
// (identical addresses broadcast); extra = cycles - 1 is what
// SQ_LDS_BANK_CONFLICT counts, base + extra what SQ_LDS_IDX_ACTIVE counts.
// (ds_write2_b64 pairs bank like two ds_write_b64.)
//
//   ./lds_model report          model ratio of the default and the picked layouts
//   ./lds_model gen <out.inc> [part nparts]   search and write the LdsPick
//                                specializations (of every nparts-th instance)
#define PIFFT_LDS_DEFAULT_ONLY 1
#include "../cs87project-msolano2_amd/csrc/pifft_kernels.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace pifft;

struct Cost {
    long base = 0, extra = 0;
    double ratio() const { return base + extra ? (double)extra / (double)(base + extra) : 0.0; }
};

// one wave instruction of an exchange: lane l touches element r[l] of line
// c[l] (c < 0: lane inactive)
struct Instr {
    bool write;
    int c[64], r[64];
};

static void cost_instr(Cost& cost, const Instr& in, LdsLayout L, int esz) {
    const int gsize = (esz == 8 && in.write) ? 16 : 32;
    const int mod = (esz == 8 && !in.write) ? 64 : 32;
    const int nd = esz / 4;
    for (int g = 0; g < 64; g += gsize) {
        // distinct dwords per bank within the lane group
        long dws[64];
        int nb[64] = {0};
        long seen[64][8];
        bool any = false;
        int worst = 1;
        (void)dws;
        for (int l = g; l < g + gsize; l++) {
            if (in.c[l] < 0) continue;
            any = true;
            const long a = (long)lds_at(L, in.c[l], in.r[l]) * nd;  // dword address
            for (int d = 0; d < nd; d++) {
                const long dw = a + d;
                const int bk = (int)(dw % mod);
                bool dup = false;
                for (int i = 0; i < nb[bk] && i < 8; i++) dup |= seen[bk][i] == dw;
                if (!dup) {
                    if (nb[bk] < 8) seen[bk][nb[bk]] = dw;
                    nb[bk]++;
                    if (nb[bk] > worst) worst = nb[bk];
                }
            }
        }
        if (!any) continue;
        cost.base += 1;
        cost.extra += worst - 1;
    }
}

template <typename T, int R, int C, int MODE, int S, int VPT>
static void exchanges(std::vector<Instr>& out) {
    using St = Stage<R, C, MODE, S, VPT>;
    if constexpr (!St::last) {
        using Nx = Stage<R, C, MODE, S + 1, VPT>;
        if constexpr (!Nx::perm) {
            constexpr int NT = St::NT;
            for (int w = 0; w * 64 < NT; w++) {
                for (int u = 0; u < St::U; u++)
                    for (int k = 0; k < St::q; k++) {
                        Instr in;
                        in.write = true;
                        for (int l = 0; l < 64; l++) {
                            const int tid = w * 64 + l;
                            in.c[l] = -1;
                            if (tid >= NT) continue;
                            int c, b;
                            St::map(tid, u, c, b);
                            in.c[l] = c;
                            in.r[l] = (b / St::ns) * St::ns * St::q + (b & (St::ns - 1)) + k * St::ns;
                        }
                        out.push_back(in);
                    }
                for (int u = 0; u < Nx::U; u++)
                    for (int k = 0; k < Nx::q; k++) {
                        Instr in;
                        in.write = false;
                        for (int l = 0; l < 64; l++) {
                            const int tid = w * 64 + l;
                            in.c[l] = -1;
                            if (tid >= NT) continue;
                            int c, b;
                            Nx::map(tid, u, c, b);
                            in.c[l] = c;
                            in.r[l] = b + k * Nx::NB;
                        }
                        out.push_back(in);
                    }
            }
        }
        exchanges<T, R, C, MODE, S + 1, VPT>(out);
    }
}

// the layout maps (c < C, r < R) one-to-one into [0, C ls)
static bool valid(LdsLayout L, int R, int C) {
    std::vector<char> used((size_t)C * L.ls, 0);
    for (int c = 0; c < C; c++)
        for (int r = 0; r < R; r++) {
            const int a = lds_at(L, c, r);
            if (a < 0 || a >= C * L.ls || used[a]) return false;
            used[a] = 1;
        }
    return true;
}

struct Inst {
    const char* tname;
    int esz, R, C, mode, vpt;
    void (*fn)(std::vector<Instr>&);
};

template <typename T, int R, int C, int MODE, int VPT>
static void list(std::vector<Instr>& v) {
    exchanges<T, R, C, MODE, 0, VPT>(v);
}

#define I(T, R, C, M, V) Inst{#T, (int)sizeof(T), R, C, M, V, &list<T, R, C, M, V>}
// every (precision, R, C, mode) with an LDS exchange that the instance tables hold
static std::vector<Inst> instances() {
    std::vector<Inst> v;
#include "lds_model_instances.inc"
    return v;
}

static Cost evaluate(const std::vector<Instr>& ins, LdsLayout L, int esz) {
    Cost c;
    for (const Instr& in : ins) cost_instr(c, in, L, esz);
    c.base *= 2;  // two components (re, im) per exchange, same pattern
    c.extra *= 2;
    return c;
}

static LdsLayout lds_default_of(int R) { return LdsLayout{R + R / 16 + 1, 4, 0, 4, 0, 0}; }

static LdsLayout search(const Inst& in, const std::vector<Instr>& ins, Cost& best_cost) {
    LdsLayout best = lds_default_of(in.R);
    best_cost = evaluate(ins, best, in.esz);
    const int max_ls = best.ls;  // never more LDS than the default
    for (int ps : {0, 4, 5})
        for (int xs = 3; xs <= 6; xs++)
            for (int xm = 0; xm < 8; xm++) {
                if (xm >= (1 << xs)) continue;
                if (xm == 0 && xs != 3) continue;  // one no-XOR candidate per ps
                const int pad = ps ? in.R >> ps : 0;
                for (int dd = 0; dd <= 33; dd++) {
                    LdsLayout L{in.R + pad + dd, xs, xm, ps, 0, 0};
                    if (L.ls > max_ls) continue;
                    const Cost c = evaluate(ins, L, in.esz);
                    const long t = c.base + c.extra, tb = best_cost.base + best_cost.extra;
                    if ((t < tb || (t == tb && L.ls < best.ls)) && valid(L, in.R, in.C)) {
                        best = L;
                        best_cost = c;
                    }
                }
            }
    // still conflicted: add a per-line XOR of the bank bits ((c & cm) << cs)
    if (best_cost.extra > 0)
        for (int ps : {0, 4, 5})
            for (int xs = 3; xs <= 6; xs++)
                for (int xm = 0; xm < 8; xm++) {
                    if (xm >= (1 << xs) || (xm == 0 && xs != 3)) continue;
                    for (int cm : {1, 3, 7, 15})
                        for (int cs = 0; cs <= 5; cs++) {
                            if ((cm << cs) >= in.R) continue;
                            const int pad = ps ? in.R >> ps : 0;
                            for (int dd = 0; dd <= 33; dd++) {
                                LdsLayout L{in.R + pad + dd, xs, xm, ps, cm, cs};
                                if (L.ls > max_ls) continue;
                                const Cost c = evaluate(ins, L, in.esz);
                                const long t = c.base + c.extra, tb = best_cost.base + best_cost.extra;
                                if ((t < tb || (t == tb && L.ls < best.ls)) && valid(L, in.R, in.C)) {
                                    best = L;
                                    best_cost = c;
                                }
                            }
                        }
                }
    return best;
}

int main(int argc, char** argv) {
    const std::string cmd = argc > 1 ? argv[1] : "report";
    FILE* out = nullptr;
    if (cmd == "gen") {
        out = fopen(argc > 2 ? argv[2] : "pifft_lds_layouts.inc", "w");
        if (!out) return 1;
        if (argc <= 4)
            fprintf(out, "// generated by tools/lds_model.hip (tools/gen_lds_layouts.sh) -- LdsPick specializations:\n"
                         "// per pass instance, the LDS layout with the fewest modelled LDS-array cycles\n"
                         "// (bank conflicts) at no more LDS than lds_default; instances not listed keep it.\n");
    }
    const int part = argc > 4 ? atoi(argv[3]) : 0, nparts = argc > 4 ? atoi(argv[4]) : 1;
    int idx = -1;
    for (const Inst& in : instances()) {
        if (++idx % nparts != part) continue;
        std::vector<Instr> ins;
        in.fn(ins);
        const Cost c0 = evaluate(ins, lds_default_of(in.R), in.esz);
        Cost cb;
        const LdsLayout b = search(in, ins, cb);
        printf("%-6s R=%5d C=%2d mode=%d vpt=%2d  default %.3f (%ld+%ld)  best %.3f (%ld+%ld) ls=%d xs=%d xm=%d ps=%d cm=%d cs=%d\n",
               in.tname, in.R, in.C, in.mode, in.vpt, c0.ratio(), c0.base, c0.extra, cb.ratio(), cb.base, cb.extra, b.ls, b.xs,
               b.xm, b.ps, b.cm, b.cs);
        fflush(stdout);
        // (VPT 32, the packed fp32 passes: modelled since round 6 and reported,
        // but their searched layouts -- fp32 last pass 43 -> 20 % conflict
        // cycles -- ran no faster on MI355X (fp32 2^28 2.47 vs 2.49 ms,
        // profiles/r06f_ab_fp32_2e28.txt): they keep the default layout)
        if (out && in.vpt != 32 && cb.base + cb.extra < c0.base + c0.extra)
            fprintf(out, "template <> struct LdsPick<%s, %d, %d, %d, %d> { static constexpr LdsLayout value{%d, %d, %d, %d, %d, %d}; };\n",
                    in.tname, in.R, in.C, in.mode, in.vpt, b.ls, b.xs, b.xm, b.ps, b.cm, b.cs);
    }
    if (out) fclose(out);
    return 0;
}
