"""Generates cs87project-msolano2_amd/csrc/pifft_instances_{0..NPART-1}.inc:
the k_pass<T, R, C, MODE, NTS, LP> instantiations the planner may pick,
spread over NPART translation units (compiled in parallel).

Rules: NT = C*R/VPT threads (VPT = 16 values per thread) <= 1024; LDS = C*(R + R/16 + 1)*sizeof(T)
<= 160 KiB.  MODE 0 single pass (any C); MODE 1/2 strided passes (C >= 4);
MODE 10 = MODE 2 on the worker-interleaved layout (all-worker plans); MODE 11 =
MODE 3 on it (the tree fused into an all-worker plan's first pass).
MODE 3 = MODE 1 with the tree fused in, LP = log2 P in 1..4, at the planner's
tile (8192 elements, both precisions) and C = 4.  MODE 4 / 6 = MODE 0 / 2
storing in bit-reversed order (the last pass of a PIFFT_OUT_BITREV plan), for
the C the planner can pick (C <= its tile / R).  NTS: 0 plain, 1 non-temporal
loads and stores, 2 / 3 non-temporal loads / stores only (MODE 2 at the
planner's tile: the halves of a chunked pass pair)."""
import os

NPART = 8
items = []
for T, prec, esz, tile, vpt in (("double", 64, 8, 8192, 16), ("float", 32, 4, 16384, 16)):
    for lr in range(1, 15):
        R = 1 << lr
        for C in (1, 2, 4, 8, 16, 32, 64):
            if R <= 8 and C != 64:
                continue
            Q = vpt if R >= vpt else min(R, 16)
            nt = C * R // Q
            lds = C * (R + R // 16 + 1) * esz if R > 16 else 0
            if nt > 1024 or lds > 160 * 1024:
                continue
            for nts in (0, 1):
                items.append(f"PK({T}, {prec}, {R}, {C}, 0, {nts}, 0),")
                if C <= max(1, 4096 // R) or R <= 8:
                    items.append(f"PK({T}, {prec}, {R}, {C}, 4, {nts}, 0),")
                if 16 <= R <= 4096 and C >= 4:
                    items.append(f"PK({T}, {prec}, {R}, {C}, 1, {nts}, 0),")
                    items.append(f"PK({T}, {prec}, {R}, {C}, 2, {nts}, 0),")
                    if C <= max(4, tile // R):
                        items.append(f"PK({T}, {prec}, {R}, {C}, 6, {nts}, 0),")
                        # MODE 10 = 2 | 8: the worker-interleaved layout of
                        # all-worker plans (multi-pass local FFTs: R <= 1024)
                        if R <= 1024:
                            items.append(f"PK({T}, {prec}, {R}, {C}, 10, {nts}, 0),")
                    # chunked pass pairs (nt loads only / nt stores only) at
                    # the planner's tile
                    # (and the 4096-value tile of fp64 R <= 256 later passes)
                    if nts == 1 and 64 <= R and (C == 8192 // R or (T == "double" and R <= 256 and C == 4096 // R)):
                        items.append(f"PK({T}, {prec}, {R}, {C}, 2, 2, 0),")
                        items.append(f"PK({T}, {prec}, {R}, {C}, 2, 3, 0),")
                # the planner's first-pass tile (tile_elems(): 8192 values for both precisions)
                # (and at half that C for R <= 256: the planner halves C to keep >= 512
                # workgroups on small local sizes, e.g. 2^21 = 128 x 128 x 128)
                cf = max(4, min(64, 8192 // R))
                if 16 <= R <= 2048 and (C == 4 or C == cf or (R <= 256 and C == cf // 2)):
                    for lp in (1, 2, 3, 4):
                        items.append(f"PK({T}, {prec}, {R}, {C}, 3, {nts}, {lp}),")
# the fused tree + first pass of an all-worker plan (PIFFT_FUSE_ALL_MAX_MIB:
# the input stays in the Infinity Cache, each worker's lines re-read its P
# leaves) at the C the planner picks for 2^18-2^22 (>= 512 workgroups)
for T, prec in (("double", 64), ("float", 32)):
    for R in (128, 256, 512, 1024):
        for C in (8, 16):
            if C == max(4, min(64, 8192 // R)) or (R <= 256 and C == max(4, min(64, 8192 // R)) // 2):
                continue  # already instantiated above
            for nts in (0, 1):
                for lp in (1, 2, 3, 4):
                    items.append(f"PK({T}, {prec}, {R}, {C}, 3, {nts}, {lp}),")
# MODE 11 = 3 | 8: the tree fused into the first pass of an all-worker plan in
# the worker-interleaved layout (PIFFT_WIL_FUSE), P = 4..16, C >= 8 lines (a
# whole number of P-worker line blocks) at tiles of <= 8192 values
for T, prec in (("double", 64), ("float", 32)):
    for R in (128, 256, 512, 1024):
        for C in (8, 16, 32, 64):
            if R * C > 8192:
                continue
            for nts in (0, 1):
                for lp in (2, 3, 4):
                    items.append(f"PK({T}, {prec}, {R}, {C}, 11, {nts}, {lp}),")
# two sub-tiles per workgroup (k_pass H = 2, one workgroup per CU): the
# 2^28 three-pass plans' strided passes with twice the lines per workgroup on
# the read side (PIFFT_SUBTILES)
for T, prec in (("double", 64), ("float", 32)):
    for R, C in ((1024, 8), (512, 16)):
        for mode in (1, 2):
            items.append(f"PKVH({T}, {prec}, {R}, {C}, {mode}, 1, 0, 16, 2),")
# fp64 strided passes at C = 2 for the latency-bound 2^20 sizes (two
# workgroups of 128 threads per CU instead of one of 256: PIFFT_STRIDED_CMIN=2)
for R in (512, 1024, 2048):
    for nts in (0, 1):
        for mode in (1, 2):
            items.append(f"PK(double, 64, {R}, 2, {mode}, {nts}, 0),")
# fp32 strided passes at 32 values per thread: a 16384-value tile (the bytes
# and row-segment widths of the fp64 8192-value tile) on 512 threads, two
# workgroups per CU (PIFFT_VPT32; three passes 1024-512-512 at 2^28)
# (R = 512 and 1024: the radices of 2^27-2^30 three-pass plans; 256 and 2048
# spill 44-100 B per lane in this form)
for R in (512, 1024):
    C = 16384 // R
    for nts in (0, 1):
        for mode in (1, 2):
            items.append(f"PKV(float, 32, {R}, {C}, {mode}, {nts}, 0, 32),")
# (8 values per thread -- PKV(..., 8), radix-8 stages -- measured slower than
# 16 for every single pass and batch tried, fp32 4096 x 128..4096 and fp64
# 2^12 / 2^13 x 1..1024 (profiles/r02_vpt_sweep.log): not instantiated)
d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cs87project-msolano2_amd", "csrc")
for k in range(NPART):
    with open(os.path.join(d, f"pifft_instances_{k}.inc"), "w") as f:
        f.write(f"// generated by tools/gen_instances.py -- part {k} of {NPART}\n")
        f.write("\n".join(items[k::NPART]) + "\n")
old = os.path.join(d, "pifft_instances.inc")
if os.path.exists(old):
    os.remove(old)
print(len(items), "instances in", NPART, "parts")
