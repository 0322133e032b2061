"""Host-side planning (pifft_plan_dry_run: no device needed) for the
BASELINE.json configurations and the edge cases -- the launch structure the
GPU tests then execute."""
import pytest

import pifft

F64, F32 = pifft.F64, pifft.F32
GiB = 1 << 30


def test_config1_2e20_fp64_one_worker():
    d = pifft.dry_run(1 << 20, 1, 1, F64)
    assert d["launch_kind"] == ["pass"] * d["num_passes"] and d["num_passes"] == 2
    assert d["radix"] == [1024, 1024]


def test_config2_2e20_fp64_eight_workers_one_gpu(monkeypatch):
    d = pifft.dry_run(1 << 20, 8, 1, F64)
    # the worker-interleaved layout with every worker's tree fused into the
    # first pass (MODE 11: 4 adjacent line indices x 8 workers at the 4096-value
    # tile -- 256 workgroups --, first radix 128), the last pass storing
    # natural order itself: two launches
    assert d["worker_interleaved"] and d["launch_kind"] == ["tree+pass", "pass"]
    assert d["launch_mode"] == [11, 10] and d["radix"] == [128, 1024] and d["lines"] == [32, 8]
    assert d["local_n"] == 1 << 17 and d["out_elems"] == 1 << 20
    assert d["launch_bytes"] == [2 * (1 << 20) * 16] * 2  # each leaf read once, every value written once
    monkeypatch.setenv("PIFFT_WIL_FUSE", "0")  # the tree as its own launch
    assert pifft.dry_run(1 << 20, 8, 1, F64)["launch_kind"] == ["tree", "pass", "pass"]


def test_fused_all_worker_rule():
    """Which all-worker plans fuse the tree into the first pass (MODE 11) and
    at which J (the tile's adjacent line indices: first radix tile / (J P)) --
    the planner's measured rule (profiles/r05m_wil_fuse_j.log; the 4096-value
    tile and J = 4 refinements: r05s-u_*)."""
    def first(n, P, prec, b=1):
        d = pifft.dry_run(n, P, b, prec)
        return d["launch_mode"][0], d["radix"][0], d["lines"][0]
    assert first(1 << 21, 8, F64) == (11, 128, 64)     # fp64 P <= 8: J = 8
    assert first(1 << 28, 8, F64) == (11, 128, 64)
    assert first(1 << 21, 2, F64) == (11, 512, 16)
    assert first(1 << 23, 16, F64)[0] == 0               # fp64 P = 16 below 256 MiB: the tree launch
    assert first(1 << 22, 16, F64) == (11, 256, 32)     # ... but J = 2 at 32-64 MiB
    assert first(1 << 28, 16, F64) == (11, 64, 128)     # ... and from 256 MiB fused
    assert first(1 << 21, 2, F32) == (11, 512, 16)      # fp32 up to 32 MiB: J = 8
    assert first(1 << 24, 8, F32) == (11, 64, 128)      # up to 1 GiB: J = 16
    assert first(1 << 28, 8, F32)[0] == 0                # beyond: the tree launch
    # fewer than 256 workgroups at the 8192-value tile (<= 2^20 values): the
    # 4096-value tile at J = 4, both precisions, batch counted
    assert first(1 << 20, 8, F64) == (11, 128, 32)
    assert first(1 << 20, 2, F64) == (11, 512, 8)
    assert first(1 << 18, 4, F64, b=4) == (11, 256, 16)
    assert first(1 << 19, 4, F64, b=4) == (11, 256, 32)  # 2^21 values: the 8192 tile, J = 8
    assert first(1 << 20, 8, F32) == (11, 128, 32)
    # J = 8 would leave a remainder split in two passes, J = 4 one: J = 4 (fp64
    # P <= 8; fp32 only at P = 8, from a 2048-point remainder)
    for P in (2, 4, 8):
        d = pifft.dry_run(1 << 22, P, 1, F64)
        assert d["launch_mode"] == [11, 10] and d["lines"][0] == 4 * P and d["radix"][1] == 2048
    assert pifft.dry_run(1 << 21, 8, 1, F64)["radix"] == [128, 2048]   # a 2048-point remainder: J = 8
    assert pifft.dry_run(1 << 23, 8, 1, F64)["radix"] == [128, 128, 64]  # J = 4 splits too: J = 8
    assert pifft.dry_run(1 << 21, 8, 1, F32)["radix"] == [256, 1024]
    assert pifft.dry_run(1 << 22, 8, 1, F32)["radix"] == [256, 2048]
    assert pifft.dry_run(1 << 22, 4, 1, F32)["radix"] == [256, 64, 64]  # fp32 P = 4 keeps J = 8
    assert pifft.dry_run(1 << 22, 16, 1, F32)["lines"][0] == 128        # ... and P = 16 at 2^22
    assert pifft.dry_run(1 << 21, 16, 1, F32)["radix"] == [128, 1024]   # (P = 16 fp32: a 1024-point remainder)
    assert pifft.dry_run(1 << 21, 16, 1, F64)["lines"][0] == 32         # fp64 P = 16 at 32-64 MiB: J = 2
    assert pifft.dry_run(1 << 23, 16, 1, F64)["launch_kind"][0] == "tree"


def test_single_pass_all_worker_plans_go_worker_interleaved(monkeypatch):
    """A single transform whose local FFT would be one pass (M <= 2^14) runs
    the worker-interleaved plan with every worker's tree fused into its first
    pass -- two launches instead of tree + pass + interleave -- from M = 2^12
    up (2^11 at the fused plans) where that plan exists; fp64 P = 16 (no fused pass there) the
    worker-interleaved two-pass plan after its tree launch (profiles/
    r05w_small_wil.log; batched: r05bt_batched_two_pass_ab.log).  M < 2^11 keeps the single pass."""
    def kinds(n, P, prec, b=1):
        return pifft.dry_run(n, P, b, prec)["launch_kind"]
    assert kinds(1 << 17, 8, F64) == ["tree+pass", "pass"]
    assert pifft.dry_run(1 << 17, 8, 1, F64)["radix"] == [128, 128]
    assert kinds(1 << 14, 2, F64) == ["tree+pass", "pass"]
    assert kinds(1 << 16, 16, F32) == ["tree+pass", "pass"]
    assert kinds(1 << 18, 16, F64) == ["tree", "pass", "pass"]
    assert pifft.dry_run(1 << 18, 16, 1, F64)["worker_interleaved"]
    assert kinds(1 << 14, 8, F64) == ["tree+pass", "pass"]               # M = 2^11
    assert kinds(1 << 14, 16, F64) == ["tree", "pass", "interleave"]    # M = 2^10
    assert kinds(1 << 15, 16, F64) == ["tree", "pass", "interleave"]
    assert kinds(1 << 15, 4, F64, b=4) == ["tree+pass", "pass"]           # batched too (r05bt)
    assert kinds(1 << 18, 16, F64, b=2) == ["tree", "pass", "interleave"]  # (fp64 P = 16's two-pass: batch 1 only)
    monkeypatch.setenv("PIFFT_WIL_SINGLE", "0")
    assert kinds(1 << 17, 8, F64) == ["tree", "pass", "interleave"]


def test_tiny_all_worker_plans_one_launch(monkeypatch):
    """A single transform of P M <= 8192 values (from 1024, M < 4096 but fp32 P = 2: the
    reference's GPU sweep sizes) runs as ONE fused pass: J = 1, C = P lines
    of R = M points, every worker's tree then its whole local FFT, storing
    natural order; batched, one workgroup per transform (profiles/
    r05bo_batched_one_launch_ab.log: 1.2-2.8x)."""
    for prec in (F64, F32):
        for n, P in ((1 << 10, 2), (1 << 10, 16), (1 << 12, 8), (1 << 13, 4), (1 << 13, 16)):
            d = pifft.dry_run(n, P, 1, prec)
            assert d["launch_kind"] == ["tree+pass"] and d["launch_mode"] == [11], (n, P, d)
            assert d["radix"] == [n // P] and d["lines"] == [P] and d["worker_interleaved"]
    assert pifft.dry_run(1 << 13, 2, 1, F64)["launch_kind"] == ["tree", "pass", "interleave"]  # M = 4096 ...
    assert pifft.dry_run(1 << 13, 2, 64, F64)["vpt"] == [8]                                    # ... batched: 8 per thread
    assert pifft.dry_run(1 << 13, 2, 1, F32)["launch_kind"] == ["tree+pass"]                    # (spill-free at 16)
    assert pifft.dry_run(1 << 13, 32, 1, F64)["launch_kind"][-1] == "interleave"               # P = 32 fp64 8192
    assert pifft.dry_run(1 << 12, 32, 1, F64)["launch_kind"] == ["tree+pass"]                   # ... 4096: one
    assert pifft.dry_run(1 << 13, 32, 1, F32)["launch_kind"] == ["tree+pass"]
    assert pifft.dry_run(1 << 14, 32, 1, F32)["launch_kind"][-1] == "interleave"
    assert pifft.dry_run(1 << 9, 2, 1, F64)["launch_kind"] == ["tree", "pass", "interleave"]   # < 1024
    assert pifft.dry_run(1 << 12, 8, 2, F64)["launch_kind"] == ["tree+pass"]                   # batched too
    assert pifft.dry_run(4096, 4, 4096, F32)["launch_kind"] == ["tree+pass"]                    # one workgroup each
    monkeypatch.setenv("PIFFT_WIL_ONE_LAUNCH", "0")
    assert pifft.dry_run(1 << 12, 8, 1, F64)["launch_kind"] == ["tree", "pass", "interleave"]


def test_natural_store_rule(monkeypatch):
    """The planner's rule for the last pass storing natural order itself
    (pifft.hip build_plan, PIFFT_ILV) on the slice-major layout (multi-pass
    all-worker plans use the worker-interleaved layout by default, off here):
    small outputs with enough tiles; the separate interleave launch above
    64 MiB (fp64) / 16 MiB (fp32) and for tiny plans; batched single-pass
    plans up to 128 MiB."""
    monkeypatch.setenv("PIFFT_WORKER_IL", "0")

    def kinds(n, P, b, prec):
        return pifft.dry_run(n, P, b, prec)["launch_kind"]
    assert kinds(1 << 22, 8, 1, F64)[-1] == "pass"
    assert kinds(1 << 23, 8, 1, F64)[-1] == "interleave"
    assert kinds(1 << 20, 8, 1, F32)[-1] == "pass"
    assert kinds(1 << 22, 8, 1, F32)[-1] == "interleave"
    assert kinds(1 << 16, 8, 1, F64)[-1] == "interleave"  # 8 tiles
    assert kinds(4096, 4, 4096, F32)[-1] == "pass"  # single-pass, 128 MiB
    assert kinds(4096, 4, 8192, F32)[-1] == "interleave"  # 256 MiB
    assert kinds(1 << 20, 8, 1, F64)[-1] == "pass" and kinds(1 << 20, 1, 1, F64)[-1] == "pass"
    slices = pifft.dry_run(1 << 20, 8, 1, F64, first=0, count=1)
    assert "interleave" not in slices["launch_kind"]  # slice plans never interleave


def test_config3_batched_fp32_single_pass():
    d = pifft.dry_run(4096, 1, 4096, F32)
    assert d["launch_kind"] == ["pass"] and d["radix"] == [4096]
    assert d["launch_bytes"] == [2 * 4096 * 4096 * 8]


def test_config4_2e28_fp64():
    """The 1024-point pass (128-B row segments at C = 8) goes last, where its
    narrow segments cost least (planner pass_rate, measured round 3)."""
    d = pifft.dry_run(1 << 28, 1, 1, F64)
    assert d["radix"] == [512, 512, 1024] and d["lines"] == [16, 16, 8]
    assert pifft.dry_run(1 << 29, 1, 1, F64)["radix"] == [512, 1024, 1024]
    assert d["launch_bytes"] == [2 * (1 << 28) * 16] * 3
    assert d["workspace_bytes"] >= 4 * GiB


@pytest.mark.parametrize("P", [2, 4, 8, 16])
def test_config4_split_fuses_the_tree(P):
    d = pifft.dry_run(1 << 28, P, 1, F64, first=P - 1, count=1)
    assert d["launch_kind"][0] == "tree+pass" and "tree" not in d["launch_kind"]
    assert d["local_n"] == (1 << 28) // P and d["out_elems"] == (1 << 28) // P
    # the fused pass reads the whole input replica once and writes the worker's N/P
    assert d["launch_bytes"][0] == ((1 << 28) + (1 << 28) // P) * 16
    # fused first pass: the larger radix first (R = 512, C = 16 measured 1-3 %
    # faster than the widest row segments at P = 4, 8)
    assert d["radix"][0] == max(d["radix"])


def test_config5_2e32_one_worker_of_8():
    d = pifft.dry_run(1 << 32, 8, 1, F64, first=5, count=1)
    assert d["local_n"] == 1 << 29 and d["launch_kind"][0] == "tree+pass"
    assert d["launch_bytes"][0] == ((1 << 32) + (1 << 29)) * 16
    # the fused pass keeps 256-B leaf segments (R = 512) and the plan stays at 3 passes: measured
    # 19.7 ms vs 21.3 ms for 256-128-128-128 (profiles/r01_tune_c5.log)
    assert d["radix"] == [512, 1024, 1024]
    # where the larger radix already gives 256-B leaf segments it still goes first (P = 8 at 2^28)
    assert pifft.dry_run(1 << 28, 8, 1, F64, first=7, count=1)["radix"] == [512, 256, 256]


def test_fp32_large_prefers_wide_segments(monkeypatch):
    """fp32 beyond 1 GiB per side: three passes on the 16384-value tile with
    the packed 32-values-per-thread passes (C4's segment widths: 256 B, and
    128 B on the last pass, where the narrow pass costs least); below it, or
    with PIFFT_VPT32=0, the 8192-value tile with >= 256-B row segments
    everywhere."""
    d = pifft.dry_run(1 << 28, 1, 1, F32)
    assert d["radix"] == [512, 512, 1024] and d["lines"] == [32, 32, 16] and d["vpt"] == [32, 32, 32]
    assert pifft.dry_run(1 << 26, 1, 1, F32)["vpt"] == [16, 16, 16]
    monkeypatch.setenv("PIFFT_VPT32", "0")
    d = pifft.dry_run(1 << 28, 1, 1, F32)
    assert all(c * 8 >= 256 for c in d["lines"]) and set(d["vpt"]) == {16}


@pytest.mark.parametrize("n,P,kinds", [
    (2, 1, ["pass"]), (2, 2, ["tree", "interleave"]), (16, 16, ["tree", "interleave"]),
    (256, 256, ["tree", "tree", "interleave"]), (1 << 16, 32, ["tree", "tree", "pass", "interleave"]),
])
def test_edge_plans(n, P, kinds):
    assert pifft.dry_run(n, P, 1, F64)["launch_kind"] == kinds


def test_dry_run_validation():
    with pytest.raises(pifft.PifftError, match="More processors than inputs"):
        pifft.dry_run(8, 16)
    with pytest.raises(pifft.PifftError, match="worker range"):
        pifft.dry_run(64, 8, first=3, count=2)


@pytest.mark.parametrize("P", [1, 8])
def test_bitrev_output_needs_no_interleave(P, monkeypatch):
    """PIFFT_OUT_BITREV (the reference's scratch order): the
    whole transform on one GPU skips the interleave launch."""
    # (2^23 on the slice-major layout: above the size where natural plans
    # store natural order from their last pass, so the natural plan has the
    # interleave launch)
    monkeypatch.setenv("PIFFT_WORKER_IL", "0")
    nat = pifft.dry_run(1 << 23, P, 1, F64)
    d = pifft.dry_run(1 << 23, P, 1, F64, flags=pifft.OUT_BITREV)
    assert "interleave" not in d["launch_kind"]
    assert d["num_launches"] == nat["num_launches"] - (1 if P > 1 else 0)
    assert d["out_elems"] == 1 << 23


def test_bitrev_output_slices_and_bad_flags():
    d = pifft.dry_run(1 << 28, 8, 1, F64, first=3, count=1, flags=pifft.OUT_BITREV)
    assert d["launch_kind"][0] == "tree+pass" and d["out_elems"] == (1 << 28) // 8
    with pytest.raises(pifft.PifftError):
        pifft.dry_run(1 << 10, 2, 1, F64, flags=7)


@pytest.mark.parametrize("prec", [F64, F32])
def test_every_multipass_worker_plan_fuses_its_tree(prec):
    """One worker of P (one GPU of a P-GPU job) with a multi-pass local FFT
    evaluates its tree inside the first pass: a fused kernel instance exists
    for whatever radix and lines the planner picks (fp32 plans once fell back
    to a separate tree launch for want of one)."""
    for logn in range(16, 33):
        for P in (2, 4, 8, 16):
            d = pifft.dry_run(1 << logn, P, 1, prec, first=P - 1, count=1)
            if d["num_passes"] > 1:
                assert d["launch_kind"][0] == "tree+pass", (logn, P, d["radix"], d["lines"])


def test_padded_workspace_rows(monkeypatch):
    """Padded workspace rows (PassArgs::in_pad/out_pad, PIFFT_W_PAD): W rows
    16 KiB + 256 B apart for a W of 2 GiB or more (C4: the 1024 rows pass 3
    reads),
    none below (the worker of 8 at 2^28: 512 MiB); PIFFT_W_PAD=0 turns it off."""
    def ws(n, P=1, prec=F64, **kw):
        return pifft.dry_run(n, P, 1, prec, **kw)["workspace_bytes"]
    padded = ws(1 << 28)
    monkeypatch.setenv("PIFFT_W_PAD", "0")
    assert padded - ws(1 << 28) == 1024 * 1040 * 16
    # fp32 2^28 (three packed passes 512 x 512 x 1024): the last hand-off reads 1024 rows
    monkeypatch.delenv("PIFFT_W_PAD")
    padded32 = ws(1 << 28, prec=F32)
    monkeypatch.setenv("PIFFT_W_PAD", "0")
    assert padded32 - ws(1 << 28, prec=F32) == 1024 * 2080 * 8
    monkeypatch.delenv("PIFFT_W_PAD")
    small = ws(1 << 28, 8, first=0, count=1, flags=pifft.OUT_SLICES)
    monkeypatch.setenv("PIFFT_W_PAD", "0")
    assert small == ws(1 << 28, 8, first=0, count=1, flags=pifft.OUT_SLICES)


def test_separate_tree_flag():
    """PIFFT_SEPARATE_TREE (CLI -u): a one-worker plan keeps its tree as a
    separate launch instead of fusing it into the first pass."""
    n, P = 1 << 24, 8
    fused = pifft.dry_run(n, P, 1, F64, first=0, count=1)
    sep = pifft.dry_run(n, P, 1, F64, first=0, count=1, flags=pifft.OUT_SLICES | pifft.SEPARATE_TREE)
    assert fused["launch_kind"][0] == "tree+pass" and fused["tree_launches"] == 0
    assert sep["launch_kind"][0] == "tree" and sep["tree_launches"] == 1
    assert sep["num_passes"] == fused["num_passes"]
    with pytest.raises(pifft.PifftError, match="unknown flags"):
        pifft.dry_run(n, P, 1, F64, first=0, count=1, flags=8)


def test_worker_interleaved_layout(monkeypatch):
    """All P <= 16 workers of a natural-order plan with a multi-pass local FFT
    use the worker-interleaved layout: tree + passes, no interleave launch and
    no scattered natural-order store; PIFFT_WORKER_IL=0 restores the
    slice-major layout.  Single-pass local FFTs that neither fit one fused
    launch nor reach 2^11 points (from there two-pass worker-interleaved), P > 16 and worker ranges keep
    the slice-major layout."""
    d = pifft.dry_run(1 << 20, 8, 1, F64)
    assert d["worker_interleaved"] and not d["natural_store"] and d["launch_kind"] == ["tree+pass", "pass"]
    big = pifft.dry_run(1 << 28, 8, 1, F64)
    assert big["worker_interleaved"] and "interleave" not in big["launch_kind"]
    assert not pifft.dry_run(1 << 14, 16, 1, F64)["worker_interleaved"]         # single-pass local FFT
    assert not pifft.dry_run(1 << 20, 32, 1, F64)["worker_interleaved"]         # two tree launches
    assert not pifft.dry_run(1 << 20, 8, 1, F64, first=0, count=4)["worker_interleaved"]
    assert not pifft.dry_run(1 << 20, 1, 1, F64)["worker_interleaved"]
    monkeypatch.setenv("PIFFT_WORKER_IL", "0")
    d0 = pifft.dry_run(1 << 20, 8, 1, F64)
    assert not d0["worker_interleaved"] and d0["natural_store"]
    assert pifft.dry_run(1 << 28, 8, 1, F64)["launch_kind"][-1] == "interleave"


def test_position_model_off_restores_bandwidth_model(monkeypatch):
    """PIFFT_POS_MODEL=0: the round-2 segment-width model (1024-point pass
    first); plans with a fused tree or resident in the Infinity Cache never
    used the position rates."""
    fused = pifft.dry_run(1 << 28, 8, 1, F64, first=0, count=1)["radix"]
    small = pifft.dry_run(1 << 20, 1, 1, F64)["radix"]
    monkeypatch.setenv("PIFFT_POS_MODEL", "0")
    assert pifft.dry_run(1 << 28, 1, 1, F64)["radix"] == [1024, 512, 512]
    assert pifft.dry_run(1 << 28, 1, 1, F32)["radix"] == [1024, 512, 512]
    assert pifft.dry_run(1 << 28, 8, 1, F64, first=0, count=1)["radix"] == fused
    assert pifft.dry_run(1 << 20, 1, 1, F64)["radix"] == small


def test_position_model_not_for_worker_interleaved_plans(monkeypatch):
    """All-worker plans in the worker-interleaved layout keep the segment-width
    model's order (the narrow pass last measured 1-14 % slower there,
    profiles/r03_pos_model_shapes.log); one-worker plans of the same local
    size put it last.  (The tree as its own launch: with it fused, MODE 11,
    the first radix is the fused tile's and the rest is planned after it.)"""
    assert pifft.dry_run(1 << 29, 2, 1, F64)["radix"] == [512, 1024, 512]
    monkeypatch.setenv("PIFFT_WIL_FUSE", "0")
    wil = pifft.dry_run(1 << 29, 2, 1, F64)
    assert wil["worker_interleaved"] and wil["radix"] == [1024, 512, 512]
    assert pifft.dry_run(1 << 28, 1, 1, F64)["radix"] == [512, 512, 1024]
    assert pifft.dry_run(1 << 27, 2, 1, F32)["radix"] == [512, 512, 256]


STRAY = {"PIFFT_ORDER": "1", "PIFFT_PASSES": "4", "PIFFT_RADIX_LOGS": "10,10,8", "PIFFT_NT": "0",
         "PIFFT_WORKER_IL": "0", "PIFFT_POS_MODEL": "0", "PIFFT_VPT32": "0", "PIFFT_W_PAD": "0",
         "PIFFT_TILE64": "4096", "PIFFT_LAST_C": "16", "PIFFT_FUSE_TREE": "0", "PIFFT_ILV": "1",
         "PIFFT_SINGLE_TILE32": "8192", "PIFFT_LAST_VPT": "16", "PIFFT_FUSED_VPT": "16", "PIFFT_WIL_VPT": "16",
         "PIFFT_WIL_FUSE": "0", "PIFFT_WIL_FUSE_J": "16", "PIFFT_WIL_TREE_DIRECT": "1", "PIFFT_WIL_TREE_MIN_LOG": "0",
         "PIFFT_PERMLANE": "0", "PIFFT_FAULT": "broadcast",
         "PIFFT_WIL_FUSE_TILE": "2048", "PIFFT_WIL_SINGLE": "0", "PIFFT_WIL_ONE_LAUNCH": "0"}


@pytest.mark.parametrize("shape", [(1 << 28, 1, 1, F64, 0, 1, 0), (1 << 28, 1, 1, F32, 0, 1, 0),
                                   (1 << 20, 8, 1, F64, 0, 8, 0), (1 << 20, 8, 1, F64, 0, 1, 1),
                                   (4096, 1, 4096, F32, 0, 1, 0), (1 << 32, 8, 1, F64, 7, 1, 1)])
def test_stray_tuning_variables_are_ignored(shape, monkeypatch):
    """Without PIFFT_TUNING=1 the planner reads none of its tuning variables:
    a stray PIFFT_ORDER / PIFFT_PASSES / ... inherited from a shell leaves the
    product's plan unchanged (round-3 verdict, knob debt)."""
    n, P, b, prec, first, count, flags = shape
    monkeypatch.delenv("PIFFT_TUNING")
    want = pifft.dry_run(n, P, b, prec, first=first, count=count, flags=flags)
    for k, v in STRAY.items():
        monkeypatch.setenv(k, v)
    assert pifft.dry_run(n, P, b, prec, first=first, count=count, flags=flags) == want
    monkeypatch.setenv("PIFFT_TUNING", "0")
    assert pifft.dry_run(n, P, b, prec, first=first, count=count, flags=flags) == want
    # ... and the same variables do take effect under PIFFT_TUNING=1
    monkeypatch.setenv("PIFFT_TUNING", "1")
    assert pifft.dry_run(n, P, b, prec, first=first, count=count, flags=flags) != want


def test_small_slices_run_the_fused_pass_at_8_values_per_thread(monkeypatch):
    """Round 4 (profiles/r04d_fused_vpt8.log): a one-worker slice's fused tree
    pass runs at 8 values per thread when it has R <= 512 points and at most
    128 workgroups (config 2's slice: 14.05 -> 12.66 us); R = 1024 and larger
    launches keep 16; config-2-sized worker-interleaved passes run at 8.  And
    (profiles/r04k_*.log) the last strided pass of a small fp64 plan -- R <=
    512, <= 256 workgroups -- runs at 8 too (the slice 12.7 -> 12.2 us)."""
    d = pifft.dry_run(1 << 20, 8, 1, F64, first=0, count=1)   # config 2's slice: 512 x 256, 64 workgroups
    assert d["launch_kind"][0] == "tree+pass" and d["radix"] == [512, 256] and d["vpt"] == [8, 8]
    assert d["launch_mode"] == [3, 2]
    assert pifft.dry_run(1 << 21, 8, 1, F64, first=7, count=1)["vpt"] == [8, 8]   # 128 workgroups each
    assert pifft.dry_run(1 << 20, 2, 1, F64, first=0, count=1)["vpt"] == [16, 8]  # R = 1024 first
    assert pifft.dry_run(1 << 23, 8, 1, F64, first=0, count=1)["vpt"] == [16, 16]  # 256 workgroups, R = 1024
    assert pifft.dry_run(1 << 28, 8, 1, F64, first=0, count=1)["vpt"] == [16, 16, 16]
    assert pifft.dry_run(1 << 17, 1, 1, F64)["vpt"] == [16, 8]                    # P = 1: the last pass only
    assert pifft.dry_run(1 << 20, 1, 1, F64)["vpt"] == [16, 16]                   # config 1 (R = 1024)
    assert pifft.dry_run(1 << 17, 1, 1, F32)["vpt"] == [16, 16]                   # fp64 only
    # config 2: the fused all-worker pass (MODE 11) and a 1024-point pass at 16; with the tree as
    # its own launch the worker-interleaved passes run at 8
    assert pifft.dry_run(1 << 20, 8, 1, F64)["vpt"] == [16, 16]
    monkeypatch.setenv("PIFFT_WIL_FUSE", "0")
    assert pifft.dry_run(1 << 20, 8, 1, F64)["vpt"] == [8, 8]                     # config 2 (worker-interleaved)
    assert pifft.dry_run(1 << 28, 8, 1, F64)["vpt"] == [16, 16, 16]
