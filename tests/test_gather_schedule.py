"""pifft_allgather's multi-device branch logic on the CPU (no GPU): the copy
schedule of csrc/pifft_gather.h -- which device pairs need peer access, one
copy stream per source plan, where every slice of every transform lands --
for mocked device lists: the 8-GPU split of the driver's scaling run, several
plans per device, one GPU, batches.  The gathered buffer is then exactly the
transform-major slice layout the interleave reads (CPU.c:496-499's `out`
ownership): every element written once."""
import json
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "gather_schedule_main.cpp")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("gs") / "gather_schedule")
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-o", out, SRC], check=True)
    return out


def schedule(exe, n, P, batch, dst_mask, plans):
    args = [exe, str(n), str(P), str(batch), hex(dst_mask)] + [f"{d}:{q0}:{nq}" for d, q0, nq in plans]
    return json.loads(subprocess.run(args, check=True, capture_output=True, text=True).stdout)


def covered_once(g, n, batch, dst):
    hits = [0] * (n * batch)
    for c in g["copies"]:
        if c["dst"] == dst:
            for e in range(c["dst_off"], c["dst_off"] + c["elems"]):
                hits[e] += 1
    return all(h == 1 for h in hits)


def test_eight_gpu_split_gather_on_every_gpu(exe):
    """The driver's --gpus 8 line: one worker per GPU, every GPU a destination."""
    n, P = 1 << 12, 8
    plans = [(d, d, 1) for d in range(8)]
    g = schedule(exe, n, P, 1, 0xFF, plans)
    assert g["streams"] == 8
    # every ordered pair of distinct devices needs peer access, once
    assert sorted(map(tuple, g["peer"])) == sorted((a, b) for a in range(8) for b in range(8) if a != b)
    assert len(g["copies"]) == 64
    for c in g["copies"]:
        assert c["stream"] == c["src"] and c["peer"] == (c["src"] != c["dst"])
        assert c["elems"] == n // P and c["dst_off"] == c["src"] * (n // P) and c["src_off"] == 0
    for d in range(8):
        assert covered_once(g, n, 1, d)


def test_gather_onto_first_gpu_only(exe):
    """pifft_execute_group's host path: gather onto plan 0's device only."""
    n, P = 1 << 10, 4
    g = schedule(exe, n, P, 1, 0x1, [(d, d, 1) for d in range(4)])
    assert sorted(map(tuple, g["peer"])) == [(0, 1), (0, 2), (0, 3)]
    assert {c["dst"] for c in g["copies"]} == {0} and len(g["copies"]) == 4
    assert [c["peer"] for c in g["copies"]] == [False, True, True, True]
    assert covered_once(g, n, 1, 0)


def test_several_plans_per_device_and_batches(exe):
    """Two plans per device (worker ranges of 2), 3 transforms: per-transform
    copies land transform-major; plans sharing the destination's device copy
    locally; peer pairs are per device, not per plan."""
    n, P, batch = 1 << 10, 8, 3
    plans = [(0, 0, 2), (0, 2, 2), (1, 4, 2), (1, 6, 2)]
    g = schedule(exe, n, P, batch, 0b0101, plans)
    assert sorted(map(tuple, g["peer"])) == [(0, 1), (1, 0)]
    assert len(g["copies"]) == 2 * 4 * batch
    M = n // P
    for c in g["copies"]:
        q0 = plans[c["src"]][1]
        bt = c["src_off"] // (2 * M)
        assert c["elems"] == 2 * M and c["dst_off"] == bt * n + q0 * M
        assert c["peer"] == (plans[c["src"]][0] != plans[c["dst"]][0])
    assert covered_once(g, n, batch, 0) and covered_once(g, n, batch, 2)


def test_single_device_needs_no_peer(exe):
    """All plans on one GPU (the tests' and the 1-GPU rehearsals' case)."""
    g = schedule(exe, 1 << 8, 4, 2, 0b1111, [(0, q, 1) for q in range(4)])
    assert g["peer"] == [] and not any(c["peer"] for c in g["copies"])
    for d in range(4):
        assert covered_once(g, 1 << 8, 2, d)
