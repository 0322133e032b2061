"""The compiled k_pass instances are exactly the ones plans use (round-5
verdict: 1474 instances, 6.3 MB, several of them reachable by no plan).

  * every instance the default planner launches over its whole domain
    (tools/instance_sweep.py: N = 2^1..2^32, P = 2^0..2^12, every worker range
    [0, count), all output orders, with and without a separate tree, batches
    1..4096, fp32 and fp64) is compiled, and that set is the committed
    tests/golden/instances_default.txt -- a planner change that reaches a new
    instance, or stops using one, shows here;
  * every compiled instance is in that list or in
    tests/golden/instances_tests.txt / instances_tests_cpu.txt, the instances
    the GPU tests' plans (recorded on MI355X) and the CPU tests' dry runs
    depend on under their tuning variables (PIFFTTEST_RECORD_INSTANCES,
    conftest.py) -- nothing is compiled that no plan depends on, and nothing
    a plan depends on is left out.
Host-side planning only (pifft_plan_dry_run_instances): no GPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import pifft  # noqa: E402
import instance_sweep  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def _read(name):
    with open(os.path.join(GOLD, name)) as f:
        return {ln.strip() for ln in f if ln.strip()}


@pytest.fixture(scope="module")
def registry():
    return {instance_sweep.fmt(d) for d in pifft.instances()}


@pytest.fixture(scope="module")
def default_used():
    table, used, _ = instance_sweep.sweep(jobs=4)
    return {instance_sweep.fmt(table[i]) for i in used}


def test_instance_registry_descriptors():
    table = pifft.instances()
    assert len(table) == pifft.lib().pifft_instance_count() > 0
    assert len(set(table)) == len(table)  # no instance twice
    for prec, R, C, mode, nts, lp, vpt in table:
        assert prec in (32, 64) and R & (R - 1) == 0 and C & (C - 1) == 0 and nts in (0, 1) and vpt in (8, 16, 32)
    assert pifft.lib().pifft_instance_desc(len(table), (pifft.ctypes.c_int32 * 7)()) == -1
    assert "out of range" in pifft.last_error()


def test_dry_run_instances_matches_dry_run():
    """The instance of each launch agrees with pifft_plan_dry_run's
    description of the same plan (radix, lines, values per thread, MODE)."""
    table = pifft.instances()
    for n, P, count, batch, prec in ((1 << 28, 1, 1, 1, pifft.F64), (1 << 20, 8, 8, 1, pifft.F64),
                                     (1 << 20, 8, 1, 1, pifft.F64), (1 << 12, 1, 1, 4096, pifft.F32),
                                     (1 << 28, 1, 1, 1, pifft.F32)):
        ids = pifft.dry_run_instances(n, P, batch, prec, count=count)
        d = pifft.dry_run(n, P, batch, prec, count=count)
        assert len(ids) == d["num_launches"]
        passes = [table[i] for i in ids if i >= 0]
        assert [t[1] for t in passes] == d["radix"][: len(passes)]
        assert [t[2] for t in passes] == d["lines"][: len(passes)]
        assert all(t[0] == prec for t in passes)


def test_default_planner_uses_the_committed_list(default_used, registry):
    want = _read("instances_default.txt")
    assert default_used <= registry, sorted(default_used - registry)[:5]
    assert default_used == want, (sorted(default_used - want)[:5], sorted(want - default_used)[:5])


def test_every_compiled_instance_is_used(registry):
    used = _read("instances_default.txt") | _read("instances_tests.txt") | _read("instances_tests_cpu.txt")
    unused = registry - used
    assert not unused, f"{len(unused)} compiled instances no plan launches, e.g. {sorted(unused)[:5]}"
    dropped = used - registry
    assert not dropped, f"{len(dropped)} instances a plan launches are not compiled, e.g. {sorted(dropped)[:5]}"
