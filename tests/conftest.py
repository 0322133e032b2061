"""Shared pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs the oracle-vs-golden, host-logic and ABI-load tests on CPU;
`-m gpu` runs the HIP parity tests (through the C-ABI) on an MI355X.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "cs87project-msolano2_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through libpifft.so)")


@pytest.fixture(autouse=True)
def _planner_tuning(monkeypatch):
    """Tests force alternative plans through the planner's PIFFT_* tuning
    variables, which libpifft reads only under PIFFT_TUNING=1 (include/pifft.h).
    Every test starts with tuning enabled and no inherited PIFFT_* variable, so
    a stray one in the caller's shell cannot change a test's plan."""
    for k in list(os.environ):
        if k.startswith("PIFFT_") and k != "PIFFT_LIB":
            monkeypatch.delenv(k)
    monkeypatch.setenv("PIFFT_TUNING", "1")


# PIFFTTEST_RECORD_INSTANCES=<file>: every plan a test builds (with the tuning
# variables it set) also records the k_pass instances it launches
# (pifft_plan_dry_run_instances of the same shape under the same environment),
# and at the end of the session every instance the planner found while
# choosing plans (pifft_instance_found: its probes, launched or not) joins
# them in <file> -- tests/golden/instances_tests.txt, which
# tests/test_instances.py reads beside the default planner's sweep.
_RECORD = os.environ.get("PIFFTTEST_RECORD_INSTANCES", "")
_recorded: set = set()
_table: list = []


def pytest_sessionstart(session):
    if not _RECORD:
        return
    import pifft
    orig = pifft.Plan.__init__

    def init(self, *a, **kw):
        orig(self, *a, **kw)
        i = self.info
        if not _table:
            _table.extend(pifft.instances())
        table = _table
        for k in pifft.dry_run_instances(i.n, i.workers, i.batch, i.prec, first=i.first_worker,
                                         count=i.num_workers, flags=i.flags):
            if k >= 0:
                _recorded.add(table[k])
    pifft.Plan.__init__ = init


def pytest_sessionfinish(session, exitstatus):
    if not _RECORD:
        return
    import pifft
    table = _table or pifft.instances()
    _recorded.update(table[i] for i in pifft.instances_found())
    with open(_RECORD, "w") as f:
        for d in sorted(_recorded):
            f.write("prec=%d R=%d C=%d mode=%d nts=%d lp=%d vpt=%d\n" % d)
