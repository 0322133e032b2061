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
