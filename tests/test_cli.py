"""The C host keeps the reference's command line (CPU.c:125-211): same flags,
same validation messages, same exit status, checked side by side with the
reference binary compiled from its source (oracle/_ref) when present."""
import os
import subprocess

import pytest

import pifft
import pifft_oracle as oracle

CASES = [
    (["-n", "3", "-p", "1"], "Invalid input size (should be 2^i for i>0)"),
    (["-n", "16", "-p", "3"], "Invalid number of procs (should be 2^i for i>0)"),
    (["-p", "2"], "Missing option: -n"),
    (["-n", "16"], "Missing option: -p"),
    (["-n", "16", "-p", "32"], "More processors than inputs!"),
    (["-n", "16", "-p", "2", "-q"], "Unknown or missing arg q"),
]


def _run(exe, args):
    return subprocess.run([exe] + args, capture_output=True, text=True, timeout=60)


@pytest.mark.parametrize("args,msg", CASES)
def test_cli_validation(args, msg):
    assert os.path.exists(pifft.CLI_PATH)
    r = _run(pifft.CLI_PATH, args)
    assert r.returncode == 1
    assert msg in r.stderr
    assert "Could not setup the transform from the cmdline args" in r.stderr
    ref = oracle.reference_binary(32)
    if ref:
        rr = _run(ref, args)
        assert rr.returncode == r.returncode
        assert msg in rr.stderr


def test_cli_usage_lists_reference_flags():
    r = _run(pifft.CLI_PATH, ["-n", "3", "-p", "1"])
    for flag in ("-n <n>", "-p <p>", "-o", "-t"):
        assert flag in r.stdout
