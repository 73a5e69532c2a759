"""Native C++ unit tests of the host core (csrc/tests/test_core.cpp; SURVEY.md §4.3 'unit (C++)')."""
import subprocess

from conftest import ROOT


def test_core_unit_binary():
    r = subprocess.run(["make", "-C", ROOT, "-s", "unit"], capture_output=True, timeout=600)
    out = r.stdout.decode()
    assert r.returncode == 0, out + r.stderr.decode()
    assert " 0 failed" in out and "FAILED" not in out
