"""Native C++ unit tests of the host core (csrc/tests/test_core.cpp; SURVEY.md §4.3 'unit (C++)')."""
import os
import subprocess

import pytest
from conftest import ROOT


@pytest.mark.parametrize("simd", ["1", "0"])
def test_core_unit_binary(simd):
    # MOC_FILL_SIMD=0: the portable SSE2 tokeniser/encoder; default: the AVX-512 VBMI2 one where the host has
    # it (this container's CPU does) — the parser tests run against both
    env = dict(os.environ, MOC_FILL_SIMD=simd)
    r = subprocess.run(["make", "-C", ROOT, "-s", "unit"], capture_output=True, timeout=600, env=env)
    out = r.stdout.decode()
    assert r.returncode == 0, out + r.stderr.decode()
    assert " 0 failed" in out and "FAILED" not in out
