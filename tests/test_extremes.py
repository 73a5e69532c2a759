"""Narrow-integer fast paths at their exactness bounds, CPU tier (csrc/include/moc/kernel_bounds.hpp).

The product's rules pick each kernel form; these tests pin where the rules put the bounds for fixed shapes
(so a changed rule is visible), and check the CPU engine against brute force on the adversarial inputs the
GPU tier runs at and one past each bound (tests/test_gpu.py test_extreme_values_*). The host replays of
the forms' own arithmetic at the bounds are csrc/tests/test_core.cpp *_replay_bounds (test_native_unit.py).
Reference arithmetic: plain int (/root/reference/cudaFunctions.cu:103,161)."""
import numpy as np
import pytest

from mpi_openmp_cuda_amd import Semantics, brute_force_native, search_cpu
from mpi_openmp_cuda_amd.ops.align import as_triples, kernel_bounds
from mpi_openmp_cuda_amd.utils.synthetic import make_extreme

# (name, L1, l2_min, l2_max, weights at the bound, weights one past it, bound field, value at, value past)
BOUNDS = [
    ("swipe_kbits_w4", 40, 6, 16, (31, 0, 0, 31), (32, 0, 0, 32), "swipe", "swipe_kbits", "swipe_rk"),
    ("swipe_kbits_w8", 60, 20, 32, (7, 0, 0, 7), (8, 0, 0, 8), "swipe", "swipe_kbits", "swipe_rk"),
    ("swipe_rk_w4", 40, 6, 16, (1023, 0, 0, 1023), (1024, 0, 0, 1024), "swipe", "swipe_rk", None),
    ("swipe_rk_w8", 60, 20, 32, (511, 0, 0, 511), (512, 0, 0, 512), "swipe", "swipe_rk", None),
    ("swipe_rk_w16", 70, 40, 64, (255, 0, 0, 255), (256, 0, 0, 256), "swipe", "swipe_rk", None),
    ("swipe_rk_w24", 130, 67, 96, (170, 0, 0, 170), (171, 0, 0, 171), "swipe", "swipe_rk", None),
    ("swipe_rk_w32", 190, 127, 128, (127, 0, 0, 127), (128, 0, 0, 128), "swipe", "swipe_rk", None),
    ("short_pk", 150, 130, 150, (109, 0, 0, 109), (110, 0, 0, 110), "short_pk", True, False),
    ("short_key32", 200, 150, 190, (22075, 0, 0, 22075), (22076, 0, 0, 22076), "key_shift", 8, 0),
    ("tile16", 600, 150, 400, (63, 0, 0, 64), (64, 0, 0, 64), "profile16", True, False),
    ("tile16_i16", 600, 150, 400, (255, 0, 0, 256), (256, 0, 0, 256), "profile16_i16", True, False),
    ("tiles_key32", 600, 150, 400, (5242, 0, 0, 5242), (5243, 0, 0, 5243), "key_shift", 9, 0),
    # tile16's 32-bit selection keys: L1 2600 needs 13 index bits, so max|T| * L2 < 2^18 (127 * 2064 = 262128)
    ("tile16_key32", 2600, 2000, 2064, (127, 0, 0, 0), (127, 0, 0, 0), "tile16_key_bits", 13, 13),
    ("tile16_key32_l2", 2600, 2000, 2065, (127, 0, 0, 0), (127, 0, 0, 0), "tile16_key_bits", 0, 0),
]


@pytest.mark.parametrize("case", BOUNDS, ids=[c[0] for c in BOUNDS])
def test_bound_positions(case):
    _, L1, lo, hi, w_at, w_past, field, at, past = case
    assert kernel_bounds(w_at, L1, lo, hi)[field] == at
    assert kernel_bounds(w_past, L1, lo, hi)[field] == past


def test_extreme_fixture_reaches_the_bound():
    # an even-offset piece of "AZAZ..." under W1 = W4 = w: every step adds Dt = 2w, so the diagonal difference
    # D_o(L2) is exactly the 2 w L2 the rules bound
    prob = make_extreme(40, 6, 16, (31, 0, 0, 31))
    s1 = prob.seq1
    lut = np.where(np.arange(27)[:, None] == np.arange(27)[None, :], 31, -31)
    for i in range(prob.n):
        r = prob.codes[prob.offsets[i]:prob.offsets[i + 1]]
        if len(r) == 16 and np.array_equal(r, s1[:16]):
            d = sum(int(lut[c, s1[j]]) - int(lut[c, s1[j + 1]]) for j, c in enumerate(r))
            assert d == 2 * 31 * 16
            break
    else:
        pytest.fail("no even-offset piece of Seq1 in the fixture")


@pytest.mark.parametrize("case", [c for c in BOUNDS if c[1] <= 200], ids=[c[0] for c in BOUNDS if c[1] <= 200])
@pytest.mark.parametrize("sem", [Semantics.REFERENCE, Semantics.SPEC])
def test_cpu_engine_at_bounds(case, sem):
    # the oracle the GPU tier compares with: the CPU engine equals brute force on every adversarial input
    _, L1, lo, hi, w_at, w_past, *_ = case
    for w in (w_at, w_past):
        prob = make_extreme(L1, lo, hi, w, seed=L1)
        assert np.array_equal(as_triples(search_cpu(prob, sem)), as_triples(brute_force_native(prob, sem))), w


def test_cpu_engine_long_extremes():
    # the tile16 shape: records of 150..400 letters under Seq1 = "AZ" * 300, W1 + W4 = 127
    prob = make_extreme(600, 150, 400, (63, 0, 0, 64), seed=3)
    assert np.array_equal(as_triples(search_cpu(prob)), as_triples(brute_force_native(prob)))


def test_tile16_key32_fixture_reaches_the_bound():
    # the GPU tier's tile16_key32_at input: an even-offset piece of Seq1 of 2064 letters scores 127 * 2064,
    # 16 below the 2^18 the 32-bit keys hold at L1 = 2600 (and 2065 letters pass it)
    prob = make_extreme(2600, 2000, 2064, (127, 0, 0, 0), copies=1, seed=2600)
    best = max(int(t[0]) for t in as_triples(search_cpu(prob)))
    assert best == 127 * 2064 and best < 2 ** 18 <= 127 * 2065
