"""Property tests: native O(L1*L2) engine == native brute force == Python brute force == Python prefix
oracle, on random problems, in both semantics (SURVEY.md §4.3 'property')."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from mpi_openmp_cuda_amd import Problem, Semantics, brute_force_native, search_cpu
from mpi_openmp_cuda_amd.models.reference import brute_force, prefix_oracle, solve_problem
from mpi_openmp_cuda_amd.models.scoring import score_table
from mpi_openmp_cuda_amd.ops.align import as_triples

letters = st.text(alphabet="ACDEFGHIKLMNPQRSTVWYBJOUXZ", min_size=1, max_size=24)


@st.composite
def problems(draw):
    w = draw(st.lists(st.integers(0, 20), min_size=4, max_size=4))
    s1 = draw(letters)
    recs = draw(st.lists(st.text(alphabet="ACDEFGHIKLMNPQRSTVWY", min_size=1, max_size=len(s1) + 2),
                         min_size=0, max_size=6))
    return Problem.from_strings(w, s1, recs)


@settings(max_examples=150, deadline=None)
@given(problems(), st.sampled_from([Semantics.REFERENCE, Semantics.SPEC]))
def test_native_matches_brute_force(prob, sem):
    fast = as_triples(search_cpu(prob, sem))
    brute = as_triples(brute_force_native(prob, sem))
    py = solve_problem(prob, sem, oracle=brute_force)
    assert np.array_equal(fast, brute)
    assert np.array_equal(fast, py)


@settings(max_examples=100, deadline=None)
@given(problems(), st.sampled_from([Semantics.REFERENCE, Semantics.SPEC]))
def test_prefix_oracle_matches_brute_force(prob, sem):
    t = score_table(prob.weights)
    for i in range(prob.n):
        s2 = prob.codes[prob.offsets[i]:prob.offsets[i + 1]]
        assert prefix_oracle(t, prob.seq1, s2, sem) == brute_force(t, prob.seq1, s2, sem)


def test_threads_do_not_change_results():
    rng = np.random.default_rng(1)
    from mpi_openmp_cuda_amd import make_synthetic

    prob = make_synthetic("input4", 40, seed=3)
    base = as_triples(search_cpu(prob, threads=1))
    for t in (2, 3, 8):
        assert np.array_equal(as_triples(search_cpu(prob, threads=t)), base)
    # few records -> offset-split path (the CP analogue) must agree too
    few = prob.slice(0, 2)
    assert np.array_equal(as_triples(search_cpu(few, threads=8)), base[:2])
    del rng


# Spec worked examples (PDF p.2-5) through both semantics.
@pytest.mark.parametrize("s1,s2,ref,spec", [
    ("HELLOWORLD", "OWRL", (40, 4, 2), (40, 4, 2)),
    ("APQRSBATAV", "ASQRSEAVSL", (36, 0, 0), (36, 0, 0)),
    ("APQRSBAAVV", "RSTBTL", (9, 3, 2), (9, 3, 2)),
    ("ABCDEFGH", "FGH", (16, 4, 1), (30, 5, 0)),   # bug B8: the final un-mutated offset
])
def test_spec_examples(s1, s2, ref, spec):
    prob = Problem.from_strings([10, 2, 3, 4], s1, [s2])
    assert tuple(as_triples(search_cpu(prob, Semantics.REFERENCE))[0]) == ref
    assert tuple(as_triples(search_cpu(prob, Semantics.SPEC))[0]) == spec


def test_edge_lengths():
    # L2 == L1 -> (score, 0, 0); L2 > L1 -> INT_MIN; L2 == 1, 2, 3
    prob = Problem.from_strings([3, 1, 1, 2], "ABCD", ["ABCD", "ABCDE", "C", "BC", "XYZ"])
    got = as_triples(search_cpu(prob))
    assert tuple(got[0]) == (12, 0, 0)
    assert tuple(got[1]) == (-2**31, 0, 0)
    assert np.array_equal(got, as_triples(brute_force_native(prob)))


def test_no_records():
    prob = Problem.from_strings([1, 1, 1, 1], "ABC", [])
    assert search_cpu(prob).shape == (0,)
