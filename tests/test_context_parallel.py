"""Context-parallel (offset-split) search: partial searches over disjoint offset ranges, combined with one
MAX reduction of packed 64-bit keys (the Reduce the reference never had, BASELINE.json)."""
import numpy as np
import pytest

from mpi_openmp_cuda_amd import Problem, Semantics, decode_keys, make_synthetic, search_cpu, search_keys_cpu
from mpi_openmp_cuda_amd.ops.align import as_triples, keys_to_ordered_int64, ordered_int64_to_keys


@pytest.mark.parametrize("shape,n", [("input3", 6), ("input4", 40), ("input1", 50), ("input6", 300)])
@pytest.mark.parametrize("parts", [1, 2, 3, 7])
@pytest.mark.parametrize("sem", [Semantics.REFERENCE, Semantics.SPEC])
def test_parts_combine_to_full_search(shape, n, parts, sem):
    prob = make_synthetic(shape, n, seed=parts + n)
    keys = np.zeros(prob.n, np.uint64)
    for part in range(parts):
        keys = np.maximum(keys, search_keys_cpu(prob, part, parts, sem))
    assert np.array_equal(as_triples(decode_keys(keys, prob)), as_triples(search_cpu(prob, sem)))


def test_edge_records():
    # equal length (single candidate), L2 > L1 (no candidate), more parts than offsets
    prob = Problem.from_strings([3, 1, 2, 1], "ABCDEFG", ["ABCDEFG", "ABCDEFGH", "ACE", "G"])
    for parts in (1, 4, 16):
        keys = np.zeros(prob.n, np.uint64)
        for part in range(parts):
            keys = np.maximum(keys, search_keys_cpu(prob, part, parts))
        got = as_triples(decode_keys(keys, prob))
        assert np.array_equal(got, as_triples(search_cpu(prob)))
        assert tuple(got[1]) == (-2**31, 0, 0)


def test_key_order_survives_signed_transport():
    rng = np.random.default_rng(0)
    k = rng.integers(0, 2**63, 1000, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, 1000).astype(np.uint64)
    s = keys_to_ordered_int64(k)
    assert np.array_equal(np.argsort(k, kind="stable"), np.argsort(s, kind="stable"))
    assert np.array_equal(ordered_int64_to_keys(s), k)
