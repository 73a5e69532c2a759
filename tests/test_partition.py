"""Partitioner: contiguous, covering, any p (incl. p > N and N == 0), cost-balanced (bugs B5/B6)."""
import numpy as np
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from mpi_openmp_cuda_amd.parallel.partition import CPU_COST, partition, partition_even, record_costs


@settings(max_examples=200, deadline=None)
@given(st.lists(st.integers(1, 3000), min_size=0, max_size=60), st.integers(1, 3000), st.integers(1, 17))
def test_partition_is_contiguous_cover(lengths, L1, p):
    b = partition(np.array(lengths, np.int64), L1, p)
    assert b[0] == 0 and b[-1] == len(lengths) and len(b) == p + 1
    assert (np.diff(b) >= 0).all()


def test_partition_balance():
    rng = np.random.default_rng(0)
    lengths = rng.integers(5, 1200, 4000)
    L1 = 1500
    for p in (2, 4, 8):
        b = partition(lengths, L1, p)
        c = record_costs(lengths, L1, CPU_COST)
        per = np.array([c[b[r]:b[r + 1]].sum() for r in range(p)])
        assert per.max() <= per.mean() * 1.01 + c.max()


def test_p_greater_than_n():
    b = partition(np.array([3, 4], np.int64), 10, 8)
    assert b[-1] == 2 and len(b) == 9


@pytest.mark.parametrize("n,p", [(0, 3), (5, 8), (11, 4), (32, 8)])
def test_even(n, p):
    b = partition_even(n, p)
    assert b[0] == 0 and b[-1] == n and (np.diff(b) >= 0).all() and np.diff(b).max() - np.diff(b).min() <= 1
