"""Synthetic problems shaped like the reference fixtures (no datasets are available offline).

The benchmark metric (BASELINE.json) is quoted "on input6.txt array ... on synthetic/random-init arrays
of the input6.txt shape": input6 has W = 4 3 2 10, |Seq1| = 26 and Seq2 lengths 6..11
(/root/reference/input6.txt). ``make_synthetic("input6", n)`` draws n records of that shape.
Other shapes mirror input3 (long Seq2, L2 > 1024 present), input4 (longest Seq1, tiny Seq2) and the
PDF limits (|Seq1| = 3000, |Seq2| <= 2000).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..models.problem import Problem
from ..models.scoring import Weights


@dataclass(frozen=True)
class Shape:
    weights: tuple
    L1: int
    l2_min: int
    l2_max: int


SHAPES = {
    "input6": Shape((4, 3, 2, 10), 26, 6, 11),
    "input1": Shape((100, 2, 3, 4), 51, 32, 41),
    "input3": Shape((2, 2, 1, 10), 1489, 56, 1152),
    "input4": Shape((10, 2, 3, 4), 2976, 5, 82),
    "limits": Shape((10, 2, 3, 4), 3000, 1, 2000),
}


def make_synthetic(shape: str = "input6", n_records: int = 1000, seed: int = 0) -> Problem:
    s = SHAPES[shape]
    rng = np.random.default_rng(seed)
    seq1 = rng.integers(1, 27, size=s.L1, dtype=np.uint8)
    lengths = rng.integers(s.l2_min, s.l2_max + 1, size=n_records, dtype=np.int64)
    offsets = np.zeros(n_records + 1, dtype=np.int64)
    np.cumsum(lengths, out=offsets[1:])
    codes = rng.integers(1, 27, size=int(offsets[-1]), dtype=np.uint8)
    return Problem(Weights.of(s.weights), seq1, codes, offsets)


def fill_codes(out: np.ndarray, seed: int, chunk: int = 1 << 26):
    """Fills a (possibly huge / shared) uint8 array with random letter codes, chunk by chunk."""
    rng = np.random.default_rng(seed)
    for b in range(0, out.shape[0], chunk):
        e = min(out.shape[0], b + chunk)
        out[b:e] = rng.integers(1, 27, size=e - b, dtype=np.uint8)
