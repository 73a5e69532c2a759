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
    # between the reference shapes: records too long for the swipe kernel (> 64 letters) whose offset range
    # still fits a wave (<= 64 lanes): the lane-per-offset short kernel's regime
    "mid": Shape((10, 2, 3, 4), 130, 67, 85),
    # input6's lengths under a heavy weight (W1 = 300): no room for k in the int16 keys, the RK swipe form
    "heavy6": Shape((300, 3, 2, 10), 26, 6, 11),
    # long records under weights past the int8 difference profile (W1 + max(W2, W3, W4) > 127)
    "heavy3": Shape((200, 10, 10, 10), 1489, 56, 1152),
    "heavy4": Shape((120, 20, 1, 1), 2976, 5, 82),
    "heavylim": Shape((200, 10, 10, 10), 3000, 1, 2000),  # limits' lengths, int16 profile (sliding windows)
    "mid3k": Shape((10, 2, 3, 4), 2000, 400, 900),  # L1 past the widened image, records past a widened window
}


def make_synthetic(shape: str = "input6", n_records: int = 1000, seed: int = 0) -> Problem:
    return make_shape(SHAPES[shape], n_records, seed)


def make_shape(s: Shape, n_records: int = 1000, seed: int = 0) -> Problem:
    """Random Seq1 of s.L1 letters and n_records records of s.l2_min..s.l2_max random letters."""
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


A, Z = 1, 26  # letter codes of 'A' and 'Z': in no group together, so a pair is '$' or ' '


def make_extreme(L1: int, l2_min: int, l2_max: int, weights, copies: int = 1, seed: int = 0) -> Problem:
    """Adversarial records for the kernels' integer bounds (csrc/include/moc/kernel_bounds.hpp): Seq1 =
    "AZAZ...", and records that are pieces of Seq1 at even offsets (with W1 = W4 every step adds the largest
    difference Dt = W1 + W4, so |D| reaches 2 W L2) and at odd ones (-(W1 + W4)), constant 'A' / 'Z' records,
    A/Z noise and random letters, at the extreme lengths of [l2_min, l2_max]. The periodic Seq1 makes most
    offsets tie, so the reference's tie-break (smallest offset, then k = 0) decides. ``copies`` repeats the
    list (shuffled) so the GPU kernels see every record length mixed in their waves."""
    rng = np.random.default_rng(seed)
    s1 = np.where(np.arange(L1) % 2 == 0, A, Z).astype(np.uint8)
    recs = []
    for L2 in sorted({l2_min, l2_max, (l2_min + l2_max) // 2, max(l2_min, l2_max - 1)}):
        for at in (0, 1, L1 - L2, L1 - L2 - 1):
            if 0 <= at and at + L2 <= L1:
                recs.append(s1[at:at + L2].copy())
        recs.append(np.full(L2, A, np.uint8))
        recs.append(np.full(L2, Z, np.uint8))
        recs.append(np.where(rng.integers(0, 2, L2) == 0, A, Z).astype(np.uint8))
        recs.append(rng.integers(1, 27, size=L2, dtype=np.uint8))
    order = np.concatenate([rng.permutation(len(recs)) for _ in range(copies)])
    lengths = np.array([len(recs[i]) for i in order], dtype=np.int64)
    offsets = np.zeros(len(order) + 1, dtype=np.int64)
    np.cumsum(lengths, out=offsets[1:])
    codes = np.concatenate([recs[i] for i in order]) if len(order) else np.zeros(0, np.uint8)
    return Problem(Weights.of(weights), s1, codes, offsets)
