"""Pure-Python oracles of the search, independent of the native code.

* ``brute_force`` replays the reference kernel's loops literally (cudaFunctions.cu:74-172, race-free
  reading): every (offset, mutant) candidate is re-scored from scratch, O(L1*L2^2).
* ``prefix_oracle`` is the O(L1*L2) closed form the engines implement, vectorised
  with numpy cumulative sums.
Both return (score, n, k) and follow the reference tie-break (first maximum in offset-major,
mutant-minor order, mutant 0 = no hyphen first).
"""
from __future__ import annotations

import numpy as np

from .scoring import Semantics, score_table

INT_MIN = -(2**31)


def brute_force(table: np.ndarray, s1: np.ndarray, s2: np.ndarray, semantics=Semantics.REFERENCE):
    L1, L2 = len(s1), len(s2)
    if L2 > L1:
        return (INT_MIN, 0, 0)
    if L2 == L1:
        return (int(sum(table[s2[i], s1[i]] for i in range(L2))), 0, 0)
    best = None
    for o in range(L1 - L2):
        for m in range(L2):
            s = 0
            for i in range(L2):
                j = i + o if (i < m or m == 0) else i + o + 1
                s += int(table[s2[i], s1[j]])
            if best is None or best[0] < s:
                best = (s, o, m)
    if Semantics.parse(semantics) == Semantics.SPEC:
        o = L1 - L2
        s = int(sum(table[s2[i], s1[i + o]] for i in range(L2)))
        if best is None or best[0] < s:
            best = (s, o, 0)
    return best


def prefix_oracle(table: np.ndarray, s1: np.ndarray, s2: np.ndarray, semantics=Semantics.REFERENCE):
    L1, L2 = len(s1), len(s2)
    if L2 > L1:
        return (INT_MIN, 0, 0)
    s1 = np.asarray(s1, dtype=np.int64)
    s2 = np.asarray(s2, dtype=np.int64)
    if L2 == L1:
        return (int(table[s2, s1].sum()), 0, 0)
    nd = L1 - L2 + 1  # diagonals 0..L1-L2
    idx = np.arange(L2)[None, :] + np.arange(nd)[:, None]  # [nd, L2]
    cell = table[s2[None, :], s1[idx]].astype(np.int64)
    P = np.concatenate([np.zeros((nd, 1), np.int64), np.cumsum(cell, axis=1)], axis=1)  # P[d, k]
    tot = P[:, L2]
    n_off = L1 - L2
    # candidates per offset o < n_off: k = 0 -> tot[o]; k >= 1 -> P[o,k] - P[o+1,k] + tot[o+1]
    scores = np.empty((n_off, L2), np.int64)
    scores[:, 0] = tot[:n_off]
    if L2 > 1:
        scores[:, 1:] = P[:n_off, 1:L2] - P[1:n_off + 1, 1:L2] + tot[1:n_off + 1, None]
    flat = scores.reshape(-1)
    best_i = int(np.argmax(flat))  # first maximum = reference order
    best = (int(flat[best_i]), best_i // L2, best_i % L2)
    if Semantics.parse(semantics) == Semantics.SPEC and int(tot[n_off]) > best[0]:
        best = (int(tot[n_off]), n_off, 0)
    return best


def solve_problem(problem, semantics=Semantics.REFERENCE, oracle=prefix_oracle):
    """Runs an oracle over every record of a Problem; returns an (n, 3) int64 array."""
    t = score_table(problem.weights)
    out = np.zeros((problem.n, 3), np.int64)
    for i in range(problem.n):
        s2 = problem.codes[problem.offsets[i]:problem.offsets[i + 1]]
        out[i] = oracle(t, problem.seq1, s2, semantics)
    return out
