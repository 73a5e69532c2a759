"""The alignment "model": letter alphabet, conservation groups, pair classes and the fused score table.

Reference: the group strings hard-coded at main.c:59-60 (spec: parallel_finalEx2021_summer.pdf p.1-2),
the two 27x27 membership matrices of build_mat (main.c:14-44) and the class if/else chain of
calc_result (cudaFunctions.cu:132-153). The framework fuses the chain and the weights into one int32
table T[a][b] (+W1 / -W2 / -W3 / -W4), built natively (csrc/src/score_table.cpp); this module is the
pure-Python statement of the same rules, used as an independent test oracle.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass
from typing import Sequence

import numpy as np

FIRST_TYPE_GROUPS = ("NDEQ", "NEQK", "STA", "MILV", "QHRK", "NHQK", "FYW", "HY", "MILF")
SECOND_TYPE_GROUPS = ("SAG", "ATV", "CSA", "SGND", "STPA", "STNK", "NEQHRK", "NDEQHK", "SNDEQK", "HFY", "FVLIM")

LUT_STRIDE = 32  # rows padded to 32 ints on the device


class PairClass(enum.IntEnum):
    DOLLAR = 0  # '$' identical
    PERCENT = 1  # '%' same first-type group
    HASH = 2  # '#' same second-type group
    SPACE = 3  # ' ' otherwise

    @property
    def char(self) -> str:
        return "$%# "[int(self)]


class Semantics(enum.IntEnum):
    """Candidate set. REFERENCE reproduces cudaFunctions.cu:116 (offsets [0, L1-L2)); SPEC also tries the
    un-mutated sequence at the final offset n = L1-L2 (PDF p.3; SURVEY.md bug B8)."""

    REFERENCE = 0
    SPEC = 1

    @classmethod
    def parse(cls, s) -> "Semantics":
        if isinstance(s, Semantics):
            return s
        return {"reference": cls.REFERENCE, "ref": cls.REFERENCE, "spec": cls.SPEC}[str(s).lower()]


def letter_code(ch: str) -> int:
    c = ord(ch.upper()) - ord("A") + 1
    if not 1 <= c <= 26:
        raise ValueError(f"non-letter character {ch!r}")
    return c


def encode(seq: str) -> np.ndarray:
    """Letters (any case) -> uint8 codes 1..26."""
    b = np.frombuffer(seq.upper().encode("ascii"), dtype=np.uint8)
    if b.size and (b.min() < ord("A") or b.max() > ord("Z")):
        raise ValueError("sequence contains a non-letter character")
    return (b - (ord("A") - 1)).astype(np.uint8)


def decode(codes: np.ndarray) -> str:
    return (np.asarray(codes, dtype=np.uint8) + (ord("A") - 1)).tobytes().decode("ascii")


def pair_class(a: str, b: str) -> PairClass:
    """Classify a (Seq2 letter, Seq1 letter) pair exactly as the spec/reference chain does."""
    a, b = a.upper(), b.upper()
    if a == b:
        return PairClass.DOLLAR
    if any(a in g and b in g for g in FIRST_TYPE_GROUPS):
        return PairClass.PERCENT
    if any(a in g and b in g for g in SECOND_TYPE_GROUPS):
        return PairClass.HASH
    return PairClass.SPACE


@dataclass(frozen=True)
class Weights:
    w1: int
    w2: int
    w3: int
    w4: int

    @classmethod
    def of(cls, w: Sequence[int]) -> "Weights":
        if isinstance(w, Weights):
            return w
        w = [int(x) for x in w]
        if len(w) != 4 or min(w) < 0:
            raise ValueError("weights must be four non-negative integers (PDF p.2)")
        return cls(*w)

    def as_list(self):
        return [self.w1, self.w2, self.w3, self.w4]

    def class_value(self, c: PairClass) -> int:
        return [self.w1, -self.w2, -self.w3, -self.w4][int(c)]


def class_table() -> np.ndarray:
    """[32, 32] uint8 PairClass table over letter codes (row = Seq2 letter, col = Seq1 letter)."""
    t = np.full((LUT_STRIDE, LUT_STRIDE), int(PairClass.SPACE), dtype=np.uint8)
    for a in range(1, 27):
        for b in range(1, 27):
            t[a, b] = int(pair_class(chr(64 + a), chr(64 + b)))
    return t


def score_table(weights) -> np.ndarray:
    """[32, 32] int32 fused score table (pure Python statement of ScoreTable::build)."""
    w = Weights.of(weights)
    vals = np.array([w.w1, -w.w2, -w.w3, -w.w4], dtype=np.int32)
    return vals[class_table()]


def alignment_string(seq1: str, seq2: str, n: int, k: int) -> str:
    """The '$%# ' marker line of the spec's worked examples for Seq2 placed at offset n with mutant k
    (k = 0: no hyphen; k >= 1: hyphen after the k-th letter, facing Seq1[n+k], not scored)."""
    out = []
    for i, ch in enumerate(seq2):
        j = i + n if (k == 0 or i < k) else i + n + 1
        out.append(pair_class(ch, seq1[j]).char)
    if k:
        out.insert(k, "-")
    return "".join(out)
