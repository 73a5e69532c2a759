"""Problem container: weights + Seq1 + a CSR batch of Seq2 records (letters encoded 1..26).

Reference: int weights[4] (main.c:55), seq1 = malloc(3000) (main.c:66) and the fixed 2000-byte-stride
seq2_all buffer (main.c:93). Here records are packed CSR (codes + int64 offsets), the layout every
native engine, transport and kernel consumes.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import Iterable, Sequence

import numpy as np

from .. import _lib
from .scoring import Weights, decode, encode


def packed5_bytes(n_chars: int) -> int:
    """Bytes of a 5-bit packed letter stream (incl. 16 bytes of read slack)."""
    return int(_lib.lib().moc_packed5_bytes(int(n_chars)))


def pack5(codes: np.ndarray, out: np.ndarray = None) -> np.ndarray:
    """Byte letter codes (1..26) -> 5-bit packed stream (char j at bits [5j, 5j+5)); native + OpenMP.

    26 letters need only 5 bits, so every transfer of a packed batch (PCIe, xGMI, MPI) moves 37.5% fewer
    bytes; the gfx950 streaming kernel decodes the fields in registers."""
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    nb = packed5_bytes(codes.shape[0])
    if out is None:
        out = np.empty(nb, dtype=np.uint8)
    assert out.dtype == np.uint8 and out.shape[0] >= nb
    _lib.check(_lib.lib().moc_pack5(_lib.ptr(codes), codes.shape[0], _lib.ptr(out)))
    return out


def pack_lengths3(lengths: np.ndarray, base: int, out: np.ndarray = None) -> np.ndarray:
    """Record lengths in [base, base + 7] -> 3 bits each (record i at bits [3i, 3i+3), LSB first), plus
    one slack byte (the kernels read two bytes per length) — for batches whose lengths span <= 8 values
    (input6-shaped: 6..11), 25% fewer length bytes than nibbles."""
    v = np.asarray(lengths).astype(np.int64) - int(base)
    if v.size and (v.min() < 0 or v.max() > 7):
        raise ValueError("lengths do not fit 3 bits above the base")
    n = v.shape[0]
    nbytes = lengths3_bytes(n)
    if out is None:
        out = np.empty(nbytes, dtype=np.uint8)
    assert out.dtype == np.uint8 and out.shape[0] >= nbytes
    groups = (n + 7) // 8
    g = np.zeros(groups * 8, dtype=np.uint32)
    g[:n] = v
    g = g.reshape(groups, 8)
    word = np.zeros(groups, dtype=np.uint32)
    for k in range(8):
        word |= g[:, k] << np.uint32(3 * k)
    body = np.zeros((groups, 3), dtype=np.uint8)
    body[:, 0] = word & 0xFF
    body[:, 1] = (word >> 8) & 0xFF
    body[:, 2] = (word >> 16) & 0xFF
    flat = body.reshape(-1)
    m = min(flat.shape[0], nbytes)  # bytes past the last record's bits are zero anyway
    out[:m] = flat[:m]
    out[m:nbytes] = 0
    return out


def lengths3_bytes(n: int) -> int:
    return (3 * int(n) + 7) // 8 + 1 if n else 1


LEN_BASE6 = 6  # len_bits value of the base-6 form (moc::kLenBase6)


def lengths6_bytes(n: int) -> int:
    """Bytes of n base-6 lengths: 8-byte words of three 21-bit octets (24 records per word)."""
    return 8 * ((int(n) + 23) // 24)


def pack_lengths6(lengths: np.ndarray, base: int, out: np.ndarray = None) -> np.ndarray:
    """Record lengths in [base, base + 5] -> base 6: 8 records' lengths as one 21-bit number (record 8o + j
    = digit j of octet o, 6^8 < 2^21), three octets per little-endian 64-bit word at bits [21f, 21f+21) —
    2.667 bits per length for batches whose lengths span <= 6 values (input6-shaped: 6..11)."""
    v = np.asarray(lengths).astype(np.int64) - int(base)
    if v.size and (v.min() < 0 or v.max() > 5):
        raise ValueError("lengths do not fit base 6 above the base")
    n = v.shape[0]
    words = (n + 23) // 24
    if out is None:
        out = np.empty(8 * words, dtype=np.uint8)
    assert out.dtype == np.uint8 and out.shape[0] >= 8 * words
    d = np.zeros(words * 24, dtype=np.uint64)
    d[:n] = v
    d = d.reshape(words, 3, 8)
    octets = (d * (6 ** np.arange(8, dtype=np.uint64))).sum(axis=2, dtype=np.uint64)
    w = octets[:, 0] | (octets[:, 1] << np.uint64(21)) | (octets[:, 2] << np.uint64(42))
    out[:8 * words] = w.astype("<u8").view(np.uint8)
    return out


def pack_lengths4(lengths: np.ndarray, base: int, out: np.ndarray = None) -> np.ndarray:
    """Record lengths in [base, base + 15] -> 4 bits each, two per byte (record i in the low nibble of
    byte i // 2 when i is even, the high nibble when odd) — the streaming kernels' narrowest length form."""
    v = np.asarray(lengths).astype(np.int64) - int(base)
    if v.size and (v.min() < 0 or v.max() > 15):
        raise ValueError("lengths do not fit 4 bits above the base")
    n = v.shape[0]
    if out is None:
        out = np.empty((n + 1) // 2, dtype=np.uint8)
    lo = v[0::2].astype(np.uint8)
    hi = np.zeros_like(lo)
    hi[: n // 2] = v[1::2].astype(np.uint8)
    np.bitwise_or(lo, np.left_shift(hi, 4), out=out[: (n + 1) // 2])
    return out


def packed33_bytes(n_chars: int) -> int:
    """Bytes of a P33 letter stream (56 letters per 33 bytes, incl. 16 bytes of read slack)."""
    return int(_lib.lib().moc_packed33_bytes(int(n_chars)))


def pack33(codes: np.ndarray, out: np.ndarray = None) -> np.ndarray:
    """Byte letter codes (1..26) -> 33-bit fields: letters 7f..7f+6 as the value sum (code - 1) * 26^i at
    bits [33f, 33f+33) of a little-endian bit stream — 4.714 bits per letter (log2 26 = 4.700)."""
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    nb = packed33_bytes(codes.shape[0])
    if out is None:
        out = np.empty(nb, dtype=np.uint8)
    assert out.dtype == np.uint8 and out.shape[0] >= nb
    _lib.check(_lib.lib().moc_pack33(_lib.ptr(codes), codes.shape[0], _lib.ptr(out)))
    return out


def unpack33(packed: np.ndarray, begin: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.uint8)
    _lib.check(_lib.lib().moc_unpack33(_lib.ptr(np.ascontiguousarray(packed)), int(begin), int(n), _lib.ptr(out)))
    return out


def unpack5(packed: np.ndarray, begin: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.uint8)
    _lib.check(_lib.lib().moc_unpack5(_lib.ptr(np.ascontiguousarray(packed)), int(begin), int(n), _lib.ptr(out)))
    return out


@dataclass
class Problem:
    weights: Weights
    seq1: np.ndarray  # uint8 codes
    codes: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint8))  # uint8 codes, concatenated
    offsets: np.ndarray = field(default_factory=lambda: np.zeros(1, np.int64))  # int64, n+1

    def __post_init__(self):
        self.weights = Weights.of(self.weights)
        self.seq1 = np.ascontiguousarray(self.seq1, dtype=np.uint8)
        self.codes = np.ascontiguousarray(self.codes, dtype=np.uint8)
        self.offsets = np.ascontiguousarray(self.offsets, dtype=np.int64)

    # ------------------------------------------------------------------ construction
    @classmethod
    def from_strings(cls, weights: Sequence[int], seq1: str, seq2: Iterable[str]) -> "Problem":
        recs = [encode(s) for s in seq2]
        lengths = np.array([len(r) for r in recs], dtype=np.int64)
        offsets = np.zeros(len(recs) + 1, dtype=np.int64)
        np.cumsum(lengths, out=offsets[1:])
        codes = np.concatenate(recs) if recs else np.zeros(0, np.uint8)
        return cls(Weights.of(weights), encode(seq1), codes, offsets)

    @classmethod
    def parse(cls, text, strict_limits: bool = False) -> "Problem":
        """Parses the reference stdin format with the native OpenMP parser (csrc/src/io.cpp)."""
        if isinstance(text, str):
            text = text.encode()
        L = _lib.lib()
        h = L.moc_parse(text, len(text), 1 if strict_limits else 0)
        if not h:
            raise ValueError(L.moc_last_error().decode())
        try:
            w = (ctypes.c_int32 * 4)()
            l1, n, tot = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
            _lib.check(L.moc_problem_info(h, w, ctypes.byref(l1), ctypes.byref(n), ctypes.byref(tot)))

            def grab(p, count, dtype):
                if count == 0:
                    return np.zeros(0, dtype)
                buf = (ctypes.c_char * (count * np.dtype(dtype).itemsize)).from_address(p)
                return np.frombuffer(buf, dtype=dtype).copy()

            seq1 = grab(L.moc_problem_seq1(h), l1.value, np.uint8)
            codes = grab(L.moc_problem_codes(h), tot.value, np.uint8)
            offsets = grab(L.moc_problem_offsets(h), n.value + 1, np.int64)
            return cls(Weights.of(list(w)), seq1, codes, offsets)
        finally:
            L.moc_problem_free(h)

    @classmethod
    def read(cls, path, strict_limits: bool = False) -> "Problem":
        with open(path, "rb") as f:
            return cls.parse(f.read(), strict_limits)

    # ------------------------------------------------------------------ views
    @property
    def n(self) -> int:
        return int(self.offsets.shape[0] - 1)

    @property
    def L1(self) -> int:
        return int(self.seq1.shape[0])

    @property
    def lengths(self) -> np.ndarray:
        return np.diff(self.offsets)

    @property
    def total_chars(self) -> int:
        return int(self.offsets[-1] - self.offsets[0])

    def record(self, i: int) -> str:
        return decode(self.codes[self.offsets[i]:self.offsets[i + 1]])

    def seq1_str(self) -> str:
        return decode(self.seq1)

    def cells(self) -> int:
        """Candidate cells of the O(L1*L2) search: sum over records of (L1-L2+1)*L2 (0 if L2 > L1)."""
        L2 = self.lengths
        c = np.where(L2 <= self.L1, (self.L1 - L2 + 1) * L2, 0)
        return int(c.sum())

    def slice(self, b: int, e: int) -> "Problem":
        offs = self.offsets[b:e + 1]
        return Problem(self.weights, self.seq1, self.codes[offs[0]:offs[-1]], offs - offs[0])

    def to_text(self) -> str:
        """Serialises back to the reference stdin format (PDF p.5-6)."""
        w = self.weights.as_list()
        lines = [" ".join(map(str, w)), self.seq1_str(), str(self.n)]
        lines += [self.record(i) for i in range(self.n)]
        return "\n".join(lines) + "\n"
