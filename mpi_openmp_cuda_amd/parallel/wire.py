"""One rank's slice of records in the wire formats the GPU streams (csrc/include/moc/wire.hpp).

``./final`` writes these forms straight from its parser (``BulkParser::fill_slice``): letters as 33-bit
fields of 7 (P33, 4.714 bits per letter; or 5-bit packed, or bytes: the staged / device-resident forms),
record lengths as base-6 octets or 3/4-bit fields above the slice's shortest length (8-bit, or offsets only, when the range
is wider), results in the narrowest format the problem's bounds allow (R2: one uint16 per record). The
streaming kernel reads them zero-copy from page-locked host memory, so every byte saved is PCIe time saved.

Shared by ``bench.py`` (the headline step) and :mod:`.search` (the distributed driver that the golden tests
run on GPU ranks), so the headline's data path is the one the goldens pin. Reference: the fixed 2000-byte
record stride and three int result arrays (main.c:93,123-125).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np

from ..models.problem import (LEN_BASE6, lengths3_bytes, lengths6_bytes, pack5, pack33, pack_lengths3, pack_lengths4,
                              pack_lengths6, packed5_bytes, packed33_bytes, unpack5, unpack33)

LETTER_FORMATS = ("p33", "p5", "bytes")

# allocator(name, dtype, count) -> array: private numpy memory, /dev/shm memmaps, hipHostMalloc buffers, ...
Alloc = Callable[[str, np.dtype, int], np.ndarray]


def private_alloc(name: str, dtype, count: int) -> np.ndarray:
    return np.empty(count, dtype=dtype)


def length_bits(l2_min: int, l2_max: int, narrow: bool = True) -> int:
    """Length form: 6 (base 6, 2.667 bits), 3 or 4 bits above the minimum when the range allows, else 8
    (0: offsets only)."""
    span = l2_max - l2_min
    if narrow and span <= 5:
        return LEN_BASE6
    if narrow and span <= 7:
        return 3
    if narrow and span <= 15:
        return 4
    return 8 if l2_max <= 255 else 0


class WireSlice:
    """A CSR slice (record lengths + byte letter codes 1..26) encoded once into the wire formats.

    ``letters``: ``p33`` (default), ``p5`` or ``bytes``; ``alloc`` places every array (so a benchmark
    can put them in node-shared or hipHostMalloc memory)."""

    def __init__(self, lengths: np.ndarray, letters: Optional[np.ndarray], letter_format: str = "p33",
                 narrow: bool = True, alloc: Alloc = private_alloc):
        if letter_format not in LETTER_FORMATS:
            raise ValueError(f"letter_format must be one of {LETTER_FORMATS}")
        lengths = np.asarray(lengths)
        n = int(lengths.shape[0])
        self.n = n
        self.alloc = alloc
        self.l2_min = int(lengths.min()) if n else 0
        self.l2_max = int(lengths.max()) if n else 0
        self.narrow = bool(narrow)
        self.offsets = alloc("offsets", np.int64, n + 1)
        self.offsets[0] = 0
        np.cumsum(lengths, out=self.offsets[1:])
        self.total = int(self.offsets[-1])
        self.len_bits = length_bits(self.l2_min, self.l2_max, narrow)
        self.len_base = self.l2_min if self.len_bits in (3, 4, LEN_BASE6) else 0
        if self.len_bits == LEN_BASE6:
            self.lengths = alloc("lengths6", np.uint8, lengths6_bytes(n))
            pack_lengths6(lengths, self.len_base, out=self.lengths)
        elif self.len_bits == 3:
            self.lengths = alloc("lengths3", np.uint8, lengths3_bytes(n))
            pack_lengths3(lengths, self.len_base, out=self.lengths)
        elif self.len_bits == 4:
            self.lengths = alloc("lengths4", np.uint8, (n + 1) // 2)
            pack_lengths4(lengths, self.len_base, out=self.lengths)
        elif self.len_bits == 8:
            self.lengths = alloc("lengths", np.uint8, n)
            self.lengths[:] = lengths
        else:
            self.lengths = None
        self.letter_format = letter_format
        if letter_format == "p33":
            self.codes = alloc("codes33", np.uint8, packed33_bytes(self.total))
            if letters is not None:
                pack33(letters, out=self.codes)
        elif letter_format == "p5":
            self.codes = alloc("codes5", np.uint8, packed5_bytes(self.total))
            if letters is not None:
                pack5(letters, out=self.codes)
        else:
            self.codes = alloc("codes", np.uint8, self.total)
            if letters is not None:
                self.codes[:] = letters
        self.fmt: Optional[str] = None
        self.results: Optional[np.ndarray] = None

    @classmethod
    def from_csr(cls, codes: np.ndarray, offsets: np.ndarray, **kw) -> "WireSlice":
        """Records [codes[offsets[i]:offsets[i+1]]] (offsets may be a slice of an absolute offset array)."""
        offsets = np.asarray(offsets, dtype=np.int64)
        return cls(np.diff(offsets), np.asarray(codes)[offsets[0]:offsets[-1]], **kw)

    # ---- results
    def alloc_results(self, engine, fmt: str = "auto") -> np.ndarray:
        """Results in ``fmt`` (auto: the narrowest the engine can produce for this slice's lengths)."""
        from .. import _lib

        if fmt == "auto":
            fmt = engine.auto_format(self.l2_max, self.l2_min if self.narrow else 0)
        self.fmt = fmt
        self.results = self.alloc("results", _lib.FORMAT_DTYPES[_lib.FORMAT_NAMES.index(fmt)], self.n)
        return self.results

    def arrays(self):
        """Every host array the engine streams (for page-locking)."""
        return [a for a in (self.codes, self.offsets, self.lengths, self.results) if a is not None]

    def solve(self, engine) -> np.ndarray:
        """One search of the slice into ``results`` (zero-copy when every array is page-locked). The native
        arguments are marshalled on the first call and reused while the engine and result array stay the same
        (a job loop over one slice pays no per-call argument conversion)."""
        if self.results is None:
            self.alloc_results(engine)
        prepared = getattr(self, "_prepared", None)
        if prepared is not None and prepared[0] is engine and prepared[1] is self.results:
            engine.solve_prepared(prepared[2])
            return self.results
        from .. import _lib

        fid = _lib.FORMAT_NAMES.index(self.fmt)
        letters = {"p5": 1, "p33": 3}.get(self.letter_format, 0)
        args = (_lib.ptr(self.codes), _lib.ptr(self.offsets), _lib.ptr(self.lengths), int(self.len_bits or 8),
                int(self.len_base), self.n, _lib.ptr(self.results), fid, int(self.l2_min), int(self.l2_max), letters)
        self._prepared = (engine, self.results, args)
        self._solve_checked(engine)
        return self.results

    def _solve_checked(self, engine) -> np.ndarray:
        """The first solve through the engine's checked entry point (asserts shapes and formats)."""
        return engine.solve(self.codes, self.offsets, out=self.results, lengths=self.lengths, fmt=self.fmt,
                            l2_range=(self.l2_min, self.l2_max), packed5=self.letter_format == "p5",
                            packed33=self.letter_format == "p33",
                            lengths_bits=self.len_bits or 8, lengths_base=self.len_base)

    def triples(self, engine, count: Optional[int] = None) -> np.ndarray:
        """The first ``count`` results as int32 [n, 3] (score, n, k)."""
        from ..ops.align import as_triples

        m = self.n if count is None else count
        r2 = engine.r2_params(self.l2_min, self.l2_max) if self.fmt == "r2" else None
        return as_triples(self.results[:m], r2=r2)

    # ---- decoding (tests, verification)
    def letters(self, begin: int = 0, end: Optional[int] = None) -> np.ndarray:
        end = self.total if end is None else end
        if self.letter_format == "p33":
            return unpack33(self.codes, begin, end - begin)
        if self.letter_format == "p5":
            return unpack5(self.codes, begin, end - begin)
        return np.asarray(self.codes[begin:end])

    def decoded_lengths(self) -> np.ndarray:
        """Record lengths back from the narrow fields (or the offsets when there are none)."""
        n = self.n
        if self.len_bits == LEN_BASE6:
            w = np.asarray(self.lengths[:lengths6_bytes(n)]).view("<u8").astype(np.uint64)
            octets = np.stack([(w >> np.uint64(21 * f)) & np.uint64(0x1FFFFF) for f in range(3)], axis=1).reshape(-1)
            digits = (octets[:, None] // (6 ** np.arange(8, dtype=np.uint64))) % np.uint64(6)
            return digits.reshape(-1)[:n].astype(np.int64) + self.len_base
        if self.len_bits == 3:
            b = np.zeros(lengths3_bytes(n) + 4, np.uint8)
            b[:self.lengths.shape[0]] = self.lengths
            bit = 3 * np.arange(n, dtype=np.int64)
            w = b[bit >> 3].astype(np.int64) | (b[(bit >> 3) + 1].astype(np.int64) << 8)
            return ((w >> (bit & 7)) & 7) + self.len_base
        if self.len_bits == 4:
            v = np.asarray(self.lengths[:(n + 1) // 2])
            out = np.empty(2 * v.shape[0], np.int64)
            out[0::2] = v & 15
            out[1::2] = v >> 4
            return out[:n] + self.len_base
        if self.len_bits == 8:
            return np.asarray(self.lengths[:n]).astype(np.int64)
        return np.diff(self.offsets)
