"""Score table, parser and formatter units (SURVEY.md §4.3 'unit')."""
import numpy as np
import pytest

from mpi_openmp_cuda_amd import PairClass, Problem, format_results
from mpi_openmp_cuda_amd.models.scoring import (FIRST_TYPE_GROUPS, SECOND_TYPE_GROUPS, alignment_string, class_table,
                                                pair_class, score_table)
from mpi_openmp_cuda_amd.ops.align import native_score_table
from mpi_openmp_cuda_amd.utils.io import format_results_py


def test_groups_match_spec():
    assert len(FIRST_TYPE_GROUPS) == 9 and len(SECOND_TYPE_GROUPS) == 11
    assert set(FIRST_TYPE_GROUPS) == {"NDEQ", "MILV", "FYW", "NEQK", "QHRK", "HY", "STA", "NHQK", "MILF"}


@pytest.mark.parametrize("w", [(10, 2, 3, 4), (4, 3, 2, 10), (100, 2, 3, 4), (0, 0, 0, 0)])
def test_native_table_matches_python(w):
    assert np.array_equal(native_score_table(w), score_table(w))


def test_table_symmetric_and_fully_initialised():
    t = class_table()
    assert np.array_equal(t, t.T)
    assert set(np.unique(t)) <= {0, 1, 2, 3}
    for a in range(1, 27):
        assert t[a, a] == PairClass.DOLLAR
    # padding rows/cols are "space" (bug B1: the reference left 416/729 entries uninitialised)
    assert (t[0, :] == PairClass.SPACE).all() and (t[:, 27:] == PairClass.SPACE).all()


def test_pdf_alignment_example():
    # PDF p.2-3: APQRSBATAV vs ASQRSEAVSL, W = 10 2 3 4 -> 5*10 - 2*2 - 2*3 - 1*4 = 36
    line = alignment_string("APQRSBATAV", "ASQRSEAVSL", 0, 0)
    assert line == "$#$$$ $#%%"
    assert pair_class("A", "S") == PairClass.PERCENT  # STA
    assert pair_class("P", "S") == PairClass.HASH  # STPA


def test_parser_crlf_lowercase_whitespace():
    text = b"10 2 3 4\r\napqrsbatav\r\n  2\r\n asqreavsl \r\n\tHELLO\r\n"
    p = Problem.parse(text)
    assert p.weights.as_list() == [10, 2, 3, 4]
    assert p.seq1_str() == "APQRSBATAV"
    assert p.n == 2 and p.record(0) == "ASQREAVSL" and p.record(1) == "HELLO"


def test_parser_large_parallel_path():
    # > 64 KiB record area -> the two-pass OpenMP tokeniser; order must be input order
    rng = np.random.default_rng(0)
    recs = ["".join(chr(65 + x) for x in rng.integers(0, 26, rng.integers(1, 40))) for _ in range(5000)]
    text = "1 2 3 4\nABCDEFGHIJKLMNOPQRSTUVWXYZ\n%d\n" % len(recs) + "\n".join(recs) + "\n"
    p = Problem.parse(text)
    assert p.n == len(recs)
    assert all(p.record(i) == recs[i] for i in range(0, len(recs), 97))
    assert p.record(len(recs) - 1) == recs[-1]


@pytest.mark.parametrize("text,msg", [
    (b"1 2 3\n", "W4"),
    (b"1 2 3 4\nABC\n3\nAB\nCD\n", "expected 3"),
    (b"1 2 3 4\nAB1C\n1\nAB\n", "non-letter"),
    (b"1 2 3 4\nABC\n1\nA-B\n", "non-letter"),
    (b"1 -2 3 4\nABC\n1\nAB\n", "out of range"),
    (b"1 2 3 4\nABC\nx\n", "integer"),
])
def test_parser_errors(text, msg):
    with pytest.raises(ValueError, match=msg):
        Problem.parse(text)


def test_strict_limits():
    long1 = "A" * 3001
    with pytest.raises(ValueError, match="limit"):
        Problem.parse(f"1 1 1 1\n{long1}\n1\nA\n", strict_limits=True)
    assert Problem.parse(f"1 1 1 1\n{long1}\n1\nA\n").L1 == 3001


def test_extra_tokens_ignored():
    p = Problem.parse(b"1 2 3 4\nABCD\n1\nAB\nEXTRA\n")
    assert p.n == 1 and p.record(0) == "AB"


def test_formatter_matches_python():
    r = np.array([[1, 2, 3], [-2**31, 0, 0], [2**31 - 1, 2999, 1999]], dtype=np.int32)
    assert format_results(r, first_index=7) == format_results_py(r, first_index=7)


@pytest.mark.parametrize("n", [0, 1, 7, 8, 9, 1000, 300_001])
def test_pack5_roundtrip(n):
    from mpi_openmp_cuda_amd.models.problem import pack5, packed5_bytes, unpack5

    rng = np.random.default_rng(n)
    codes = rng.integers(1, 27, n, dtype=np.uint8)
    p = pack5(codes)
    assert p.shape[0] == packed5_bytes(n) == (5 * n + 7) // 8 + 16
    assert np.array_equal(unpack5(p, 0, n), codes)
    if n > 10:
        assert np.array_equal(unpack5(p, 3, n - 5), codes[3:n - 2])
    # bit layout: char j at bits [5j, 5j+5) of the little-endian stream
    if n >= 2:
        assert (int(p[0]) & 31) == codes[0] and ((int(p[0]) >> 5) | ((int(p[1]) & 3) << 3)) == codes[1]


def test_roundtrip_text():
    p = Problem.from_strings([4, 3, 2, 10], "ABCDEFGHIJKLMNOPQRSTUVWXYZ", ["ABCDEF", "MNOPQRSTXXX"])
    q = Problem.parse(p.to_text())
    assert np.array_equal(p.codes, q.codes) and np.array_equal(p.offsets, q.offsets)


@pytest.mark.parametrize("n", [0, 1, 2, 7, 1000])
def test_pack_lengths4(n):
    from mpi_openmp_cuda_amd.models.problem import pack_lengths4

    rng = np.random.default_rng(n)
    L = rng.integers(6, 22, n)
    p = pack_lengths4(L, 6)
    assert p.shape[0] == (n + 1) // 2
    got = np.empty(n, np.int64)
    got[0::2] = (p & 15)[: (n + 1) // 2] + 6
    got[1::2] = (p >> 4)[: n // 2] + 6
    assert np.array_equal(got, L)
    with pytest.raises(ValueError):
        pack_lengths4(np.array([5, 30]), 6)


def test_r2_decode_python_and_native():
    # R2 code = (score - smin) * j + n * kw + k, 0xFFFF = none; python and native decoders agree
    from mpi_openmp_cuda_amd import _lib
    from mpi_openmp_cuda_amd.ops.align import as_triples

    smin, kw, j = -110, 11, 231
    trip = np.array([[-110, 0, 0], [44, 20, 10], [3, 7, 2], [-2**31, 0, 0]], np.int32)
    codes = np.array([(s - smin) * j + n * kw + k if s != -2**31 else 0xFFFF for s, n, k in trip], np.uint16)
    assert np.array_equal(as_triples(codes, r2=(smin, kw, j)), trip)
    out = np.empty(len(codes), _lib.RESULT_DTYPE)
    prm = np.array([smin, kw, j], np.int32)
    _lib.check(_lib.lib().moc_expand_results(_lib.ptr(codes), 3, len(codes), _lib.ptr(prm), _lib.ptr(out)))
    assert np.array_equal(as_triples(out), trip)
    with pytest.raises(ValueError):
        as_triples(codes)


def test_pack_lengths3_roundtrip():
    from mpi_openmp_cuda_amd.models.problem import lengths3_bytes, pack_lengths3

    rng = np.random.default_rng(3)
    for n in (0, 1, 7, 8, 9, 1001):
        lens = rng.integers(6, 14, n)
        out = pack_lengths3(lens, 6)
        assert out.shape[0] == lengths3_bytes(n)
        bits = np.unpackbits(out, bitorder="little")
        got = [int(bits[3 * i] + 2 * bits[3 * i + 1] + 4 * bits[3 * i + 2]) + 6 for i in range(n)]
        assert got == [int(x) for x in lens]
    with pytest.raises(ValueError):
        pack_lengths3(np.array([6, 14]), 6)
