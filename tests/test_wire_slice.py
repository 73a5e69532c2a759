"""WireSlice (mpi_openmp_cuda_amd/parallel/wire.py): the wire formats shared by bench.py's headline step and
the distributed driver's GPU ranks must encode any CSR slice losslessly — letters 5-bit packed or bytes,
lengths in 3/4/8-bit fields or offsets only — whatever allocator places the arrays."""
import numpy as np
import pytest

from mpi_openmp_cuda_amd.parallel.wire import WireSlice, length_bits
from mpi_openmp_cuda_amd.utils.synthetic import make_synthetic


@pytest.mark.parametrize("lo,hi,narrow,bits", [(6, 11, True, 6), (6, 13, True, 3), (6, 11, False, 8),
                                               (5, 20, True, 4), (1, 200, True, 8), (1, 300, True, 0),
                                               (7, 7, True, 6)])
def test_length_fields_round_trip(lo, hi, narrow, bits):
    rng = np.random.default_rng(lo * 1000 + hi)
    n = 1001
    lengths = rng.integers(lo, hi + 1, size=n)
    letters = rng.integers(1, 27, size=int(lengths.sum()), dtype=np.uint8)
    assert length_bits(int(lengths.min()), int(lengths.max()), narrow) == bits
    for fmt in ("p33", "p5", "bytes"):
        ws = WireSlice(lengths, letters, letter_format=fmt, narrow=narrow)
        assert ws.len_bits == bits
        assert np.array_equal(ws.decoded_lengths(), lengths)
        assert np.array_equal(ws.offsets[1:], np.cumsum(lengths))
        assert np.array_equal(ws.letters(), letters)
        i = n // 2  # any record's letters from its offset
        b, e = int(ws.offsets[i]), int(ws.offsets[i + 1])
        assert np.array_equal(ws.letters(b, e), letters[b:e])


def test_from_csr_slice_of_absolute_offsets():
    prob = make_synthetic("input6", 5000, seed=3)
    b, e = 1234, 4321
    ws = WireSlice.from_csr(prob.codes, prob.offsets[b:e + 1])
    assert ws.n == e - b
    assert np.array_equal(ws.decoded_lengths(), np.diff(prob.offsets[b:e + 1]))
    assert np.array_equal(ws.letters(), prob.codes[prob.offsets[b]:prob.offsets[e]])
    assert ws.letter_format == "p33" and ws.len_bits == 6 and ws.len_base == 6


def test_custom_allocator_places_every_array():
    names = []

    def alloc(name, dtype, count):
        names.append(name)
        return np.zeros(count, dtype=dtype)

    prob = make_synthetic("input6", 100, seed=1)
    ws = WireSlice.from_csr(prob.codes, prob.offsets, alloc=alloc)
    assert names == ["offsets", "lengths6", "codes33"]
    assert len(ws.arrays()) == 3  # results come later (their format is the engine's choice)


def test_p33_fields():
    from mpi_openmp_cuda_amd.models.problem import pack33, packed33_bytes

    codes = np.array([2, 1, 1, 1, 1, 1, 26] + [26] * 7 + [3], np.uint8)
    p = pack33(codes)
    stream = int.from_bytes(bytes(p[:33]), "little")
    mask = (1 << 33) - 1
    assert stream & mask == 1 + 25 * 26 ** 6
    assert (stream >> 33) & mask == 26 ** 7 - 1
    assert (stream >> 66) & mask == 2
    # 4.714 bits per letter: 33 bytes per 56 letters (5-bit packing: 35)
    n = 56 * 1000
    assert packed33_bytes(n) - 16 == 33000 and (5 * n // 8) == 35000


def test_base6_lengths_match_native_packer():
    # the numpy packer (WireSlice, bench.py) and the native one (final's parser) write the same words
    from mpi_openmp_cuda_amd import _lib
    from mpi_openmp_cuda_amd.models.problem import lengths6_bytes, pack_lengths6

    rng = np.random.default_rng(6)
    for n in (1, 7, 8, 23, 24, 25, 1000, 99_991):
        lengths = rng.integers(6, 12, size=n)
        offsets = np.zeros(n + 1, np.int64)
        np.cumsum(lengths, out=offsets[1:])
        got = pack_lengths6(lengths, 6)
        assert got.shape[0] == lengths6_bytes(n) == 8 * ((n + 23) // 24)
        want = np.zeros_like(got)
        _lib.check(_lib.lib().moc_pack_lengths(_lib.ptr(offsets), n, 6, 6, _lib.ptr(want)))
        assert np.array_equal(got, want), n
    with pytest.raises(ValueError):
        pack_lengths6(np.array([6, 12]), 6)


def test_prepared_solve_passes_the_checked_arguments(monkeypatch):
    # WireSlice.solve marshals the native arguments once and replays them: the replay must equal what the
    # checked HipSearchEngine.solve passes, and a new result array must go through the checked path again
    import ctypes

    from mpi_openmp_cuda_amd import _lib
    from mpi_openmp_cuda_amd.ops.align import HipSearchEngine

    calls = []

    class Stub:
        def __getattr__(self, name):
            return lambda *a: (calls.append((name, a)) or 0)

    monkeypatch.setattr(_lib, "lib", lambda: Stub())
    eng = HipSearchEngine.__new__(HipSearchEngine)
    eng._h, eng._problem_key, eng._stats_buf = ctypes.c_void_p(1), None, (ctypes.c_double * 14)()
    prob = make_synthetic("input6", 5000, seed=2)
    for fmt in ("p33", "p5", "bytes"):
        ws = WireSlice.from_csr(prob.codes, prob.offsets, letter_format=fmt)
        ws.fmt, ws.results = "r2", np.zeros(ws.n, np.uint16)
        ws.solve(eng)
        ws.solve(eng)
        (n1, a1), (n2, a2) = calls[-2], calls[-1]
        val = lambda args: [getattr(x, "value", x) for x in args[1:]]
        assert n1 == n2 == "moc_engine_solve_ex" and val(a1) == val(a2), fmt
        ws.results = np.zeros(ws.n, np.uint16)  # another result array: re-marshalled
        ws.solve(eng)
        assert val(calls[-1][1])[6] == ws.results.ctypes.data
    # set_problem: an unchanged problem makes no native call
    w, s1 = np.array([4, 3, 2, 10], np.int32), prob.seq1
    eng.set_problem(w, s1)
    k = len(calls)
    eng.set_problem(w.copy(), s1.copy())
    assert len(calls) == k
    eng.set_problem(np.array([4, 3, 2, 9], np.int32), s1)
    assert len(calls) == k + 1
