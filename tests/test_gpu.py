"""GPU (MI355X / gfx950) tests: HIP engine == CPU engine == goldens. Numerics oracle: the CPU engine,
itself pinned to the brute-force replay of the reference loops (test_oracles.py)."""
import json

import numpy as np
import pytest

from conftest import expected, gpu_available, input_path, run_final

pytestmark = pytest.mark.gpu

if not gpu_available():  # pragma: no cover - collected on CPU hosts only with -m gpu
    pytest.skip("no GPU", allow_module_level=True)

import torch  # noqa: E402

from mpi_openmp_cuda_amd import (HipSearchEngine, Problem, Semantics, brute_force_native, format_results,  # noqa: E402
                                 make_synthetic, search_cpu)
from mpi_openmp_cuda_amd.ops.align import align_search_device, as_triples, device_info  # noqa: E402


@pytest.fixture(scope="module")
def engine():
    e = HipSearchEngine(device=0)
    yield e
    e.close()


def check(engine, prob, sem=Semantics.REFERENCE):
    engine.set_problem(prob.weights, prob.seq1, sem)
    got = as_triples(engine.solve(prob.codes, prob.offsets))
    ref = as_triples(search_cpu(prob, sem))
    bad = np.nonzero((got != ref).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} mismatches, first #{bad[:5]}: got {got[bad[:5]]} ref {ref[bad[:5]]}"
    return got


def test_dpp_primitives():
    # the kernels rely on DPP wave_shl:1 = "lane i reads lane i+1", lane 63 bound (0 or fill value)
    from mpi_openmp_cuda_amd import _lib

    out = np.zeros(192, np.int32)
    _lib.check(_lib.lib().moc_dpp_probe(_lib.ptr(out)))
    assert out[:63].tolist() == list(range(1, 64)) and out[63] == 0
    assert out[64:127].tolist() == list(range(1, 64)) and out[127] == 777
    assert (out[128:] == 60).all()


def test_mfma_i8_layout():
    # the matrix-core sweep relies on the i8 32x32x32 operand packing (element j of lane half h <-> k = 16h + j,
    # the same for A and B) and the C layout row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5): checked with
    # asymmetric integer data against a host product
    from mpi_openmp_cuda_amd import _lib

    rng = np.random.default_rng(11)
    a = rng.integers(-128, 128, size=(32, 32)).astype(np.int8)
    b = rng.integers(-128, 128, size=(32, 32)).astype(np.int8)
    c = np.zeros((32, 32), np.int32)
    _lib.check(_lib.lib().moc_mfma_i8_probe(_lib.ptr(a), _lib.ptr(b), _lib.ptr(c)))
    assert np.array_equal(c, a.astype(np.int32) @ b.astype(np.int32))


@pytest.mark.parametrize("shape,n,L1", [("input3", 24, None), ("input4", 60, None), ("input3", 6, 3000),
                                        ("input1", 300, 700)])
def test_mfma_sweep_matches_cpu(monkeypatch, shape, n, L1):
    # MOC_MFMA=1: the long-record sweep on the matrix cores (tile_mfma_kernels.hip) == the CPU engine,
    # both semantics, records longer and shorter than Seq1, ties resolved to the reference's order
    monkeypatch.setenv("MOC_MFMA", "1")
    eng = HipSearchEngine(device=0)
    prob = make_synthetic(shape, n, seed=n + 3)
    if L1:
        rng = np.random.default_rng(L1)
        prob = Problem(prob.weights, rng.integers(1, 27, size=L1, dtype=np.uint8), prob.codes, prob.offsets)
    for sem in (Semantics.REFERENCE, Semantics.SPEC):
        eng.set_problem(prob.weights, prob.seq1, sem)
        got = as_triples(eng.solve(prob.codes, prob.offsets))
        assert np.array_equal(got, as_triples(search_cpu(prob, sem))), sem
    assert "tile16" in eng.stats()["kernels"], eng.stats()


def test_device_is_gfx950():
    info = device_info(0)
    assert info["arch"].startswith("gfx950"), info
    assert info["wave"] == 64


@pytest.mark.parametrize("i", [1, 2, 3, 4, 5, 6])
def test_goldens(engine, i):
    prob = Problem.read(input_path(i))
    engine.set_problem(prob.weights, prob.seq1)
    assert format_results(engine.solve(prob.codes, prob.offsets)) == expected(i)


@pytest.mark.parametrize("shape,n", [("input6", 5000), ("input1", 700), ("input3", 40), ("input4", 300),
                                     ("limits", 24)])
@pytest.mark.parametrize("sem", [Semantics.REFERENCE, Semantics.SPEC])
def test_random_shapes(engine, shape, n, sem):
    check(engine, make_synthetic(shape, n, seed=n), sem)


def test_mixed_packed_and_tiles(engine):
    # one batch mixing packed records (offset range <= 64), tile records, equal length and L2 > L1
    rng = np.random.default_rng(7)
    s1 = "".join(chr(65 + x) for x in rng.integers(0, 26, 300))
    recs = [s1, s1 + "A", s1[:250], s1[5:299], "A", "AB", s1[::3]]
    recs += ["".join(chr(65 + x) for x in rng.integers(0, 26, rng.integers(1, 300))) for _ in range(200)]
    prob = Problem.from_strings([5, 1, 2, 3], s1, recs)
    for sem in (Semantics.REFERENCE, Semantics.SPEC):
        check(engine, prob, sem)
    got = as_triples(engine.solve(prob.codes, prob.offsets))
    assert tuple(got[1]) == (-2**31, 0, 0)


def test_small_brute_force(engine):
    rng = np.random.default_rng(3)
    for _ in range(20):
        L1 = int(rng.integers(1, 90))
        recs = ["".join(chr(65 + x) for x in rng.integers(0, 26, rng.integers(1, L1 + 3))) for _ in range(30)]
        s1 = "".join(chr(65 + x) for x in rng.integers(0, 26, L1))
        prob = Problem.from_strings(rng.integers(0, 12, 4), s1, recs)
        engine.set_problem(prob.weights, prob.seq1)
        got = as_triples(engine.solve(prob.codes, prob.offsets))
        assert np.array_equal(got, as_triples(brute_force_native(prob)))


def test_wide_keys(engine):
    # large weights force the 64-bit hot-loop key path
    prob = make_synthetic("limits", 12, seed=5)
    prob.weights = type(prob.weights)(200000, 100, 300, 2)
    check(engine, prob)


def test_chunked_pipeline():
    prob = make_synthetic("input6", 200_000, seed=11)
    eng = HipSearchEngine(device=0, chunk_records=30_000, chunk_bytes=1 << 18)
    check(eng, prob)
    st = eng.stats()
    assert st["chunks"] >= 7 and st["records"] == prob.n
    eng.close()


@pytest.mark.parametrize("fmt", ["r12", "r8", "r4"])
@pytest.mark.parametrize("use_lengths", [False, True])
def test_zero_copy_direct(fmt, use_lengths):
    # pinned host buffers + short records -> one streaming kernel reading/writing host memory
    prob = make_synthetic("input6", 300_001, seed=21)
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    from mpi_openmp_cuda_amd import _lib

    out = np.zeros(prob.n, dtype=_lib.FORMAT_DTYPES[_lib.FORMAT_NAMES.index(fmt)])
    lengths = np.diff(prob.offsets).astype(np.uint8) if use_lengths else None
    eng.pin(prob.codes, prob.offsets, out, lengths)
    eng.solve(prob.codes, prob.offsets, out=out, lengths=lengths, fmt=fmt)
    assert eng.stats()["direct"] == 1
    assert np.array_equal(as_triples(out), as_triples(search_cpu(prob)))
    eng.close()


@pytest.mark.parametrize("shape,n", [("input6", 250_003), ("input1", 3000), ("input4", 200), ("input3", 20)])
@pytest.mark.parametrize("pinned", [False, True])
def test_packed5_letters(shape, n, pinned):
    # 5-bit packed letters (the dense wire form): unpacked on the device by the staged pipeline, pinned or
    # not (the streaming kernels take P33 or byte letters)
    from mpi_openmp_cuda_amd.models.problem import pack5

    prob = make_synthetic(shape, n, seed=n)
    packed = pack5(prob.codes)
    eng = HipSearchEngine(device=0, chunk_records=max(n // 3, 1))
    eng.set_problem(prob.weights, prob.seq1)
    out = np.zeros(prob.n, dtype=np.dtype([("score", "<i4"), ("n", "<i4"), ("k", "<i4")]))
    if pinned:
        eng.pin(packed, prob.offsets, out)
    eng.solve(packed, prob.offsets, out=out, packed5=True)
    st = eng.stats()
    assert np.array_equal(as_triples(out), as_triples(search_cpu(prob))), st
    assert st["direct"] == 0, st
    if shape == "input6":
        assert st["kernels"] == ["swipe"], st
    eng.close()


@pytest.mark.parametrize("shape,n", [("input6", 250_003), ("input1", 3000), ("input4", 200), ("input3", 20)])
@pytest.mark.parametrize("pinned", [False, True])
def test_group_coded_letters(shape, n, pinned):
    # P33 letters (7 per 33-bit field): decoded per tile in LDS by the swipe kernel (pinned, tiny
    # problems), or unpacked on the host for the staged pipeline
    from mpi_openmp_cuda_amd.models.problem import pack33

    prob = make_synthetic(shape, n, seed=n + 1)
    packed = pack33(prob.codes)
    eng = HipSearchEngine(device=0, chunk_records=max(n // 3, 1))
    eng.set_problem(prob.weights, prob.seq1)
    out = np.zeros(prob.n, dtype=np.dtype([("score", "<i4"), ("n", "<i4"), ("k", "<i4")]))
    if pinned:
        eng.pin(packed, prob.offsets, out)
    eng.solve(packed, prob.offsets, out=out, packed33=True)
    st = eng.stats()
    assert np.array_equal(as_triples(out), as_triples(search_cpu(prob))), st
    if pinned and shape == "input6":
        assert st["direct"] == 1 and st["kernels"] == ["swipe"]
    eng.close()


@pytest.mark.parametrize("L1,lo,hi,w", [(26, 6, 11, (4, 3, 2, 10)), (12, 1, 14, (3, 1, 1, 2)),
                                        (40, 20, 32, (5, 2, 3, 4)), (60, 10, 16, (2, 2, 1, 3)),
                                        (9, 9, 9, (7, 1, 2, 3)), (51, 32, 41, (100, 2, 3, 4)),
                                        (70, 40, 64, (3, 1, 2, 1)), (30, 5, 12, (120, 1, 1, 1)),
                                        (130, 67, 85, (10, 2, 3, 4)), (190, 127, 128, (3, 1, 1, 2)),
                                        (40, 30, 40, (300, 2, 3, 4))])
@pytest.mark.parametrize("letters", ["p33", "p5"])
def test_swipe_wire_slices(L1, lo, hi, w, letters):
    # the headline's wire path (parallel/wire.py: narrow lengths, R2/R4 results, zero-copy) across swipe
    # instantiations (NOFF 8..64, record widths <= 16 / 32 / 64 / 96 / 128, keys with k bits and the RK form
    # that re-walks k, weights past 127) with P33 letters; 5-bit letters take the staged pipeline to the same
    # kernel
    from mpi_openmp_cuda_amd._lib import Pinned
    from mpi_openmp_cuda_amd.parallel.wire import WireSlice

    rng = np.random.default_rng(L1 * 7 + lo)
    s1 = "".join(chr(65 + x) for x in rng.integers(0, 26, L1))
    lens = rng.integers(max(1, min(lo, hi)), max(lo, hi) + 1, 20000)
    recs = ["".join(chr(65 + x) for x in rng.integers(0, 26, n)) for n in lens]
    prob = Problem.from_strings(w, s1, recs)
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    ws = WireSlice.from_csr(prob.codes, prob.offsets, letter_format=letters)
    ws.alloc_results(eng)
    with Pinned(*ws.arrays()):
        ws.solve(eng)
    st = eng.stats()
    assert np.array_equal(ws.triples(eng), as_triples(search_cpu(prob))), st
    if L1 - min(lo, hi) + 1 <= 64:
        assert st["kernels"] == ["swipe"] and st["direct"] == (1 if letters == "p33" else 0), st
    eng.close()


@pytest.mark.parametrize("L1,lo,hi", [(200, 150, 155), (210, 160, 165)])
def test_short_kernel_base6_lengths(L1, lo, hi):
    # byte letters + base-6 lengths through the lane-per-offset short kernel (records longer than 128 letters
    # leave the swipe kernel; at most 64 lanes per record keep them on the short one)
    from mpi_openmp_cuda_amd._lib import Pinned
    from mpi_openmp_cuda_amd.parallel.wire import WireSlice

    rng = np.random.default_rng(L1 + lo)
    s1 = "".join(chr(65 + x) for x in rng.integers(0, 26, L1))
    lens = rng.integers(lo, hi + 1, 30011)
    recs = ["".join(chr(65 + x) for x in rng.integers(0, 26, n)) for n in lens]
    prob = Problem.from_strings((3, 2, 1, 4), s1, recs)
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    ws = WireSlice.from_csr(prob.codes, prob.offsets, letter_format="bytes")
    assert ws.len_bits == 6
    ws.alloc_results(eng)
    with Pinned(*ws.arrays()):
        ws.solve(eng)
    st = eng.stats()
    assert np.array_equal(ws.triples(eng), as_triples(search_cpu(prob))), st
    assert st["direct"] == 1 and st["kernels"] == ["short"], st
    eng.close()


@pytest.mark.parametrize("fmt", ["r8", "r4", "auto"])
def test_staged_formats(engine, fmt):
    prob = make_synthetic("input1", 5000, seed=4)
    engine.set_problem(prob.weights, prob.seq1)
    got = engine.solve(prob.codes, prob.offsets, fmt=fmt)
    assert engine.stats()["direct"] == 0
    assert np.array_equal(as_triples(got, r2=engine.stats()["r2"]), as_triples(search_cpu(prob)))


@pytest.mark.parametrize("L1,lo,hi,w", [(26, 6, 11, (4, 3, 2, 10)), (12, 1, 14, (3, 1, 1, 2)),
                                        (40, 20, 32, (5, 2, 3, 4)), (60, 10, 16, (2, 2, 1, 3)),
                                        (100, 40, 32, (1, 1, 1, 1)), (9, 9, 9, (7, 1, 2, 3)),
                                        # the RK form (no k bits in the keys; k re-walked): input1's shape,
                                        # records <= 16 / <= 32 / <= 64 letters, 64 offsets per lane
                                        (51, 32, 41, (100, 2, 3, 4)), (30, 5, 12, (120, 1, 1, 1)),
                                        (40, 20, 30, (60, 2, 3, 4)), (70, 40, 64, (3, 1, 2, 1)),
                                        (40, 20, 40, (2, 1, 1, 1)), (56, 25, 56, (90, 7, 3, 5)),
                                        # 64 offsets and 64-letter records: the largest instance (8 profile
                                        # copies of 144-entry rows, 66 KB of LDS)
                                        (66, 3, 64, (2, 1, 1, 1))])
@pytest.mark.parametrize("sem", [Semantics.REFERENCE, Semantics.SPEC])
def test_swipe_kernel_shapes(engine, L1, lo, hi, w, sem):
    # lane-per-record packed-int16 kernel across offset widths (NOFF 8..64), record widths (<= 16, <= 32,
    # <= 64) and both key forms
    rng = np.random.default_rng(L1 * 100 + lo)
    s1 = "".join(chr(65 + x) for x in rng.integers(0, 26, L1))
    lens = rng.integers(max(1, min(lo, hi)), max(lo, hi) + 1, 3000)
    recs = ["".join(chr(65 + x) for x in rng.integers(0, 26, n)) for n in lens]
    prob = Problem.from_strings(w, s1, recs)
    engine.set_problem(prob.weights, prob.seq1, sem)
    got = engine.solve(prob.codes, prob.offsets, fmt="auto")
    kinds = engine.stats()["kernels"]
    assert np.array_equal(as_triples(got, r2=engine.stats()["r2"]), as_triples(search_cpu(prob, sem))), kinds
    if L1 - min(lo, hi) + 1 <= 64:
        assert kinds == ["swipe"], kinds


@pytest.mark.parametrize("noff", list(range(4, 65, 4)))
@pytest.mark.parametrize("sem", [Semantics.REFERENCE, Semantics.SPEC])
def test_swipe_every_offset_width(engine, noff, sem):
    # every swipe code object (offsets per lane: multiples of 4, sized by the semantics' widest record range:
    # L1 - L2 offsets under the reference, one more under the spec), host-streamed and device-resident,
    # against the CPU engine; the batch's shortest record needs exactly `noff` offsets (reference; 63 for the
    # widest instance: a record needing 65 lanes under the spec semantics belongs to the tile kernels)
    L1 = 70
    lo = L1 - noff + (1 if noff == 64 else 0)
    rng = np.random.default_rng(noff * 3 + int(sem == Semantics.SPEC))
    s1 = "".join(chr(65 + x) for x in rng.integers(0, 26, L1))
    lens = np.concatenate([[lo], rng.integers(lo, min(lo + 7, L1) + 1, 2999)])
    recs = ["".join(chr(65 + x) for x in rng.integers(0, 26, n)) for n in lens]
    prob = Problem.from_strings((4, 3, 2, 10), s1, recs)
    want = as_triples(search_cpu(prob, sem))
    engine.set_problem(prob.weights, prob.seq1, sem)
    got = engine.solve(prob.codes, prob.offsets, fmt="auto")
    assert engine.stats()["kernels"] == ["swipe"], engine.stats()
    assert np.array_equal(as_triples(got, r2=engine.stats()["r2"]), want)
    dev = torch.device("cuda:0")
    out = torch.empty((len(prob.offsets) - 1, 3), dtype=torch.int32, device=dev)
    engine.solve_device(torch.from_numpy(prob.codes).to(dev), torch.from_numpy(prob.offsets).to(dev), prob.offsets,
                        out)
    torch.cuda.synchronize()
    assert engine.stats()["kernels"] == ["swipe"], engine.stats()
    assert np.array_equal(out.cpu().numpy(), want)


def test_kernel_selection(engine):
    p6 = make_synthetic("input6", 2000, seed=1)
    engine.set_problem(p6.weights, p6.seq1)
    engine.solve(p6.codes, p6.offsets)
    assert engine.stats()["kernels"] == ["swipe"]
    p1 = make_synthetic("input1", 2000, seed=1)  # W1 = 100: no room for k in the int16 keys -> RK swipe
    engine.set_problem(p1.weights, p1.seq1)
    engine.solve(p1.codes, p1.offsets)
    assert engine.stats()["kernels"] == ["swipe"]
    engine.set_problem([300, 2, 3, 4], p1.seq1)  # W1 300, L2 <= 41: 2 W L2 < 2^15 still -> RK swipe
    got = engine.solve(p1.codes, p1.offsets)
    assert engine.stats()["kernels"] == ["swipe"]
    assert np.array_equal(as_triples(got), as_triples(search_cpu(Problem([300, 2, 3, 4], p1.seq1, p1.codes,
                                                                          p1.offsets))))
    engine.set_problem([500, 2, 3, 4], p1.seq1)  # 2 * 500 * 41 >= 2^15: the int16 sums would wrap -> lane/offset
    engine.solve(p1.codes, p1.offsets)
    assert engine.stats()["kernels"] == ["short"]
    p4 = make_synthetic("input4", 50, seed=1)  # long records: packed-int16 profile kernel
    engine.set_problem(p4.weights, p4.seq1)
    engine.solve(p4.codes, p4.offsets)
    assert engine.stats()["kernels"] == ["tile16"]
    engine.set_problem([120, 20, 1, 1], p4.seq1)  # Dt range 140 > 127: the int16 profile, widened windows
    got = engine.solve(p4.codes, p4.offsets)
    assert engine.stats()["kernels"] == ["tile16"] and "tile16_i16" in engine.stats()["forms"]
    assert np.array_equal(as_triples(got), as_triples(search_cpu(Problem([120, 20, 1, 1], p4.seq1, p4.codes,
                                                                          p4.offsets))))
    engine.set_problem([300, 300, 1, 1], p4.seq1)  # Dt range 600 > 511: past the int16 profile -> DPP tiles
    engine.solve(p4.codes, p4.offsets)
    assert engine.stats()["kernels"] == ["tiles"]


def _letters(rng, n, alphabet):
    return "".join(chr(65 + x) for x in rng.integers(0, alphabet, n))


@pytest.mark.parametrize("L1,weights,alphabet", [
    (3000, [10, 2, 3, 4], 26),     # reference buffer limit
    (3050, [100, 27, 5, 3], 3),    # largest Seq1 whose profile fits the LDS; T range 127; tie-heavy
    (700, [1, 0, 0, 0], 2),        # scores tie everywhere: the k re-walk must pick the smallest
    (200, [0, 0, 0, 0], 26),       # all zero
])
@pytest.mark.parametrize("sem", [Semantics.REFERENCE, Semantics.SPEC])
def test_tile16_edges(engine, L1, weights, alphabet, sem):
    rng = np.random.default_rng(L1 + alphabet)
    s1 = _letters(rng, L1, alphabet)
    lens = [1, 2, 63, 64, 65, 127, 128, 129, L1 - 64, L1 - 65, L1 - 1, L1, L1 + 1]
    lens += list(rng.integers(1, min(L1, 2000), 40))
    recs = [_letters(rng, n, alphabet) for n in lens] + [s1[3:L1 - 70], s1[::2]]
    prob = Problem.from_strings(weights, s1, recs)
    check(engine, prob, sem)
    assert "tile16" in engine.stats()["kernels"]


@pytest.mark.parametrize("L1,alphabet", [(3000, 26), (3040, 3), (1030, 2), (300, 5)])
def test_tile16_wide_tiles(engine, L1, alphabet):
    # short records (mean |Seq2| < 96) take 1024-offset tiles (U = 8) when the profile's 1024-entry
    # overhang fits the LDS (L1 3000, 1030, 300), 512-offset ones otherwise (L1 3040)
    rng = np.random.default_rng(L1 * 7 + alphabet)
    s1 = _letters(rng, L1, alphabet)
    lens = [1, 2, 63, 64, 65, 95, L1 - 1, L1, L1 + 1] + list(rng.integers(1, 60, 300))
    recs = [_letters(rng, n, alphabet) for n in lens]
    prob = Problem.from_strings([7, 2, 3, 1], s1, recs)
    for sem in (Semantics.REFERENCE, Semantics.SPEC):
        check(engine, prob, sem)
    assert "tile16" in engine.stats()["kernels"]


def test_short_config_fallback(engine):
    # records far longer than Seq1 blow the short kernel's LDS tile budget -> everything via tiles
    rng = np.random.default_rng(9)
    s1 = "".join(chr(65 + x) for x in rng.integers(0, 26, 30))
    recs = ["".join(chr(65 + x) for x in rng.integers(0, 26, n)) for n in (70000, 20, 29, 30, 31, 5)]
    prob = Problem.from_strings([3, 1, 2, 1], s1, recs)
    check(engine, prob)


def test_device_resident_torch(engine):
    prob = make_synthetic("input4", 64, seed=2)
    engine.set_problem(prob.weights, prob.seq1)
    dev = torch.device("cuda:0")
    codes_t = torch.from_numpy(prob.codes).to(dev)
    offs_t = torch.from_numpy(prob.offsets).to(dev)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        out = align_search_device(engine, codes_t, offs_t, prob.offsets, stream=s)
    s.synchronize()
    assert np.array_equal(out.cpu().numpy(), as_triples(search_cpu(prob)))


@pytest.mark.parametrize("i", [3, 6])
def test_final_cli_hip(i):
    r = run_final(["--backend=hip"], stdin_path=input_path(i), np_=1)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == expected(i)


@pytest.mark.parametrize("transport", ["shm", "mpi"])
def test_final_cli_two_ranks_one_gpu(transport):
    # two ranks share the single test GPU (RCCL needs distinct GPUs; shm/mpi transports do not)
    r = run_final(["--backend=hip", f"--transport={transport}", "--device=0"], stdin_path=input_path(4), np_=2)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == expected(4)


def test_final_cli_rccl_single_rank():
    r = run_final(["--backend=hip", "--transport=rccl"], stdin_path=input_path(3), np_=1)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == expected(3)


@pytest.mark.parametrize("shape,n", [("input3", 8), ("input4", 60), ("input1", 200), ("input6", 3000)])
@pytest.mark.parametrize("parts", [1, 2, 5])
def test_context_parallel_keys(engine, shape, n, parts):
    # GPU partial searches (shares of the global tile list) combine by MAX into the full search
    from mpi_openmp_cuda_amd import decode_keys, search_keys_cpu

    prob = make_synthetic(shape, n, seed=n + parts)
    for sem in (Semantics.REFERENCE, Semantics.SPEC):
        engine.set_problem(prob.weights, prob.seq1, sem)
        keys = np.zeros(prob.n, np.uint64)
        for part in range(parts):
            keys = np.maximum(keys, engine.search_keys(prob.codes, prob.offsets, part, parts))
        ref = as_triples(search_cpu(prob, sem))
        assert np.array_equal(as_triples(decode_keys(keys, prob)), ref)
        # each GPU share is a lower bound of the CPU full-range key (same encoding on both sides)
        full = search_keys_cpu(prob, 0, 1, sem)
        assert np.array_equal(keys, full)


@pytest.mark.parametrize("shape", ["limits", "heavylim"])
def test_context_parallel_keys_sliding_windows(engine, shape):
    # search_keys / search_keys_device with one part take the sliding-window plan (byte pairs and
    # the int16 profile) and 32-bit selection keys where the bounds allow; their keys equal the CPU's
    from mpi_openmp_cuda_amd import search_keys_cpu

    prob = make_synthetic(shape, 1024, seed=17)
    for sem in (Semantics.REFERENCE, Semantics.SPEC):
        engine.set_problem(prob.weights, prob.seq1, sem)
        want = search_keys_cpu(prob, 0, 1, sem)
        keys = engine.search_keys(prob.codes, prob.offsets, 0, 1)
        assert "tile16_slide" in engine.stats()["forms"], engine.stats()
        assert np.array_equal(keys, want)
        dev = torch.device("cuda:0")
        k = torch.zeros(prob.n, dtype=torch.int64, device=dev)
        engine.search_keys_device(torch.from_numpy(prob.codes).to(dev), torch.from_numpy(prob.offsets).to(dev),
                                  prob.offsets, 0, 1, k)
        torch.cuda.synchronize()
        assert "tile16_slide" in engine.stats()["forms"], engine.stats()
        assert np.array_equal(k.cpu().numpy().view(np.uint64), want)


def test_context_parallel_device_finalize(engine):
    prob = make_synthetic("input3", 6, seed=3)
    engine.set_problem(prob.weights, prob.seq1)
    dev = torch.device("cuda:0")
    codes_t = torch.from_numpy(prob.codes).to(dev)
    offs_t = torch.from_numpy(prob.offsets).to(dev)
    keys = torch.zeros(prob.n, dtype=torch.int64, device=dev)
    parts = []
    for part in range(3):
        k = torch.empty_like(keys)
        engine.search_keys_device(codes_t, offs_t, prob.offsets, part, 3, k)
        parts.append(k)
    torch.cuda.synchronize()
    # uint64 max == signed max after flipping the top bit
    flip = torch.tensor(-2**63, dtype=torch.int64, device=dev)
    best = torch.stack([p ^ flip for p in parts]).max(dim=0).values ^ flip
    out = torch.empty(prob.n, 3, dtype=torch.int32, device=dev)
    engine.finalize_keys_device(codes_t, offs_t, prob.offsets, best, out)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), as_triples(search_cpu(prob)))


@pytest.mark.parametrize("args", [["--partition=offsets", "--transport=shm"], ["--partition=offsets", "--transport=rccl"],
                                  ["--partition=offsets", "--transport=mpi"], ["--batch-records=3"],
                                  ["--batch-records=2", "--transport=rccl"], ["--pin-window=0"], ["--collectives=rccl"],
                                  ["--partition=offsets", "--transport=shm", "--collectives=rccl"]])
def test_final_cli_hip_modes(args):
    for i in (1, 3, 4, 6):
        r = run_final(["--backend=hip"] + args, stdin_path=input_path(i), np_=1)
        assert r.returncode == 0, r.stderr.decode()
        assert r.stdout.decode() == expected(i), args


def test_final_cli_hip_two_ranks_offsets():
    r = run_final(["--backend=hip", "--transport=shm", "--partition=offsets", "--device=0"], stdin_path=input_path(3),
                  np_=2)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == expected(3)


@pytest.mark.parametrize("np_", [1, 2])
def test_final_cli_zero_copy_window(tmp_path, np_):
    # GPU ranks encode their own slice (P33 letters, narrow lengths, sparse offsets), page-lock only that
    # slice and stream it zero-copy; output == CPU. Two ranks share the one test GPU (--device=0).
    import json

    prob = make_synthetic("input6", 100_000, seed=8)
    path = tmp_path / "in6.txt"
    path.write_text(prob.to_text())
    r = run_final(["--backend=hip", "--transport=shm", f"--input={path}", "--timing", "--device=0"], stdin_bytes=b"",
                  np_=np_)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == format_results(search_cpu(prob))
    d = json.loads([l for l in r.stderr.decode().splitlines() if l.startswith("{")][-1])
    assert d["sliced"] is True and sum(d["rank_records"]) == prob.n
    b = np.concatenate([[0], np.cumsum(d["rank_records"])])
    for q in range(np_):
        n = d["rank_records"][q]
        letters = int(prob.offsets[b[q + 1]] - prob.offsets[b[q]])
        # this rank's slice only: P33 letters (33 bytes per 56) + 1/64 offsets + 3-bit lengths + R2 results
        lb = 33 * letters // 56
        assert lb <= d["rank_pinned_bytes"][q] <= lb + n * (8 / 64 + 3 / 8 + 2) + 64, d
        assert d["rank_h2d_bytes"][q] <= lb + 3 * n // 8 + 64, d


@pytest.mark.parametrize("source", ["input", "stdin"])
@pytest.mark.parametrize("np_", [1, 2])
def test_final_cli_streaming_slices(tmp_path, np_, source):
    # streaming batches (--batch-records) through the node's streaming flow: every GPU rank encodes its slice
    # of each batch into its two persistent, page-locked ring slots (P33 letters, sparse offsets, base-6
    # lengths, R2 results) and the kernel of batch b streams while batch b+1 is encoded
    import json

    import os
    import subprocess

    from conftest import ROOT

    # stdin through mpiexec: MPICH's hydra proxy aborts ("process reading stdin too slowly") when a rank
    # does not drain more than ~64 KB while MPI starts up — a small input there; one rank reads a 1.1 MB
    # pipe as a singleton (no proxy)
    small = source == "stdin" and np_ > 1
    n, batch = (4500, 1500) if small else (120_000, 50000)
    prob = make_synthetic("input6", n, seed=9)
    path = tmp_path / "in6.txt"
    path.write_text(prob.to_text())
    args = ["--backend=hip", "--transport=shm", "--timing", "--device=0", f"--batch-records={batch}"]
    if source == "input":
        r = run_final(args + [f"--input={path}"], stdin_bytes=b"", np_=np_)
    elif np_ > 1:
        r = run_final(args, stdin_path=str(path), np_=np_)
    else:
        r = subprocess.run([os.path.join(ROOT, "final")] + args, input=path.read_bytes(), capture_output=True,
                           timeout=120, env=dict(os.environ, OMP_NUM_THREADS="4"))
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == format_results(search_cpu(prob))
    d = json.loads([l for l in r.stderr.decode().splitlines() if l.startswith("{")][-1])
    assert d["batches"] == 3 and d["records"] == prob.n and sum(d["rank_records"]) == prob.n
    assert 0 < d["max_rank_kernel_ms"] and d["rank0_batch_kernel_ms"]["batches"] == 3, d
    # pinned once, O(batch): two slots of (P33 letters + sparse offsets + base-6 lengths + R2 results) of
    # the largest batch share, with the rings' 25 % growth slack — not per batch, not the whole input
    share = batch / np_ + 64
    per_slot = (33 * 12 * share // 56 + 8 * (share / 64 + 2) + share / 3 + 8 + 2 * share + 64 * 4) * 1.25
    assert sum(d["rank_pinned_bytes"]) <= np_ * 2 * per_slot, d


def test_final_cli_stdin_batches_larger_than_read_buffer():
    # One rank streaming a pipe: each batch (~14 MB of text) is larger than the stream buffer's first load
    # (>= 4 MiB), so the root's count-ahead while the GPU runtime starts has to load more text while batch 0
    # is cut but not yet encoded. The batch's text must survive that load (it was dropped before
    # the encode, and a load could move or free it under the encoder).
    import json
    import os
    import subprocess

    from conftest import ROOT

    prob = make_synthetic("input6", 4_000_000, seed=31)
    text = prob.to_text().encode()
    assert len(text) > 3 * 8 * 2**20
    args = ["--backend=hip", "--transport=shm", "--timing", "--device=0", "--batch-records=1500000"]
    r = subprocess.run([os.path.join(ROOT, "final")] + args, input=text, capture_output=True, timeout=120,
                       env=dict(os.environ, OMP_NUM_THREADS="8"))
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    assert r.stdout.decode() == format_results(search_cpu(prob))
    d = json.loads([l for l in r.stderr.decode().splitlines() if l.startswith("{")][-1])
    assert d["batches"] == 3 and d["records"] == prob.n, d


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("shape,n", [("input6", 200_003)])  # input1's bounds do not fit R2 (auto_format: R4)
def test_r2_results_and_nibble_lengths(pinned, packed, shape, n):
    # 2-byte results + 4-bit lengths: the narrowest wire formats of the streaming path
    from mpi_openmp_cuda_amd import _lib
    from mpi_openmp_cuda_amd.models.problem import pack5, pack_lengths4
    from mpi_openmp_cuda_amd.utils.synthetic import SHAPES

    sh = SHAPES[shape]
    prob = make_synthetic(shape, n, seed=n)
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    assert eng.auto_format(sh.l2_max, sh.l2_min) == "r2"
    codes = pack5(prob.codes) if packed else prob.codes
    lengths = pack_lengths4(np.diff(prob.offsets), sh.l2_min)
    out = np.zeros(prob.n, dtype=_lib.R2_DTYPE)
    if pinned:
        eng.pin(codes, prob.offsets, out, lengths)
    eng.solve(codes, prob.offsets, out=out, lengths=lengths, lengths_bits=4, lengths_base=sh.l2_min, fmt="r2",
              l2_range=(sh.l2_min, sh.l2_max), packed5=packed)
    st = eng.stats()
    assert st["r2"] == eng.r2_params(sh.l2_min, sh.l2_max)
    assert np.array_equal(as_triples(out, r2=st["r2"]), as_triples(search_cpu(prob))), st
    if pinned and shape == "input6":
        assert st["direct"] == (0 if packed else 1)  # 5-bit letters: the staged pipeline
    eng.close()


@pytest.mark.parametrize("seed", range(12))
def test_long_records_random_sweep(engine, seed):
    # random long-record problems (tile16 or its DPP fallback by weight range), tie-heavy alphabets,
    # lengths around the 64-step flush and the 128-offset sub-tiles, both semantics, vs the CPU engine
    rng = np.random.default_rng(1000 + seed)
    L1 = int(rng.integers(70, 3000))
    alphabet = int(rng.choice([2, 3, 5, 26]))
    w = [int(x) for x in rng.integers(0, 70, 4)]
    s1 = _letters(rng, L1, alphabet)
    lens = list(rng.integers(1, L1 + 2, 24)) + [63, 64, 65, 128, 129, L1 - 127, L1 - 128, L1 - 129]
    recs = [_letters(rng, max(int(n), 1), alphabet) for n in lens]
    prob = Problem.from_strings(w, s1, recs)
    for sem in (Semantics.REFERENCE, Semantics.SPEC):
        check(engine, prob, sem)


def test_pinned_neighbours_staged_copies():
    # offsets and results carved from one buffer and pinned separately: the results' first page belongs
    # to the offsets' registration, the rest to a second one. Async copies must not span the two
    # (the runtime rejects that with hipErrorInvalidValue): they are split per registration.
    from mpi_openmp_cuda_amd import _lib

    prob = make_synthetic("input4", 2000, seed=5)
    n = prob.n
    buf = np.zeros(64 << 10, np.uint8)
    offs = buf[: 8 * (n + 1)].view(np.int64)
    offs[:] = prob.offsets
    ob = 8 * (n + 1)
    out = buf[ob: ob + 12 * n].view(_lib.FORMAT_DTYPES[_lib.FORMAT_NAMES.index("r12")])
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    eng.pin(prob.codes)
    eng.pin(offs)
    eng.pin(out)
    eng.solve(prob.codes, offs, out=out)
    assert eng.stats()["direct"] == 0
    assert np.array_equal(as_triples(out), as_triples(search_cpu(prob)))
    eng.close()


# every (letters, lengths) combination a pinned batch can come in: 5-bit letters take the staged pipeline
# (input6), 3-bit lengths need a span of at most 8 values and base-6 at most 6 (input6: 6..11)
@pytest.mark.parametrize("shape,n,packed,len_bits", [
    ("input6", 100_003, False, 0), ("input6", 100_003, False, 8), ("input6", 100_003, True, 4),
    ("input6", 100_003, True, 8), ("input6", 100_003, True, 3), ("input6", 100_003, False, 3),
    ("input6", 100_003, True, 6), ("input6", 100_003, False, 6),
    ("input1", 20_001, False, 0), ("input1", 20_001, False, 8)])
def test_host_stream_lengths(packed, len_bits, shape, n):
    # pinned host batches streamed zero-copy by the kernel with every narrow length form — same answers
    from mpi_openmp_cuda_amd import _lib
    from mpi_openmp_cuda_amd.models.problem import pack5, pack_lengths3, pack_lengths4, pack_lengths6
    from mpi_openmp_cuda_amd.utils.synthetic import SHAPES

    sh = SHAPES[shape]
    prob = make_synthetic(shape, n, seed=n + len_bits)
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    codes = pack5(prob.codes) if packed else prob.codes
    kw = {}
    lengths = None
    if len_bits == 8:
        lengths = np.diff(prob.offsets).astype(np.uint8)
        kw = dict(lengths=lengths)
    elif len_bits == 4:
        lengths = pack_lengths4(np.diff(prob.offsets), sh.l2_min)
        kw = dict(lengths=lengths, lengths_bits=4, lengths_base=sh.l2_min)
    elif len_bits == 3:
        assert sh.l2_max - sh.l2_min <= 7
        lengths = pack_lengths3(np.diff(prob.offsets), sh.l2_min)
        kw = dict(lengths=lengths, lengths_bits=3, lengths_base=sh.l2_min)
    elif len_bits == 6:
        assert sh.l2_max - sh.l2_min <= 5
        lengths = pack_lengths6(np.diff(prob.offsets), sh.l2_min)
        kw = dict(lengths=lengths, lengths_bits=6, lengths_base=sh.l2_min)
    out = np.zeros(prob.n, dtype=_lib.FORMAT_DTYPES[_lib.FORMAT_NAMES.index("r8")])
    eng.pin(codes, prob.offsets, out, *([lengths] if lengths is not None else []))
    eng.solve(codes, prob.offsets, out=out, fmt="r8", packed5=packed, **kw)
    st = eng.stats()
    assert st["direct"] == (0 if packed else 1), st  # 5-bit letters: the staged pipeline
    assert np.array_equal(as_triples(out), as_triples(search_cpu(prob))), st
    eng.close()


@pytest.mark.parametrize("L1,lo,hi,kernel", [(90, 3, 11, "tile16"), (40, 33, 38, "swipe")])
def test_r2_tiles_and_short_kernels(engine, L1, lo, hi, kernel):
    # R2 through the tile kernel's finalize and the swipe kernel's RK form from HBM (staged path). Every
    # problem whose results fit R2 and whose records need <= 64 lanes now runs on swipe, not the lane/offset
    # kernel (its R2 store is the shared store_result)
    rng = np.random.default_rng(5)
    s1 = "".join(chr(65 + x) for x in rng.integers(0, 26, L1))
    recs = ["".join(chr(65 + x) for x in rng.integers(0, 26, rng.integers(lo, hi + 1))) for _ in range(501)]
    prob = Problem.from_strings([2, 1, 1, 1], s1, recs)
    engine.set_problem(prob.weights, prob.seq1)
    L2 = np.diff(prob.offsets)
    rng2 = (int(L2.min()), int(L2.max()))
    assert engine.auto_format(rng2[1], rng2[0]) == "r2"
    got = engine.solve(prob.codes, prob.offsets, fmt="r2", l2_range=rng2)
    assert engine.stats()["kernels"] == [kernel]
    assert np.array_equal(as_triples(got, r2=engine.stats()["r2"]), as_triples(search_cpu(prob)))


def test_pinned_registry_neighbours():
    # arrays sharing pages: every page is locked exactly once, coverage is exact, release is clean
    from mpi_openmp_cuda_amd import _lib

    L = _lib.lib()
    bufs = [np.zeros(3000 + 1000 * i, np.uint8) for i in range(6)]  # small heap arrays: shared pages
    e1, e2 = HipSearchEngine(device=0), HipSearchEngine(device=0)
    e1.pin(bufs[0], bufs[2], bufs[4])
    for i, b in enumerate(bufs):
        if i % 2 == 0:
            assert L.moc_pinned_covers(_lib.ptr(b), b.nbytes) == 1
    e2.pin(*bufs)  # overlaps e1's pages: only the missing pages get registered
    assert all(L.moc_pinned_covers(_lib.ptr(b), b.nbytes) == 1 for b in bufs)
    e2.close()
    assert all(L.moc_pinned_covers(_lib.ptr(bufs[i]), bufs[i].nbytes) == 1 for i in (0, 2, 4))
    e1.close()
    assert not any(L.moc_pinned_covers(_lib.ptr(b), b.nbytes) for b in bufs)


def test_graph_replay_sees_new_data():
    # repeated direct solves over the same pinned buffers replay a captured hipGraph; the replay must do
    # the full work on the buffers' current contents (self-resetting work counter, no stale results)
    prob = make_synthetic("input6", 100_003, seed=31)
    other = make_synthetic("input6", 100_003, seed=32)
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    codes = prob.codes.copy()
    offsets = prob.offsets.copy()
    out = np.zeros(prob.n, dtype=np.dtype([("score", "<i4"), ("n", "<i4"), ("k", "<i4")]))
    eng.pin(codes, offsets, out)
    for _ in range(3):
        eng.solve(codes, offsets, out=out)
        assert eng.stats()["direct"] == 1
    assert np.array_equal(as_triples(out), as_triples(search_cpu(prob)))
    # same buffers and lengths, new letters
    m = min(codes.shape[0], other.codes.shape[0])
    codes[:m] = other.codes[:m]
    out[:] = 0
    eng.solve(codes, offsets, out=out)
    newp = Problem(prob.weights, prob.seq1, codes, offsets)
    assert np.array_equal(as_triples(out), as_triples(search_cpu(newp)))
    eng.close()


def test_final_binary_built_from_these_sources():
    # the ./final (and its GPU plugin) under test were built from the checked-out sources, not shipped stale
    from test_cli import _source_hash

    r = run_final(["--help"], np_=1)
    assert r.returncode == 0
    assert f"src={_source_hash()}" in r.stdout.decode()


@pytest.mark.parametrize("chunk", [None, "2640"])
@pytest.mark.parametrize("shape,n", [("input6", 100_000), ("input1", 3000), ("input3", 40)])
def test_final_cli_rccl_device_batches(tmp_path, shape, n, chunk):
    # the rccl transport's device driver on one rank: the root encodes its slice from the text into a
    # page-locked block that uploads in pieces (2640-byte pieces: many), the packed narrow form streams
    # through the swipe kernel from device memory (R2 results), the dense form is unpacked on the device
    prob = make_synthetic(shape, n, seed=n)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    r = run_final(["--backend=hip", "--transport=rccl", f"--input={path}"], stdin_bytes=b"", np_=1,
                  env={"MOC_SEND_CHUNK": chunk} if chunk else None)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == format_results(search_cpu(prob))


@pytest.mark.parametrize("extra", [["--batch-records=30000"], ["--batch-chars=200000", "--skip-records=777"]])
def test_final_cli_rccl_streaming(tmp_path, extra):
    # the rccl transport streamed (flow_device_stream.cpp): batches cut from the text, encoded into wire blocks,
    # searched from HBM, results alternating between two page-locked buffers while the previous batch prints
    prob = make_synthetic("input6", 100_000, seed=3)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    r = run_final(["--backend=hip", "--transport=rccl", f"--input={path}"] + extra, stdin_bytes=b"", np_=1)
    assert r.returncode == 0, r.stderr.decode()
    want = format_results(search_cpu(prob))
    if "--skip-records=777" in extra:
        want = "".join(want.splitlines(keepends=True)[777:])
    assert r.stdout.decode() == want


def test_final_cli_rccl_event_pool_bounded(tmp_path):
    # the rccl device comm's completion events are pooled: over a streamed job of >= 50 batches (2 uploads
    # + marks per piece, MOC_SEND_CHUNK: many pieces per batch) the events alive stay at the pipeline's
    # depth instead of growing per piece (reference: a cudaMalloc leaked per record, cudaFunctions.cu:206)
    prob = make_synthetic("input6", 60_000, seed=11)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    r = run_final(["--backend=hip", "--transport=rccl", f"--input={path}", "--batch-records=1000", "--timing"],
                  stdin_bytes=b"", np_=1, env={"MOC_SEND_CHUNK": "2640"})
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == format_results(search_cpu(prob))
    d = json.loads([l for l in r.stderr.decode().splitlines() if l.startswith("{")][-1])
    assert d["batches"] >= 50
    assert 0 < d["comm_events_live"] <= 16, d["comm_events_live"]


def test_final_cli_rccl_comm_timeout_fires(tmp_path):
    # the RCCL comm's poll path driven to its deadline at world size 1: a bounded spin kernel (2 s) holds the
    # comm lane at the start of the gather; the rank's download waits on it with a 0.3 s deadline, aborts the
    # communicator and exits non-zero naming the wait and the phase
    r = run_final(["--backend=hip", "--transport=rccl", "--comm-timeout=0.3", "--inject-fault=stall-device:gather"],
                  stdin_path=input_path(3), np_=1, env={"MOC_STALL_S": "2"}, timeout=60)
    err = r.stderr.decode()
    assert r.returncode != 0, err
    assert "injected device comm lane stall" in err
    line = [l for l in err.splitlines() if "fatal: comm timeout" in l]
    assert line and "comm lane" in line[0] and "phase 'gather'" in line[0], err[-2000:]
    # and a deadline that the same stall fits inside lets the job finish with the golden output
    r = run_final(["--backend=hip", "--transport=rccl", "--comm-timeout=20", "--inject-fault=stall-device:gather"],
                  stdin_path=input_path(3), np_=1, env={"MOC_STALL_S": "0.5"}, timeout=60)
    assert r.returncode == 0 and r.stdout.decode() == expected(3), r.stderr.decode()[-2000:]


def _long_problem(L1, lengths, seed):
    rng = np.random.default_rng(seed)
    seq1 = rng.integers(1, 27, size=L1, dtype=np.uint8)
    lengths = np.asarray(lengths, dtype=np.int64)
    codes = rng.integers(1, 27, size=int(lengths.sum()), dtype=np.uint8)
    offsets = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    return Problem([4, 3, 2, 10], seq1, codes, offsets)


@pytest.mark.parametrize("L1,lengths", [(20_000, [10_000, 9_000, 150]), (150_000, [40_000])])
def test_long_context_engine(engine, L1, lengths):
    # beyond the reference's 3000/2000-letter buffers (myProto.h:3-4): L1 * L2 up to 6e9 (> 2^32: pass-1 keys,
    # k resolved on the winning diagonal), records of 40 000 letters; both semantics vs the CPU engine
    prob = _long_problem(L1, lengths, seed=L1)
    for sem in (Semantics.REFERENCE, Semantics.SPEC):
        engine.set_problem(prob.weights, prob.seq1, sem)
        got = as_triples(engine.solve(prob.codes, prob.offsets))
        assert np.array_equal(got, as_triples(search_cpu(prob, sem))), sem


def test_long_context_cli_offsets_three_ranks(tmp_path):
    # one huge pair (L1 = 150 000, L2 = 40 000: 4.4e9 cells, L1 * L2 > 2^32) split by offsets over 3 ranks
    # sharing the GPU; pass-1 keys MAX-combined, k resolved on the root
    prob = _long_problem(150_000, [40_000, 39_000], seed=3)
    path = tmp_path / "long.txt"
    path.write_text(prob.to_text())
    r = run_final(["--backend=hip", "--partition=offsets", "--transport=shm", "--device=0", f"--input={path}"],
                  stdin_bytes=b"", np_=3, timeout=300)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == format_results(search_cpu(prob))


@pytest.mark.parametrize("L1,shape,n", [(20_000, "input3", 40), (5_000, "input4", 300), (3_100, "input3", 12),
                                        (60_000, "input1", 100)])
def test_tile16_windowed(engine, L1, shape, n):
    # Seq1 longer than one LDS image (3052 letters): the windowed tile16 sweep (each workgroup stages a
    # window of the profile; window-major plan) == the CPU engine, both semantics; and context-parallel
    # shares of it MAX-combine to the same answers
    from mpi_openmp_cuda_amd import decode_keys

    base = make_synthetic(shape, n, seed=L1 + n)
    rng = np.random.default_rng(L1)
    prob = Problem(base.weights, rng.integers(1, 27, size=L1, dtype=np.uint8), base.codes, base.offsets)
    for sem in (Semantics.REFERENCE, Semantics.SPEC):
        engine.set_problem(prob.weights, prob.seq1, sem)
        ref = as_triples(search_cpu(prob, sem))
        assert np.array_equal(as_triples(engine.solve(prob.codes, prob.offsets)), ref), sem
        assert "tile16" in engine.stats()["kernels"], engine.stats()
        keys = np.zeros(prob.n, np.uint64)
        for part in range(3):
            keys = np.maximum(keys, engine.search_keys(prob.codes, prob.offsets, part, 3))
        assert np.array_equal(as_triples(decode_keys(keys, prob)), ref), sem


@pytest.mark.parametrize("L1", [1600, 2001, 2976])
def test_tile16_window_wide(engine, L1):
    # short records on a Seq1 whose widened image does not fit one CU (L1 ~ 1500..3050): the sweep stages a
    # widened window (tile16_search_kernel<U, true, true>; L1 = 2001 takes the unaligned staging loop), ==
    # the CPU engine, both semantics, and against the whole byte-pair image (MOC_TILE16_WINWIDE=0 path)
    base = make_synthetic("input4", 300, seed=L1)
    rng = np.random.default_rng(L1)
    prob = Problem(base.weights, rng.integers(1, 27, size=L1, dtype=np.uint8), base.codes, base.offsets)
    for sem in (Semantics.REFERENCE, Semantics.SPEC):
        engine.set_problem(prob.weights, prob.seq1, sem)
        assert np.array_equal(as_triples(engine.solve(prob.codes, prob.offsets)), as_triples(search_cpu(prob, sem)))
        assert engine.stats()["kernels"] == ["tile16"], engine.stats()


@pytest.mark.parametrize("L1,lo,hi", [(2000, 400, 900), (2001, 600, 1200), (3000, 1, 2000), (1600, 1100, 1500)])
def test_tile16_slide(engine, L1, lo, hi):
    # long records on a Seq1 whose widened image does not fit one CU: sliding widened windows
    # (tile16_slide_kernel; L1 2001 takes the unaligned staging loop; groups of 16 with empty members when
    # the count is not a multiple of 16), == the CPU engine, both semantics
    from mpi_openmp_cuda_amd.utils.synthetic import Shape, make_shape

    prob = make_shape(Shape((10, 2, 3, 4), L1, lo, hi), 301, seed=L1 + lo)
    for sem in (Semantics.REFERENCE, Semantics.SPEC):
        engine.set_problem(prob.weights, prob.seq1, sem)
        got = engine.solve(prob.codes, prob.offsets)
        st = engine.stats()
        assert st["kernels"] == ["tile16"] and "tile16_slide" in st["forms"], st
        assert np.array_equal(as_triples(got), as_triples(search_cpu(prob, sem)))


@pytest.mark.parametrize("n,w,slide", [(5, (10, 2, 3, 4), False), (5, (200, 10, 10, 10), True),
                                        (40, (10, 2, 3, 4), True), (36, (10, 2, 3, 4), False)])
def test_tile16_slide_group_fill(engine, n, w, slide):
    # sliding windows need groups of 16 similar records: with fewer than 0.8 of the groups' waves filled the
    # byte-pair image keeps every wave on a tile of its own; an int16 profile (whose other plan is the LUT
    # tile kernel) slides from a quarter filled
    from mpi_openmp_cuda_amd.utils.synthetic import Shape, make_shape

    prob = make_shape(Shape(w, 2400, 1100, 1400), n, seed=n)
    engine.set_problem(prob.weights, prob.seq1)
    got = engine.solve(prob.codes, prob.offsets)
    st = engine.stats()
    assert st["kernels"] == ["tile16"] and ("tile16_slide" in st["forms"]) == slide, st
    assert np.array_equal(as_triples(got), as_triples(search_cpu(prob)))


def test_tile16_slide_sub_tiles_and_previous_plan(monkeypatch):
    # the U = 2 and U = 8 slide kernels (MOC_TILE_U; default 4), one workgroup per CU (MOC_TILE16_SLIDE_WG=1;
    # default two, the 64-VGPR instances) and the plan without sliding windows
    # (MOC_TILE16_SLIDE=0: the whole byte-pair image) give the same results as the CPU engine
    from mpi_openmp_cuda_amd.utils.synthetic import Shape, make_shape

    prob = make_shape(Shape((10, 2, 3, 4), 2500, 700, 1700), 100, seed=5)
    ref = as_triples(search_cpu(prob))
    for env, form in (({"MOC_TILE_U": "2"}, True), ({"MOC_TILE16_SLIDE_WG": "1"}, True),
                      ({"MOC_TILE16_SLIDE_WG": "1", "MOC_TILE_U": "8"}, True), ({"MOC_TILE16_SLIDE": "0"}, False)):
        with monkeypatch.context() as m:
            for k, v in env.items():
                m.setenv(k, v)
            eng = HipSearchEngine(device=0)
            eng.set_problem(prob.weights, prob.seq1)
            assert np.array_equal(as_triples(eng.solve(prob.codes, prob.offsets)), ref), env
            assert ("tile16_slide" in eng.stats()["forms"]) == form, (env, eng.stats())


@pytest.mark.parametrize("w,forms", [((63, 0, 0, 64), ["tile16", "tile16_key32"]),
                                     ((64, 0, 0, 64), ["tile16", "tile16_key32", "tile16_i16"]),
                                     ((256, 0, 0, 256), ["tiles_key32"])])
def test_extreme_values_tile16_window_wide(engine, w, forms):
    # the profile bounds on the widened-window image: the byte pairs at |Dt| = 127, the int16 profile one past
    # it, the LUT tile kernel past |Dt| = 511
    from mpi_openmp_cuda_amd.utils.synthetic import make_extreme

    prob = make_extreme(2400, 40, 90, w, copies=3, seed=7)
    engine.set_problem(prob.weights, prob.seq1)
    got = engine.solve(prob.codes, prob.offsets, fmt="auto")
    st = engine.stats()
    assert st["forms"] == forms, st
    assert np.array_equal(as_triples(got, r2=st["r2"]), _extreme_ref(prob, Semantics.REFERENCE)), st


# ---- the Python distributed driver on GPU ranks (parallel/search.py -> parallel/wire.py WireSlice): the same
# wire-format step bench.py times, pinned here to the goldens and to the CPU engine
@pytest.mark.parametrize("transport", ["shm"])
def test_python_driver_hip_goldens(transport):
    from mpi_openmp_cuda_amd.parallel.dist import DistContext
    from mpi_openmp_cuda_amd.parallel.search import DistributedSearch

    ds = DistributedSearch(DistContext(), backend="hip", transport=transport)
    for i in range(1, 7):
        prob = Problem.read(input_path(i))
        assert format_results(ds.run(prob)) == expected(i), f"input{i}"
    big = make_synthetic("input6", 300000, seed=21)  # R2 results, 3-bit lengths, zero-copy swipe stream
    assert np.array_equal(as_triples(ds.run(big)), as_triples(search_cpu(big)))


def test_python_driver_hip_two_ranks(tmp_path):
    import os
    import subprocess
    import sys

    from conftest import ROOT

    prob = make_synthetic("input6", 200000, seed=22)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    want = format_results(search_cpu(prob))
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="4")
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    for transport in ("shm",):
        r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                            "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "mpi_openmp_cuda_amd",
                            "--backend=hip", "--dist-backend=gloo", f"--transport={transport}", f"--input={path}"],
                           capture_output=True, timeout=110, env=env, cwd="/tmp")
        assert r.returncode == 0, r.stderr.decode()[-3000:]
        assert r.stdout.decode() == want, transport


@pytest.mark.parametrize("mode", ["bulk", "stream"])
def test_final_narrow_guess_fails_stdin_two_ranks(mode):
    # a GPU rank whose narrow-form guess (L1 <= 200, mean length <= 64) is refused by the
    # engine (here L1 - min_l2 + 1 > 64 lanes) re-encodes its slice as 5-bit letters + CSR offsets. That
    # must happen while the node-shared stdin text is still there — before the helpers release their
    # shares of it — and every row must match the CPU engine.
    rng = np.random.default_rng(31)
    seq1 = rng.integers(1, 27, size=150, dtype=np.uint8)
    lengths = rng.integers(10, 31, size=2400)  # ~50 KB: under what hydra forwards to a rank still starting
    offsets = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64)
    codes = rng.integers(1, 27, size=int(offsets[-1]), dtype=np.uint8)
    from mpi_openmp_cuda_amd.models.scoring import Weights

    prob = Problem(Weights.of((10, 2, 3, 4)), seq1, codes, offsets)
    extra = ["--batch-records=1000"] if mode == "stream" else []
    r = run_final(["--backend=hip", "--device=0"] + extra, stdin_bytes=prob.to_text().encode(), np_=2)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == format_results(search_cpu(prob))


@pytest.mark.parametrize("tail", ["4", "8", "0"])
def test_swipe_tail_tiles_every_record(tail):
    # the persistent grid's tail tiles (the last `slots` tiles cut to 1/4 or 1/8) only
    # start beyond 2 * slots tiles — millions of records at full size. A small grid (MOC_SWIPE_SLOTS) and
    # 256-record tiles reach them with 60 K records; every result, head to tail, against the CPU engine.
    import os
    import subprocess
    import sys

    from conftest import ROOT

    code = r"""
import numpy as np, sys
sys.path.insert(0, %r)
from mpi_openmp_cuda_amd import HipSearchEngine, search_cpu
from mpi_openmp_cuda_amd._lib import Pinned
from mpi_openmp_cuda_amd.ops.align import as_triples
from mpi_openmp_cuda_amd.parallel.wire import WireSlice
from mpi_openmp_cuda_amd.utils.synthetic import make_synthetic
prob = make_synthetic("input6", 60_003, seed=23)
eng = HipSearchEngine(device=0)
eng.set_problem(prob.weights, prob.seq1)
ws = WireSlice.from_csr(prob.codes, prob.offsets)
ws.alloc_results(eng)
with Pinned(*ws.arrays()):
    for _ in range(2):
        ws.results[:] = 0x7777
        ws.solve(eng)
        assert eng.stats()["direct"] == 1 and eng.stats()["kernels"] == ["swipe"], eng.stats()
        assert np.array_equal(ws.triples(eng), as_triples(search_cpu(prob)))
print("ok")
""" % ROOT
    # tail tiles need tiles of a multiple of 64 * divisor records
    env = dict(os.environ, MOC_SWIPE_TILE="512" if tail == "8" else "256", MOC_SWIPE_SLOTS="16", MOC_SWIPE_TAIL=tail)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, timeout=300, env=env)
    assert r.returncode == 0 and b"ok" in r.stdout, r.stderr.decode()[-3000:]


@pytest.mark.parametrize("preload", ["none", "swipe33", "tile16,short", "all"])
def test_preload_sets(monkeypatch, preload):
    # MOC_PRELOAD picks which code objects load at engine start; the rest load at their first launch — the
    # results must not depend on it (input6: swipe P33 / bytes, input3: tile16)
    monkeypatch.setenv("MOC_PRELOAD", preload)
    eng = HipSearchEngine(device=0)
    for shape, n in (("input6", 5_000), ("input3", 40)):
        check(eng, make_synthetic(shape, n, seed=41))
    eng.close()


def test_preload_set_unknown_name(monkeypatch):
    from mpi_openmp_cuda_amd._lib import NativeError

    monkeypatch.setenv("MOC_PRELOAD", "swipe33,nosuchfile")
    with pytest.raises(NativeError, match="MOC_PRELOAD"):
        HipSearchEngine(device=0)


def test_problem_image_staging_grows():
    # the problem image uploads through a page-locked staging buffer that starts at 256 KiB: a long Seq1
    # (20000 letters, a ~1 MB tile16 image in device memory) grows it, and alternating problems re-upload
    eng = HipSearchEngine(device=0)
    small = make_synthetic("input6", 3_000, seed=43)
    rng = np.random.default_rng(44)
    seq1 = rng.integers(1, 27, 20_000).astype(np.uint8)
    lens = rng.integers(50, 400, 64)
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    big = Problem((5, 2, 3, 4), seq1, rng.integers(1, 27, int(offsets[-1])).astype(np.uint8), offsets)
    for prob in (small, big, small, big):
        check(eng, prob)
    eng.close()


@pytest.mark.parametrize("n,shift", [(150, 0), (150, 1), (150, 7), (2500, 3)])
def test_staged_pinned_kernel_copies(n, shift):
    # pinned batches through the staged pipeline (long records: tile16) move their small pieces on the copy
    # kernel (dev::launch_copy) instead of the runtime's SDMA path: letters at a 1..15-byte misalignment take
    # its byte loop, aligned offsets / results its 16-byte loop; 2500 input4 records (~100 KB of letters at
    # shift 3: byte loop) and 150 (~6 KB); the results must match the CPU engine either way
    from mpi_openmp_cuda_amd import _lib

    prob = make_synthetic("input4", n, seed=50 + shift)
    raw = np.zeros(prob.codes.nbytes + 64, np.uint8)
    base = (-raw.ctypes.data) % 16 + shift
    codes = raw[base: base + prob.codes.nbytes]
    codes[:] = prob.codes
    assert codes.ctypes.data % 16 == shift % 16
    offs = prob.offsets.copy()
    out = np.zeros(n, _lib.FORMAT_DTYPES[_lib.FORMAT_NAMES.index("r12")])
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    eng.pin(raw, offs, out)
    eng.solve(codes, offs, out=out)
    assert eng.stats()["direct"] == 0
    assert np.array_equal(as_triples(out), as_triples(search_cpu(prob)))
    eng.close()


@pytest.mark.parametrize("np_", [1, 2])
def test_final_cli_gpu_isolate(np_):
    # --gpu-isolate=1 narrows each rank's runtime to the GPU it takes by node-local rank (ROCR_VISIBLE_DEVICES
    # to its index, HIP_VISIBLE_DEVICES to 0): the box's one GPU stays that GPU, the output stays the golden
    r = run_final(["--backend=hip", "--gpu-isolate=1", "--log-level=info"], stdin_path=input_path(6), np_=np_)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == expected(6)
    assert r.stderr.decode().count("runtime isolated to gpu") == np_, r.stderr.decode()
    # with --device the rank names its GPU itself: no isolation
    r = run_final(["--backend=hip", "--gpu-isolate=1", "--device=0", "--log-level=info"], stdin_path=input_path(6),
                  np_=np_)
    assert r.returncode == 0 and r.stdout.decode() == expected(6)
    assert "runtime isolated" not in r.stderr.decode()


@pytest.mark.parametrize("shape,n", [("input6", 200_003), ("input1", 30_001), ("input6", 777), ("mid", 20_001)])
def test_wire_device_resident(engine, shape, n):
    # a batch in the wire formats held in device memory (the rccl transport's form): P33 letters, narrow
    # lengths, the narrowest results; the swipe kernel reads it in place
    from mpi_openmp_cuda_amd.parallel.wire import WireSlice

    prob = make_synthetic(shape, n, seed=61)
    engine.set_problem(prob.weights, prob.seq1)
    wire = WireSlice.from_csr(prob.codes, prob.offsets)
    res = wire.alloc_results(engine)
    dev = torch.device("cuda:0")
    letters = torch.from_numpy(wire.codes).to(dev)
    offsets = torch.from_numpy(wire.offsets).to(dev)
    lengths = torch.from_numpy(wire.lengths).to(dev) if wire.lengths is not None else None
    out = torch.zeros(res.nbytes, dtype=torch.uint8, device=dev)
    engine.solve_wire_device(letters, offsets, lengths, wire.n, out, wire.fmt, (wire.l2_min, wire.l2_max),
                             lengths_bits=wire.len_bits or 8, lengths_base=wire.len_base)
    st = engine.stats()
    assert st["direct"] == 1 and st["kernels"] == ["swipe"] and st["h2d_bytes"] == 0
    res.view(np.uint8)[:] = out.cpu().numpy()
    got = wire.triples(engine)
    ref = as_triples(search_cpu(prob))
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("L1,lo,hi", [(24, 5, 16), (30, 3, 16), (50, 17, 32), (60, 33, 48), (70, 44, 48), (80, 49, 64),
                                      (14, 4, 16), (40, 20, 44)])  # the last two: records longer than Seq1 too
@pytest.mark.parametrize("sem", [Semantics.REFERENCE, Semantics.SPEC])
def test_wire_device_resident_record_words(engine, L1, lo, hi, sem):
    # P33 batches at every record-word width of the lane-direct kernel (4 — with 20 offsets per lane in
    # 128-record tiles, with 28 in 64-record ones — 8, 12 and 16 words): the decode slices are sized by the
    # batch's longest record, the base-6 lengths (every octet position and digit) decoded in f32; random
    # lengths and weights, both semantics, checked against the CPU engine
    from mpi_openmp_cuda_amd.parallel.wire import WireSlice
    from mpi_openmp_cuda_amd.utils.synthetic import Shape, make_shape

    prob = make_shape(Shape((7, 3, 2, 5), L1, lo, hi), 40_001, seed=L1 + hi)
    engine.set_problem(prob.weights, prob.seq1, sem)
    wire = WireSlice.from_csr(prob.codes, prob.offsets)
    res = wire.alloc_results(engine)
    dev = torch.device("cuda:0")
    letters = torch.from_numpy(wire.codes).to(dev)
    offsets = torch.from_numpy(wire.offsets).to(dev)
    lengths = torch.from_numpy(wire.lengths).to(dev) if wire.lengths is not None else None
    out = torch.zeros(res.nbytes, dtype=torch.uint8, device=dev)
    engine.solve_wire_device(letters, offsets, lengths, wire.n, out, wire.fmt, (wire.l2_min, wire.l2_max),
                             lengths_bits=wire.len_bits or 8, lengths_base=wire.len_base)
    st = engine.stats()
    assert st["direct"] == 1 and st["kernels"] == ["swipe"], st
    res.view(np.uint8)[:] = out.cpu().numpy()
    assert np.array_equal(wire.triples(engine), as_triples(search_cpu(prob, sem)))


# ---- narrow-integer fast paths at their exactness bounds (csrc/include/moc/kernel_bounds.hpp) --------------
# Every case runs the adversarial input (utils/synthetic.make_extreme: Seq1 = "AZAZ...", pieces of it at even
# and odd offsets, so |D| reaches 2 W L2 exactly) at the bound — the fast form must be chosen and exact — and
# one step past it — the rule must fall back to the next form, also exact. The CPU tier pins the same
# bounds (tests/test_extremes.py) and replays each form's arithmetic (csrc/tests/test_core.cpp).
EXTREMES = [
    # name, L1, l2 range, weights, kernels, forms
    ("swipe_kbits_at", 40, 6, 16, (31, 0, 0, 31), ["swipe"], ["swipe_kbits"]),
    ("swipe_kbits_past", 40, 6, 16, (32, 0, 0, 32), ["swipe"], ["swipe_rk"]),
    ("swipe_kbits_w8_at", 60, 20, 32, (7, 0, 0, 7), ["swipe"], ["swipe_kbits"]),
    ("swipe_kbits_w8_past", 60, 20, 32, (8, 0, 0, 8), ["swipe"], ["swipe_rk"]),
    ("swipe_rk_at", 70, 40, 64, (255, 0, 0, 255), ["swipe"], ["swipe_rk"]),
    ("swipe_rk_past", 70, 40, 64, (256, 0, 0, 256), ["short"], ["short_key32"]),
    ("swipe_rk_w4_at", 40, 6, 16, (1023, 0, 0, 1023), ["swipe"], ["swipe_rk"]),
    ("swipe_rk_w4_past", 40, 6, 16, (1024, 0, 0, 1024), ["short"], ["short_key32"]),
    ("swipe_rk_w24_at", 130, 67, 96, (170, 0, 0, 170), ["swipe"], ["swipe_rk"]),
    ("swipe_rk_w24_past", 130, 67, 96, (171, 0, 0, 171), ["short"], ["short_key32"]),
    ("swipe_rk_w32_at", 190, 127, 128, (127, 0, 0, 127), ["swipe"], ["swipe_rk"]),
    ("swipe_rk_w32_past", 190, 127, 128, (128, 0, 0, 128), ["short"], ["short_key32"]),
    # records over 128 letters with <= 64 offsets: the lane-per-offset short kernel
    ("short_pk_at", 150, 130, 150, (109, 0, 0, 109), ["short"], ["short_pk"]),
    ("short_pk_past", 150, 130, 150, (110, 0, 0, 110), ["short"], ["short_key32"]),
    ("short_key32_at", 200, 150, 190, (22075, 0, 0, 22075), ["short"], ["short_key32"]),
    ("short_key32_past", 200, 150, 190, (22076, 0, 0, 22076), ["short"], ["short_key64"]),
    ("tile16_at", 600, 150, 400, (63, 0, 0, 64), ["tile16"], ["tile16", "tile16_key32"]),
    # tile16's 32-bit selection keys: 127 * 2064 < 2^18 (L1 2600: 13 index bits), 127 * 2065 is not
    # (records past a widened window on a Seq1 past the widened image: sliding windows)
    ("tile16_key32_at", 2600, 2000, 2064, (127, 0, 0, 0), ["tile16"], ["tile16", "tile16_key32", "tile16_slide"]),
    ("tile16_key32_past", 2600, 2000, 2065, (127, 0, 0, 0), ["tile16"], ["tile16", "tile16_slide"]),
    # the int16 profile (widened images only): |Dt| = W1 + W4 = 511 at the bound, 512 past it
    ("tile16_i16_at", 600, 150, 400, (255, 0, 0, 256), ["tile16"], ["tile16", "tile16_key32", "tile16_i16"]),
    ("tile16_i16_past", 600, 150, 400, (256, 0, 0, 256), ["tiles"], ["tiles_key32"]),
    ("tile16_i16_window", 2400, 40, 90, (255, 0, 0, 256), ["tile16"], ["tile16", "tile16_key32", "tile16_i16"]),
    # no widened image or window holds it (L1 2400, records to 1200 letters): sliding widened windows
    ("tile16_i16_long", 2400, 1000, 1200, (255, 0, 0, 256), ["tile16"], ["tile16", "tile16_i16", "tile16_slide"]),
    ("tile16_slide_at", 2400, 900, 1400, (63, 0, 0, 64), ["tile16"], ["tile16", "tile16_key32", "tile16_slide"]),
    ("tile16_slide_i16", 2400, 900, 1400, (64, 0, 0, 64), ["tile16"],
     ["tile16", "tile16_key32", "tile16_i16", "tile16_slide"]),
    ("tile16_past", 600, 150, 400, (64, 0, 0, 64), ["tile16"], ["tile16", "tile16_key32", "tile16_i16"]),
    ("tiles_key32_at", 600, 150, 400, (5242, 0, 0, 5242), ["tiles"], ["tiles_key32"]),
    ("tiles_key32_past", 600, 150, 400, (5243, 0, 0, 5243), ["tiles"], ["tiles_key64"]),
]


def _extreme_ref(prob, sem):
    # brute force where it is cheap; the CPU engine (itself pinned to brute force on these inputs by
    # tests/test_extremes.py) for the 600-letter Seq1
    return as_triples(brute_force_native(prob, sem) if prob.L1 <= 130 else search_cpu(prob, sem))


@pytest.mark.parametrize("case", EXTREMES, ids=[c[0] for c in EXTREMES])
@pytest.mark.parametrize("sem", [Semantics.REFERENCE, Semantics.SPEC])
def test_extreme_values_staged(engine, case, sem):
    _, L1, lo, hi, w, kernels, forms = case
    from mpi_openmp_cuda_amd.utils.synthetic import make_extreme

    prob = make_extreme(L1, lo, hi, w, copies=40 if L1 <= 130 else 3, seed=L1)
    engine.set_problem(prob.weights, prob.seq1, sem)
    got = engine.solve(prob.codes, prob.offsets, fmt="auto")
    st = engine.stats()
    assert (st["kernels"], st["forms"]) == (kernels, forms), st
    assert np.array_equal(as_triples(got, r2=st["r2"]), _extreme_ref(prob, sem)), st


@pytest.mark.parametrize("case", [c for c in EXTREMES if c[5] == ["swipe"]], ids=[c[0] for c in EXTREMES if c[5] == ["swipe"]])
def test_extreme_values_wire_p33(case):
    # the headline's data path: P33 letters + narrow lengths + the narrowest results, zero-copy from pinned memory
    _, L1, lo, hi, w, kernels, forms = case
    from mpi_openmp_cuda_amd._lib import Pinned
    from mpi_openmp_cuda_amd.parallel.wire import WireSlice
    from mpi_openmp_cuda_amd.utils.synthetic import make_extreme

    prob = make_extreme(L1, lo, hi, w, copies=60, seed=L1 + 1)
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    ws = WireSlice.from_csr(prob.codes, prob.offsets, letter_format="p33")
    ws.alloc_results(eng)
    with Pinned(*ws.arrays()):
        ws.solve(eng)
    st = eng.stats()
    assert (st["kernels"], st["forms"], st["direct"]) == (kernels, forms, 1), st
    assert np.array_equal(ws.triples(eng), _extreme_ref(prob, Semantics.REFERENCE)), st
    eng.close()


@pytest.mark.parametrize("case", [c for c in EXTREMES if c[5] == ["swipe"]], ids=[c[0] for c in EXTREMES if c[5] == ["swipe"]])
def test_extreme_values_device_resident(engine, case):
    # device-resident byte letters with dense offsets only (lengths taken from the offsets in the kernel:
    # swipe_impl.hpp kDeferLens) and a record count that leaves a partial last tile
    _, L1, lo, hi, w, kernels, forms = case
    from mpi_openmp_cuda_amd.utils.synthetic import make_extreme

    prob = make_extreme(L1, lo, hi, w, copies=57, seed=L1 + 2)
    dev = torch.device("cuda:0")
    engine.set_problem(prob.weights, prob.seq1)
    fmt = engine.auto_format(hi, lo)
    from mpi_openmp_cuda_amd import _lib

    item = _lib.FORMAT_DTYPES[_lib.FORMAT_NAMES.index(fmt)].itemsize
    out_t = torch.zeros(prob.n * item, dtype=torch.uint8, device=dev)
    engine.solve_wire_device(torch.from_numpy(prob.codes).to(dev), torch.from_numpy(prob.offsets).to(dev), None,
                             prob.n, out_t, fmt, (int(np.diff(prob.offsets).min()), int(np.diff(prob.offsets).max())),
                             packed33=False)
    st = engine.stats()
    assert (st["kernels"], st["forms"]) == (kernels, forms), st
    res = out_t.cpu().numpy().view(_lib.FORMAT_DTYPES[_lib.FORMAT_NAMES.index(fmt)])[:prob.n]
    r2 = engine.r2_params(lo, hi) if fmt == "r2" else None
    assert np.array_equal(as_triples(res, r2=r2), _extreme_ref(prob, Semantics.REFERENCE)), st


@pytest.mark.parametrize("case", [c for c in EXTREMES if c[5] == ["swipe"]], ids=[c[0] for c in EXTREMES if c[5] == ["swipe"]])
def test_extreme_values_wire_p33_device(engine, case):
    # the rccl transport's batches: P33 letters, 64-record sparse offsets and narrow lengths in device memory,
    # read in place by the wave-autonomous kernel (each wave decodes its tile's fields into an LDS slice)
    _, L1, lo, hi, w, kernels, forms = case
    from mpi_openmp_cuda_amd.parallel.wire import WireSlice
    from mpi_openmp_cuda_amd.utils.synthetic import make_extreme

    prob = make_extreme(L1, lo, hi, w, copies=61, seed=L1 + 3)
    engine.set_problem(prob.weights, prob.seq1)
    wire = WireSlice.from_csr(prob.codes, prob.offsets, letter_format="p33")
    res = wire.alloc_results(engine)
    dev = torch.device("cuda:0")
    lengths = torch.from_numpy(wire.lengths).to(dev) if wire.lengths is not None else None
    out = torch.zeros(res.nbytes, dtype=torch.uint8, device=dev)
    engine.solve_wire_device(torch.from_numpy(wire.codes).to(dev), torch.from_numpy(wire.offsets).to(dev), lengths,
                             wire.n, out, wire.fmt, (wire.l2_min, wire.l2_max), lengths_bits=wire.len_bits or 8,
                             lengths_base=wire.len_base)
    st = engine.stats()
    assert (st["kernels"], st["forms"], st["h2d_bytes"]) == (kernels, forms, 0), st
    res.view(np.uint8)[:] = out.cpu().numpy()
    assert np.array_equal(wire.triples(engine), _extreme_ref(prob, Semantics.REFERENCE)), st


def test_extreme_values_wire_range_checked(engine):
    # a device batch whose stated length range is narrower than its records is refused (the kernel would
    # size its LDS from the range)
    from mpi_openmp_cuda_amd.utils.synthetic import make_extreme

    prob = make_extreme(40, 6, 16, (4, 3, 2, 10), copies=5)
    dev = torch.device("cuda:0")
    engine.set_problem(prob.weights, prob.seq1)
    out_t = torch.zeros(prob.n * 12, dtype=torch.uint8, device=dev)
    with pytest.raises(ValueError):
        engine.solve_wire_device(torch.from_numpy(prob.codes).to(dev), torch.from_numpy(prob.offsets).to(dev), None,
                                 prob.n, out_t, "r12", (6, 12), packed33=False)


@pytest.mark.parametrize("w,fmt", [(3, "r2"), (4, "r4"), (2047, "r4"), (2048, "r8")])
def test_extreme_values_result_formats(engine, w, fmt):
    # result codes at their bounds: R2 holds (2 w 16 + 1) * 35 * 16 codes <= 65535 up to w = 3; R4's int16
    # score holds w * 16 < 32767 up to w = 2047
    from mpi_openmp_cuda_amd.utils.synthetic import make_extreme

    prob = make_extreme(40, 6, 16, (w, 0, 0, w), copies=20, seed=w)
    engine.set_problem(prob.weights, prob.seq1)
    assert engine.auto_format(16, 6) == fmt
    got = engine.solve(prob.codes, prob.offsets, fmt="auto")
    st = engine.stats()
    assert st["format"] == fmt, st
    ref = as_triples(brute_force_native(prob))
    assert np.array_equal(as_triples(got, r2=st["r2"]), ref), st
    assert ref[:, 0].max() == 16 * w  # the top of the score range is exercised (a whole even piece of Seq1)
    if fmt == "r8" and w == 2048:
        from mpi_openmp_cuda_amd._lib import NativeError

        with pytest.raises(NativeError):
            engine.solve(prob.codes, prob.offsets, fmt="r4")
