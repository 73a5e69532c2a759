"""Search ops: CPU (OpenMP) and GPU (gfx950 HIP kernels) engines behind one API.

Reference: send_divided_Seq2_To_Cuda + calc_result (cudaFunctions.cu:178-242, 63-176) — one kernel
launch and device sync per record. Here a whole batch is one pipeline call (HipSearchEngine.solve) or,
for device-resident data, one launch sequence on the caller's stream (HipSearchEngine.solve_device /
align_search_device, which take torch tensors on ``cuda:N``).
"""
from __future__ import annotations

import ctypes
import json
from typing import Optional

import numpy as np

from .. import _lib
from ..models.problem import Problem
from ..models.scoring import Semantics, Weights

RESULT_DTYPE = _lib.RESULT_DTYPE


def empty_results(n: int) -> np.ndarray:
    return np.zeros(n, dtype=RESULT_DTYPE)


def as_triples(results: np.ndarray, r2=None) -> np.ndarray:
    """Results in any wire format (R12/R8/R4 structured, R2 codes with their (smin, kw, j) parameters, or
    (n,3) ints) -> (n, 3) int32 [score, n, k]."""
    r = np.asarray(results)
    if r.dtype == _lib.R2_DTYPE:
        if r2 is None:
            raise ValueError("R2 results need their (smin, kw, j) parameters")
        smin, kw, j = (int(v) for v in r2)
        c = r.astype(np.int64)
        idx = c % j
        out = np.stack([c // j + smin, idx // kw, idx % kw], axis=1).astype(np.int32)
        out[c == 0xFFFF] = (np.iinfo(np.int32).min, 0, 0)
        return out
    if r.dtype == RESULT_DTYPE:
        return r.view(np.int32).reshape(-1, 3)
    if r.dtype.names:
        score = r["score"].astype(np.int32)
        if r.dtype == _lib.R4_DTYPE:
            score[r["score"] == np.iinfo(np.int16).min] = np.iinfo(np.int32).min
        return np.stack([score, r["n"].astype(np.int32), r["k"].astype(np.int32)], axis=1)
    return np.asarray(r, dtype=np.int32).reshape(-1, 3)


# ---------------------------------------------------------------------------------------------- CPU
def search_cpu(problem: Problem, semantics=Semantics.REFERENCE, threads: int = 0) -> np.ndarray:
    """O(L1*L2) OpenMP engine (csrc/src/cpu_engine.cpp). Returns structured results (score, n, k)."""
    out = empty_results(problem.n)
    _lib.check(_lib.lib().moc_cpu_solve(
        _lib.weights_arg(problem.weights.as_list()), _lib.ptr(problem.seq1), problem.L1,
        _lib.ptr(problem.codes), _lib.ptr(problem.offsets), problem.n, int(Semantics.parse(semantics)),
        int(threads), _lib.ptr(out)))
    return out


def search_keys_cpu(problem: Problem, part: int, parts: int, semantics=Semantics.REFERENCE,
                    threads: int = 0) -> np.ndarray:
    """Context-parallel partial search: part ``part`` of ``parts`` of every record's offset
    range -> packed uint64 pass-1 keys (0 = no candidate in this part). ``np.maximum`` over all parts, then
    :func:`decode_keys`, equals :func:`search_cpu`."""
    keys = np.zeros(problem.n, np.uint64)
    _lib.check(_lib.lib().moc_cpu_solve_keys(
        _lib.weights_arg(problem.weights.as_list()), _lib.ptr(problem.seq1), problem.L1,
        _lib.ptr(problem.codes), _lib.ptr(problem.offsets), problem.n, int(Semantics.parse(semantics)),
        int(part), int(parts), int(threads), _lib.ptr(keys)))
    return keys


def decode_keys(keys: np.ndarray, problem: Problem) -> np.ndarray:
    """MAX-combined pass-1 keys ((score^2^31)<<32 | ~(2n + mutated)) -> structured (score, n, k) results; the k
    of a mutated winner is the smallest one on its diagonal with that score, so the problem's records are
    needed (no n*L2 + k index: any L1 * L2)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    out = empty_results(keys.shape[0])
    _lib.check(_lib.lib().moc_resolve_keys(
        _lib.weights_arg(problem.weights.as_list()), _lib.ptr(problem.seq1), problem.L1, _lib.ptr(problem.codes),
        _lib.ptr(problem.offsets), keys.shape[0], _lib.ptr(keys), _lib.ptr(out)))
    return out


def keys_to_ordered_int64(keys: np.ndarray) -> np.ndarray:
    """uint64 keys -> int64 with the same order (flip the top bit), for signed MAX all-reduces."""
    return (np.ascontiguousarray(keys, dtype=np.uint64) ^ np.uint64(1 << 63)).view(np.int64)


def ordered_int64_to_keys(v: np.ndarray) -> np.ndarray:
    return np.ascontiguousarray(v, dtype=np.int64).view(np.uint64) ^ np.uint64(1 << 63)


def brute_force_native(problem: Problem, semantics=Semantics.REFERENCE) -> np.ndarray:
    """Literal O(L1*L2^2) replay of the reference loops, in C++ (test oracle)."""
    out = empty_results(problem.n)
    _lib.check(_lib.lib().moc_brute_force(
        _lib.weights_arg(problem.weights.as_list()), _lib.ptr(problem.seq1), problem.L1,
        _lib.ptr(problem.codes), _lib.ptr(problem.offsets), problem.n, int(Semantics.parse(semantics)),
        _lib.ptr(out)))
    return out


def native_score_table(weights) -> np.ndarray:
    lut = np.zeros((32, 32), np.int32)
    _lib.check(_lib.lib().moc_score_table(_lib.weights_arg(Weights.of(weights).as_list()), _lib.ptr(lut), None))
    return lut


# ---------------------------------------------------------------------------------------------- GPU
def device_count() -> int:
    return int(_lib.lib().moc_device_count())


def device_info(device: int = 0) -> dict:
    buf = ctypes.create_string_buffer(1024)
    _lib.check(_lib.lib().moc_device_info_json(device, buf, 1024))
    return json.loads(buf.value.decode())


def _format_id(fmt) -> int:
    if isinstance(fmt, (int, np.integer)):
        return int(fmt)
    return _lib.FORMAT_NAMES.index(str(fmt).lower())


class HipSearchEngine:
    """Per-rank gfx950 engine: problem upload, planning, and host<->device data movement.

    ``solve`` picks the zero-copy streaming path automatically when every host buffer is pinned
    (``pin`` / ``_lib.Pinned`` / hipHostMalloc) and all records fit the short kernel; otherwise it runs
    the staged double-buffered chunk pipeline (csrc/src/hip_engine.cpp)."""

    def __init__(self, device: Optional[int] = None, chunk_records: int = 0, chunk_bytes: int = 0,
                 allow_direct: bool = True):
        L = _lib.lib()
        if L.moc_device_count() <= 0:
            raise _lib.NativeError("HipSearchEngine needs a visible HIP device (none found)")
        self._h = L.moc_engine_create(-1 if device is None else int(device), int(chunk_records), int(chunk_bytes),
                                      1 if allow_direct else 0)
        if not self._h:
            raise _lib.NativeError(L.moc_last_error().decode())
        self.problem_L1 = None
        self._problem_key = None  # (weights, seq1, semantics) bytes of the problem in the engine
        self._stats_buf = (ctypes.c_double * 14)()

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().moc_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_problem(self, weights, seq1: np.ndarray, semantics=Semantics.REFERENCE):
        seq1 = np.ascontiguousarray(seq1, dtype=np.uint8)
        if isinstance(weights, np.ndarray) and semantics is Semantics.REFERENCE:
            # a job loop re-sending the same problem (the engine keeps an unchanged image anyway): no
            # conversion or native call at all
            key = (weights.tobytes(), seq1.tobytes())
            if key == self._problem_key:
                return
        else:
            key = None
        self._problem_key = None  # not current until the native call succeeds
        _lib.check(_lib.lib().moc_engine_set_problem(
            self._h, _lib.weights_arg(Weights.of(weights).as_list()), _lib.ptr(seq1), seq1.shape[0],
            int(Semantics.parse(semantics))))
        self.problem_L1 = int(seq1.shape[0])
        self._problem_key = key

    def pin(self, *arrays):
        """Page-locks host arrays for the engine's lifetime (enables the zero-copy path)."""
        for a in arrays:
            if a is not None and a.nbytes:
                _lib.check(_lib.lib().moc_engine_pin(self._h, ctypes.c_void_p(a.ctypes.data), a.nbytes))

    def auto_format(self, max_l2: int, min_l2: int = 0) -> str:
        """Smallest result format for records of lengths [min_l2, max_l2] (min_l2 = 0: unknown -> no R2)."""
        return _lib.FORMAT_NAMES[_lib.lib().moc_engine_auto_format(self._h, int(max_l2), int(min_l2))]

    def r2_params(self, min_l2: int, max_l2: int) -> tuple:
        """(smin, kw, j) of the R2 format for records of lengths [min_l2, max_l2]."""
        v = np.zeros(3, np.int32)
        _lib.check(_lib.lib().moc_engine_r2_params(self._h, int(min_l2), int(max_l2), _lib.ptr(v)))
        return tuple(int(x) for x in v)

    def solve(self, codes: np.ndarray, offsets: np.ndarray, out: Optional[np.ndarray] = None,
              lengths: Optional[np.ndarray] = None, fmt="r12", l2_range=None, packed5: bool = False,
              lengths_bits: int = 8, lengths_base: int = 0,
              packed33: bool = False) -> np.ndarray:
        """Host CSR -> host results. ``codes[offsets[i]:offsets[i+1]]`` is record i (``offsets`` may be a
        slice of a larger absolute offset array). ``fmt``: r12 | r8 | r4 | r2 | auto (smallest that fits);
        ``lengths``: optional narrow record lengths, uint8 (``lengths_bits`` 8) or two per byte
        (``lengths_bits`` 4, low nibble first, length = ``lengths_base`` + nibble; see pack_lengths4) or
        3-bit fields (``lengths_bits`` 3, see pack_lengths3);
        ``l2_range``: optional known (min, max) length (R2 results are encoded for it: decode with
        ``r2_params(*l2_range)`` or ``stats()["r2"]``); ``packed5``: ``codes`` is a 5-bit packed stream
        (models.problem.pack5) instead of bytes; ``packed33``: 33-bit fields of 7 letters
        (models.problem.pack33)."""
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        n = offsets.shape[0] - 1
        if l2_range is None and (fmt == "auto"):
            L2 = np.diff(offsets) if n else np.zeros(1, np.int64)
            l2_range = (int(L2.min()) if n else 0, int(L2.max()) if n else 0)
        if fmt == "auto":
            fmt = self.auto_format(l2_range[1], l2_range[0])
        fid = _format_id(fmt)
        if out is None:
            out = np.empty(n, dtype=_lib.FORMAT_DTYPES[fid])
        assert out.dtype.itemsize == _lib.FORMAT_DTYPES[fid].itemsize and out.size >= n
        if lengths is not None:
            need = (n if lengths_bits == 8 else (n + 1) // 2 if lengths_bits == 4
                    else 8 * ((n + 23) // 24) if lengths_bits == 6 else (3 * n + 7) // 8 + 1)
            assert lengths.dtype == np.uint8 and lengths.shape[0] >= need
        lo, hi = l2_range if l2_range is not None else (-1, -1)
        _lib.check(_lib.lib().moc_engine_solve_ex(self._h, _lib.ptr(codes), _lib.ptr(offsets), _lib.ptr(lengths),
                                                  int(lengths_bits), int(lengths_base), n, _lib.ptr(out), fid, int(lo),
                                                  int(hi), 3 if packed33 else 1 if packed5 else 0))
        return out

    def solve_device(self, codes_t, offsets_t, h_offsets: np.ndarray, out_t, stream=None):
        """Device-resident batch (torch tensors on this engine's device). ``codes_t`` is the base so that
        record i starts at codes_t[offsets[i]]; ``out_t`` is int32 [n, 3]. Queued on ``stream``
        (torch.cuda.Stream, default: the current stream); returns immediately."""
        import torch

        h_offsets = np.ascontiguousarray(h_offsets, dtype=np.int64)
        n = h_offsets.shape[0] - 1
        assert codes_t.dtype == torch.uint8 and offsets_t.dtype == torch.int64 and out_t.dtype == torch.int32
        assert offsets_t.numel() == n + 1 and out_t.shape == (n, 3)
        if stream is None:
            stream = torch.cuda.current_stream(codes_t.device)
        _lib.check(_lib.lib().moc_engine_solve_device(
            self._h, ctypes.c_void_p(codes_t.data_ptr()), ctypes.c_void_p(offsets_t.data_ptr()), _lib.ptr(h_offsets),
            n, ctypes.c_void_p(out_t.data_ptr()), ctypes.c_void_p(stream.cuda_stream)))
        return out_t

    def solve_wire_device(self, letters_t, offsets_t, lengths_t, n: int, out_t, fmt: str, l2_range,
                          lengths_bits: int = 8, lengths_base: int = 0, packed33: bool = True):
        """Device-resident batch in the wire formats (torch tensors on this engine's GPU, as the rccl transport
        holds them): ``letters_t`` P33 fields (``packed33``) or bytes, ``offsets_t`` int64 [n + 1] letter
        offsets, ``lengths_t`` narrow lengths (as ``solve``'s) or None, results into ``out_t`` (a uint8
        tensor of n * itemsize bytes of ``fmt``, decoded on the host as ``solve``'s). Synchronous;
        ``stats()["kernel_ms"]`` is the kernel's time."""
        import torch

        fid = _format_id(fmt)
        assert letters_t.dtype == torch.uint8 and offsets_t.dtype == torch.int64 and offsets_t.numel() == n + 1
        assert out_t.dtype == torch.uint8 and out_t.numel() >= n * _lib.FORMAT_DTYPES[fid].itemsize
        if n > 0:
            # the kernel sizes its LDS and per-lane record words from l2_range and cannot re-scan device
            # lengths: a range narrower than the batch would give wrong results, so it is checked here
            d = offsets_t[1:] - offsets_t[:-1]
            lo, hi = int(d.min()), int(d.max())
            if lo < int(l2_range[0]) or hi > int(l2_range[1]):
                raise ValueError(f"l2_range {tuple(l2_range)} does not hold the batch's lengths [{lo}, {hi}]")
        lp = ctypes.c_void_p(lengths_t.data_ptr()) if lengths_t is not None else None
        _lib.check(_lib.lib().moc_engine_solve_wire_device(
            self._h, ctypes.c_void_p(letters_t.data_ptr()), ctypes.c_void_p(offsets_t.data_ptr()), lp,
            int(lengths_bits), int(lengths_base), int(n), ctypes.c_void_p(out_t.data_ptr()), fid, int(l2_range[0]),
            int(l2_range[1]), 3 if packed33 else 0))
        return out_t

    def device_kernel_ms(self) -> float:
        """Device time (ms) of the last solve_device's kernels, from events around its launches (after the
        host's per-call planning); waits for them."""
        ms = ctypes.c_double(0.0)
        _lib.check(_lib.lib().moc_engine_device_kernel_ms(self._h, ctypes.addressof(ms)))
        return float(ms.value)

    def search_keys(self, codes: np.ndarray, offsets: np.ndarray, part: int, parts: int) -> np.ndarray:
        """Context-parallel partial search on the GPU: this engine's share (part of parts) of the batch's
        offset tiles -> packed uint64 keys per record (see :func:`search_keys_cpu`)."""
        codes = np.ascontiguousarray(codes, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        n = offsets.shape[0] - 1
        keys = np.zeros(n, np.uint64)
        _lib.check(_lib.lib().moc_engine_search_keys(self._h, _lib.ptr(codes), _lib.ptr(offsets), n, int(part),
                                                     int(parts), _lib.ptr(keys)))
        return keys

    def search_keys_device(self, codes_t, offsets_t, h_offsets: np.ndarray, part: int, parts: int, keys_t,
                           stream=None):
        """Device-resident form: keys_t is an int64 tensor [n] receiving the uint64 key bits."""
        import torch

        h_offsets = np.ascontiguousarray(h_offsets, dtype=np.int64)
        n = h_offsets.shape[0] - 1
        assert keys_t.dtype == torch.int64 and keys_t.numel() == n
        if stream is None:
            stream = torch.cuda.current_stream(codes_t.device)
        _lib.check(_lib.lib().moc_engine_search_keys_device(
            self._h, ctypes.c_void_p(codes_t.data_ptr()), ctypes.c_void_p(offsets_t.data_ptr()), _lib.ptr(h_offsets),
            n, int(part), int(parts), ctypes.c_void_p(keys_t.data_ptr()), ctypes.c_void_p(stream.cuda_stream)))
        return keys_t

    def finalize_keys_device(self, codes_t, offsets_t, h_offsets: np.ndarray, keys_t, out_t, stream=None):
        """MAX-combined device keys -> int32 [n, 3] results (score, n, k); k is resolved on each record's
        winning diagonal, so the batch (codes_t, offsets_t from 0, host copy h_offsets) is needed."""
        import torch

        n = keys_t.numel()
        assert out_t.dtype == torch.int32 and out_t.shape == (n, 3)
        h_offsets = np.ascontiguousarray(h_offsets, dtype=np.int64)
        if stream is None:
            stream = torch.cuda.current_stream(keys_t.device)
        _lib.check(_lib.lib().moc_engine_finalize_keys_device(
            self._h, ctypes.c_void_p(codes_t.data_ptr()), ctypes.c_void_p(offsets_t.data_ptr()), _lib.ptr(h_offsets),
            n, ctypes.c_void_p(keys_t.data_ptr()), ctypes.c_void_p(out_t.data_ptr()), 0,
            ctypes.c_void_p(stream.cuda_stream)))
        return out_t

    def kernel_times(self) -> tuple:
        """(kernel_ms, total_ms) of the last solve: the two fields a timed loop reads, without stats()'s dict."""
        v = self._stats_buf
        _lib.check(_lib.lib().moc_engine_stats(self._h, v))
        return v[0], v[1]

    def solve_prepared(self, args: tuple):
        """Re-runs a solve whose native arguments were marshalled once (WireSlice.solve): same call."""
        _lib.check(_lib.lib().moc_engine_solve_ex(self._h, *args))

    def stats(self) -> dict:
        v = (ctypes.c_double * 14)()
        _lib.check(_lib.lib().moc_engine_stats(self._h, v))
        keys = ["kernel_ms", "total_ms", "h2d_bytes", "d2h_bytes", "chunks", "cells", "records", "direct", "format",
                "kernels"]
        d = dict(zip(keys, list(v)[:10]))
        d["r2"] = tuple(int(x) for x in list(v)[10:13])
        d["format"] = _lib.FORMAT_NAMES[int(d["format"])]
        d["kernels"] = [k for b, k in ((1, "swipe"), (2, "short"), (4, "tiles"), (8, "tile16")) if int(d["kernels"]) & b]
        d["forms"] = [k for b, k in FORM_NAMES if int(v[13]) & b]
        return d


# Arithmetic forms of the kernels (csrc/include/moc/kernel_bounds.hpp FormBits), as stats()["forms"] names them.
FORM_NAMES = ((1, "swipe_kbits"), (2, "swipe_rk"), (4, "short_pk"), (8, "short_key32"), (16, "short_key64"),
              (32, "tile16"), (64, "tiles_key32"), (128, "tiles_key64"), (256, "mfma"), (512, "tile16_key32"),
              (1024, "tile16_i16"), (2048, "tile16_slide"))


def kernel_bounds(weights, L1: int, min_l2: int, max_l2: int) -> dict:
    """The host's exactness rules for a batch (csrc/include/moc/kernel_bounds.hpp), no GPU needed:
    ``swipe`` = "swipe_kbits" | "swipe_rk" | None (the swipe kernel's integer bounds refuse it), ``short_pk``
    = the short kernel's packed int16 form is exact, ``key_shift`` = k bits of the int32 hot keys (0: int64
    keys), ``profile16`` = the tile16 int8 profile holds the table, ``tile16_key_bits`` = index bits of tile16's
    32-bit selection keys (0: 64-bit keys), ``profile16_i16`` = the int16 tile16 profile holds the table."""
    out = np.zeros(6, np.int32)
    _lib.check(_lib.lib().moc_kernel_bounds(_lib.weights_arg(Weights.of(weights).as_list()), int(L1), int(min_l2),
                                            int(max_l2), _lib.ptr(out)))
    swipe = {1: "swipe_kbits", 2: "swipe_rk"}.get(int(out[0]))
    return {"swipe": swipe, "short_pk": bool(out[1]), "key_shift": int(out[2]), "profile16": bool(out[3]),
            "tile16_key_bits": int(out[4]), "profile16_i16": bool(out[5])}


def search_hip(problem: Problem, semantics=Semantics.REFERENCE, device: Optional[int] = None,
               engine: Optional[HipSearchEngine] = None) -> np.ndarray:
    eng = engine or HipSearchEngine(device)
    eng.set_problem(problem.weights, problem.seq1, semantics)
    return eng.solve(problem.codes, problem.offsets)


def align_search(problem: Problem, backend: str = "auto", semantics=Semantics.REFERENCE, **kw) -> np.ndarray:
    """Best (score, n, k) for every record. backend: auto | hip | cpu."""
    if backend == "auto":
        backend = "hip" if device_count() > 0 else "cpu"
    if backend == "hip":
        return search_hip(problem, semantics, **kw)
    if backend == "cpu":
        return search_cpu(problem, semantics, **kw)
    raise ValueError(f"unknown backend {backend!r}")


def align_search_device(engine: HipSearchEngine, codes_t, offsets_t, h_offsets, stream=None):
    """torch-facing op: returns an int32 [n, 3] tensor (score, n, k) on the codes' device."""
    import torch

    n = int(len(h_offsets) - 1)
    out = torch.empty((n, 3), dtype=torch.int32, device=codes_t.device)
    engine.solve_device(codes_t, offsets_t, h_offsets, out, stream)
    return out
