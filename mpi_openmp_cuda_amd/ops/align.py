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


def as_triples(results: np.ndarray) -> np.ndarray:
    """Structured results -> (n, 3) int32 view [score, n, k]."""
    return results.view(np.int32).reshape(-1, 3)


# ---------------------------------------------------------------------------------------------- CPU
def search_cpu(problem: Problem, semantics=Semantics.REFERENCE, threads: int = 0) -> np.ndarray:
    """O(L1*L2) OpenMP engine (csrc/src/cpu_engine.cpp). Returns structured results (score, n, k)."""
    out = empty_results(problem.n)
    _lib.check(_lib.lib().moc_cpu_solve(
        _lib.weights_arg(problem.weights.as_list()), _lib.ptr(problem.seq1), problem.L1,
        _lib.ptr(problem.codes), _lib.ptr(problem.offsets), problem.n, int(Semantics.parse(semantics)),
        int(threads), _lib.ptr(out)))
    return out


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


class HipSearchEngine:
    """Per-rank gfx950 engine: problem upload, host planning, chunked H2D/compute/D2H pipeline."""

    def __init__(self, device: Optional[int] = None, chunk_records: int = 0, chunk_bytes: int = 0,
                 pin_host: bool = True):
        L = _lib.lib()
        if L.moc_device_count() <= 0:
            raise _lib.NativeError("HipSearchEngine needs a visible HIP device (none found)")
        self._h = L.moc_engine_create(-1 if device is None else int(device), int(chunk_records), int(chunk_bytes),
                                      1 if pin_host else 0)
        if not self._h:
            raise _lib.NativeError(L.moc_last_error().decode())
        self.problem_L1 = None

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
        _lib.check(_lib.lib().moc_engine_set_problem(
            self._h, _lib.weights_arg(Weights.of(weights).as_list()), _lib.ptr(seq1), seq1.shape[0],
            int(Semantics.parse(semantics))))
        self.problem_L1 = int(seq1.shape[0])

    def solve(self, codes: np.ndarray, offsets: np.ndarray, out: Optional[np.ndarray] = None) -> np.ndarray:
        """Host CSR -> host results (pinned DMA, double-buffered chunks). ``codes[offsets[i]:offsets[i+1]]``
        is record i; ``offsets`` may be a slice of a larger absolute offset array."""
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        n = offsets.shape[0] - 1
        if out is None:
            out = empty_results(n)
        _lib.check(_lib.lib().moc_engine_solve(self._h, _lib.ptr(codes), _lib.ptr(offsets), n, _lib.ptr(out)))
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

    def stats(self) -> dict:
        v = (ctypes.c_double * 7)()
        _lib.check(_lib.lib().moc_engine_stats(self._h, v))
        keys = ["kernel_ms", "total_ms", "h2d_bytes", "d2h_bytes", "chunks", "cells", "records"]
        return dict(zip(keys, list(v)))


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
