"""Result formatting/writing (reference output line: main.c:204 "#%d: score: %d, n: %d, k: %d")."""
from __future__ import annotations

import sys

import numpy as np

from .. import _lib


def format_results(results: np.ndarray, first_index: int = 0) -> str:
    """Native parallel formatter (csrc/src/io.cpp). ``results`` is a RESULT_DTYPE array or (n, 3) ints."""
    from ..ops.align import as_triples

    r = np.ascontiguousarray(results)
    if r.dtype != _lib.RESULT_DTYPE:
        r = np.ascontiguousarray(as_triples(r)).view(_lib.RESULT_DTYPE).reshape(-1)
    n = r.shape[0]
    cap = 96 * n + 16
    buf = np.empty(cap, np.uint8)
    w = _lib.lib().moc_format_results(_lib.ptr(r), n, int(first_index), _lib.ptr(buf), cap)
    if w < 0:
        raise _lib.NativeError(_lib.lib().moc_last_error().decode())
    return buf[:w].tobytes().decode("ascii")


def format_results_py(results, first_index: int = 0) -> str:
    """Pure-Python formatter (oracle for the native one)."""
    out = []
    for i, (s, n, k) in enumerate(np.asarray(results, dtype=np.int64).reshape(-1, 3)):
        out.append(f"#{i + first_index}: score: {s}, n: {n}, k: {k}\n")
    return "".join(out)


def write_results(results: np.ndarray, stream=None, first_index: int = 0):
    stream = stream or sys.stdout
    stream.write(format_results(results, first_index))
    stream.flush()
