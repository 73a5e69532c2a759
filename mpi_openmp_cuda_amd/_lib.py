"""ctypes binding of the native core ``lib/libmoc.so`` (C ABI: csrc/include/moc/capi.h).

The shared object is built in-tree by ``make lib`` (or ``__graft_entry__.build()``); it holds the
parser, score table, OpenMP CPU engine, partitioner and the HIP engine + gfx950 kernels. There is no
silent Python fallback for the GPU path: if the library is missing, importing an op raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int, c_int32, c_int64, c_size_t, c_uint8, c_void_p

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MOC_LIB_PATH selects an alternative build of the same library (A/B kernel experiments, the
# `make debug-kernels` build); the default is the in-tree build. A library whose kernels were built with
# extra defines (moc_build_info) loads only with MOC_ALLOW_VARIANT_LIB=1: a variant can compute different
# results and must never stand in for the product silently.
LIB_PATH = os.environ.get("MOC_LIB_PATH") or os.path.join(_HERE, "lib", "libmoc.so")

RESULT_DTYPE = np.dtype([("score", "<i4"), ("n", "<i4"), ("k", "<i4")])
# Packed result wire formats (moc/device.hpp ResultFormat): index = format id.
R8_DTYPE = np.dtype([("score", "<i4"), ("n", "<u2"), ("k", "<u2")])
R4_DTYPE = np.dtype([("score", "<i2"), ("n", "u1"), ("k", "u1")])
# R2: one uint16 per record, (score - smin) * j + n * kw + k, 0xFFFF = no candidate; decoding needs the
# (smin, kw, j) parameters the engine reports (HipSearchEngine.r2_params / stats()["r2"]).
R2_DTYPE = np.dtype("<u2")
FORMAT_DTYPES = [RESULT_DTYPE, R8_DTYPE, R4_DTYPE, R2_DTYPE]
FORMAT_NAMES = ["r12", "r8", "r4", "r2"]

_lib = None


class NativeError(RuntimeError):
    """An error reported by the native core (message from moc_last_error)."""


def _decl(lib):
    P = POINTER
    sig = {
        "moc_last_error": (c_char_p, []),
        "moc_abi_version": (c_int, []),
        "moc_set_log_level": (c_int, [c_char_p]),
        "moc_parse": (c_void_p, [c_char_p, c_size_t, c_int]),
        "moc_problem_free": (None, [c_void_p]),
        "moc_problem_info": (c_int, [c_void_p, P(c_int32), P(c_int64), P(c_int64), P(c_int64)]),
        "moc_problem_seq1": (c_void_p, [c_void_p]),
        "moc_problem_codes": (c_void_p, [c_void_p]),
        "moc_problem_offsets": (c_void_p, [c_void_p]),
        "moc_format_results": (c_int64, [c_void_p, c_int64, c_int64, c_void_p, c_int64]),
        "moc_score_table": (c_int, [P(c_int32), c_void_p, c_void_p]),
        "moc_kernel_bounds": (c_int, [P(c_int32), c_int64, c_int64, c_int64, c_void_p]),
        "moc_build_info": (c_char_p, []),
        "moc_packed5_bytes": (c_int64, [c_int64]),
        "moc_pack5": (c_int, [c_void_p, c_int64, c_void_p]),
        "moc_unpack5": (c_int, [c_void_p, c_int64, c_int64, c_void_p]),
        "moc_packed33_bytes": (c_int64, [c_int64]),
        "moc_pack33": (c_int, [c_void_p, c_int64, c_void_p]),
        "moc_unpack33": (c_int, [c_void_p, c_int64, c_int64, c_void_p]),
        "moc_pack_lengths": (c_int, [c_void_p, c_int64, c_int, c_int64, c_void_p]),
        "moc_cpu_solve": (c_int, [P(c_int32), c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p]),
        "moc_cpu_solve_keys": (c_int, [P(c_int32), c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int, c_int, c_int,
                                       c_int, c_void_p]),
        "moc_resolve_keys": (c_int, [P(c_int32), c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
        "moc_brute_force": (c_int, [P(c_int32), c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_int, c_void_p]),
        "moc_partition": (c_int, [c_void_p, c_int64, c_int64, c_int, c_double, c_double, c_double, c_void_p]),
        "moc_device_count": (c_int, []),
        "moc_host_register": (c_int, [c_void_p, c_size_t]),
        "moc_host_unregister": (c_int, [c_void_p]),
        "moc_host_alloc": (c_void_p, [c_size_t]),
        "moc_host_free": (c_int, [c_void_p]),
        "moc_pointer_info": (c_int, [c_void_p, c_size_t, c_void_p]),
        "moc_pinned_covers": (c_int, [c_void_p, c_size_t]),
        "moc_bind_numa": (c_int, [c_int]),
        "moc_device_numa_node": (c_int, [c_int]),
        "moc_dpp_probe": (c_int, [c_void_p]),
        "moc_mfma_i8_probe": (c_int, [c_void_p, c_void_p, c_void_p]),
        "moc_transfer_probe": (c_double, [c_int, c_size_t, c_int]),
        "moc_device_info_json": (c_int, [c_int, c_char_p, c_int64]),
        "moc_engine_create": (c_void_p, [c_int, c_int64, c_int64, c_int]),
        "moc_engine_destroy": (None, [c_void_p]),
        "moc_engine_set_problem": (c_int, [c_void_p, P(c_int32), c_void_p, c_int64, c_int]),
        "moc_engine_solve": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
        "moc_engine_solve_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int64, c_void_p, c_int,
                                        c_int64, c_int64, c_int]),
        "moc_engine_auto_format": (c_int, [c_void_p, c_int64, c_int64]),
        "moc_engine_r2_params": (c_int, [c_void_p, c_int64, c_int64, c_void_p]),
        "moc_engine_pin": (c_int, [c_void_p, c_void_p, c_size_t]),
        "moc_expand_results": (c_int, [c_void_p, c_int, c_int64, c_void_p, c_void_p]),
        "moc_engine_solve_device": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
        "moc_engine_solve_wire_device": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int64, c_void_p,
                                                 c_int, c_int64, c_int64, c_int]),
        "moc_engine_device_kernel_ms": (c_int, [c_void_p, c_void_p]),
        "moc_engine_stats": (c_int, [c_void_p, P(c_double)]),
        "moc_engine_search_keys": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p]),
        "moc_engine_search_keys_device": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int,
                                                  c_void_p, c_void_p]),
        "moc_engine_finalize_keys_device": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                                    c_int, c_void_p]),
    }
    for name, (res, args) in sig.items():
        if os.environ.get("MOC_LIB_PATH") and not hasattr(lib, name):
            continue  # an older build selected for an A/B run: only what it has
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args


def lib():
    """Returns the loaded native library, raising a clear error if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"native library not built: {LIB_PATH} is missing — run `make lib` "
                "(or `python -c 'import __graft_entry__ as g; g.build()'`) first")
        l = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _decl(l)
        info = build_info(l)
        if info.get("defs") and os.environ.get("MOC_ALLOW_VARIANT_LIB") != "1":
            raise NativeError(f"{LIB_PATH} is a variant build (kernel defines: {info['defs']}); "
                              "set MOC_ALLOW_VARIANT_LIB=1 to load it on purpose")
        _lib = l
    return _lib


def build_info(l=None) -> dict:
    """{"src": source hash, "defs": -D flags of the kernel objects} of the loaded library ({} for builds that
    predate moc_build_info)."""
    l = l or lib()
    if not hasattr(l, "moc_build_info"):
        return {}
    s = l.moc_build_info().decode()
    src, _, defs = s.partition(" defs=")
    return {"src": src[len("src="):], "defs": defs.strip()}


def check(rc):
    if rc != 0:
        raise NativeError(lib().moc_last_error().decode(errors="replace"))
    return rc


def ptr(a):
    """Raw pointer of a contiguous numpy array (or None)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return ctypes.c_void_p(a.ctypes.data)


def weights_arg(weights):
    w = (c_int32 * 4)(*[int(x) for x in weights])
    return w


class Pinned:
    """Context manager / handle that page-locks numpy arrays for direct DMA (hipHostRegister)."""

    def __init__(self, *arrays):
        self._ptrs = []
        for a in arrays:
            if a is None or a.nbytes == 0:
                continue
            check(lib().moc_host_register(ctypes.c_void_p(a.ctypes.data), a.nbytes))
            self._ptrs.append(a.ctypes.data)

    def release(self):
        for p in self._ptrs:
            lib().moc_host_unregister(ctypes.c_void_p(p))
        self._ptrs = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.release()


class HostBuffer:
    """Page-locked host allocation (hipHostMalloc) usable as numpy arrays by the streaming paths."""

    def __init__(self, nbytes: int):
        L = lib()
        p = L.moc_host_alloc(max(int(nbytes), 1))
        if not p:
            raise NativeError(L.moc_last_error().decode(errors="replace"))
        self._p = p
        self.nbytes = int(nbytes)

    def array(self, dtype, count: int, offset: int = 0):
        import numpy as np

        buf = (ctypes.c_uint8 * self.nbytes).from_address(self._p)
        return np.frombuffer(buf, dtype=dtype, count=count, offset=offset)

    def free(self):
        if self._p:
            lib().moc_host_free(self._p)
            self._p = None


def loaded_path():
    return LIB_PATH if _lib is not None else None
