"""Pinning diagnostics (no kernels launched): replays the pin -> close -> re-allocate -> pin sequence of
tests/test_gpu.py::test_r2_results_and_nibble_lengths and prints how the HIP runtime maps each array
(type, host pointer, device pointer, hipHostGetDevicePointer) in both rounds."""
import sys

import numpy as np

sys.path.insert(0, ".")
from mpi_openmp_cuda_amd import HipSearchEngine, _lib, make_synthetic  # noqa: E402
from mpi_openmp_cuda_amd.models.problem import pack5, pack_lengths4  # noqa: E402


def info(name, a):
    v = np.zeros(6, np.uint64)
    _lib.check(_lib.lib().moc_pointer_info(_lib.ptr(a), a.nbytes, _lib.ptr(v)))
    host = a.ctypes.data
    print(f"  {name:8s} host={host:#x} bytes={a.nbytes} type={int(v[0])} hostPtr={int(v[1]):#x} "
          f"devPtr={int(v[2]):#x} getDevPtr={int(v[3]):#x} same={int(v[3]) == host} "
          f"range=[{int(v[4]):#x}, +{int(v[5])}) covers={int(v[4]) <= host and host + a.nbytes <= int(v[4]) + int(v[5])}",
          flush=True)


# a heap array shares pages with its neighbours: register two neighbours, then ask about the middle one
a = np.zeros(30000, np.uint8)
b = np.zeros(30000, np.uint8)
c = np.zeros(30000, np.uint8)
e = HipSearchEngine(device=0)
e.pin(a, c)
print("neighbours pinned, middle not:", flush=True)
for n_, x in (("a", a), ("b", b), ("c", c)):
    info(n_, x)
e.close()

for rnd, packed in enumerate([False, True]):
    prob = make_synthetic("input6", 200_003, seed=200_003)
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    codes = pack5(prob.codes) if packed else prob.codes
    lengths = pack_lengths4(np.diff(prob.offsets), 6)
    out = np.zeros(prob.n, dtype=_lib.R2_DTYPE)
    print(f"round {rnd} packed={packed} before pin", flush=True)
    for n, a in (("codes", codes), ("offsets", prob.offsets), ("out", out), ("lengths", lengths)):
        info(n, a)
    eng.pin(codes, prob.offsets, out, lengths)
    print(f"round {rnd} after pin", flush=True)
    for n, a in (("codes", codes), ("offsets", prob.offsets), ("out", out), ("lengths", lengths)):
        info(n, a)
    eng.close()
    print(f"round {rnd} after close", flush=True)
    for n, a in (("codes", codes), ("offsets", prob.offsets), ("out", out), ("lengths", lengths)):
        info(n, a)
    del prob, codes, lengths, out, eng
