"""GPU debug helper: DPP probe + per-record HIP vs CPU comparison on a fixture (prints mismatches)."""
import sys

import numpy as np

sys.path.insert(0, ".")
from mpi_openmp_cuda_amd import HipSearchEngine, Problem, search_cpu  # noqa: E402
from mpi_openmp_cuda_amd import _lib  # noqa: E402
from mpi_openmp_cuda_amd.ops.align import as_triples  # noqa: E402

out = np.zeros(192, np.int32)
_lib.check(_lib.lib().moc_dpp_probe(_lib.ptr(out)))
print("shl1   ", out[:64].tolist())
print("fill   ", out[64:128].tolist())
print("wavemax", out[128:192].tolist())

path = sys.argv[1] if len(sys.argv) > 1 else "tests/data/input3.txt"
p = Problem.read(path)
e = HipSearchEngine(0)
e.set_problem(p.weights, p.seq1)
g = as_triples(e.solve(p.codes, p.offsets))
r = as_triples(search_cpu(p))
for i in range(p.n):
    flag = "" if (g[i] == r[i]).all() else "  <-- MISMATCH"
    print(i, p.lengths[i], g[i].tolist(), r[i].tolist(), flag)
# single-record batches
for i in range(min(p.n, 4)):
    s = p.slice(i, i + 1)
    gg = as_triples(e.solve(s.codes, s.offsets))
    print("single", i, gg[0].tolist(), r[i].tolist())
