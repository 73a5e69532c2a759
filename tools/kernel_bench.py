"""Device-resident kernel throughput (no PCIe in the loop): cells/s of the search kernels per problem
shape, timed with HIP events around HipSearchEngine.solve_device on HBM-resident torch tensors.

cells = sum over records of (L1 - L2 + 1) * L2 — the O(L1*L2) candidate cells; the
reference kernel does O(L1*L2^2) work for the same answers.
"""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: E402

from mpi_openmp_cuda_amd import HipSearchEngine, make_synthetic, search_cpu  # noqa: E402
from mpi_openmp_cuda_amd.ops.align import as_triples  # noqa: E402

CASES = [("input6", 1 << 24), ("input1", 1 << 21), ("input4", 1 << 17), ("input3", 1 << 13), ("limits", 1 << 12)]
if len(sys.argv) > 1:
    CASES = [c for c in CASES if c[0] in sys.argv[1:]]


def run(shape, n, iters=5):
    prob = make_synthetic(shape, n, seed=7)
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    dev = torch.device("cuda:0")
    codes = torch.from_numpy(prob.codes).to(dev)
    offs = torch.from_numpy(prob.offsets).to(dev)
    out = torch.empty((prob.n, 3), dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    eng.solve_device(codes, offs, prob.offsets, out, s)  # warm-up (and host planning cache warm)
    torch.cuda.synchronize()
    t_host = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        eng.solve_device(codes, offs, prob.offsets, out, s)
    e1.record(s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t_host) / iters
    ms = e0.elapsed_time(e1) / iters
    nv = min(prob.n, 4000)
    ref = as_triples(search_cpu(prob.slice(0, nv)))
    ok = bool(np.array_equal(out[:nv].cpu().numpy(), ref))
    cells = prob.cells()
    return {"shape": shape, "records": prob.n, "L1": prob.L1, "letters": prob.total_chars, "cells": cells,
            "gpu_ms": round(ms, 4), "host_wall_ms": round(wall * 1e3, 4), "cells_per_s": cells / (ms / 1e3),
            "records_per_s": prob.n / (ms / 1e3), "verified": ok}


if __name__ == "__main__":
    res = [run(s, n) for s, n in CASES]
    for r in res:
        print(json.dumps(r))
