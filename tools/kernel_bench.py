"""Device-resident kernel throughput (no PCIe in the loop): cells/s of the search kernels per problem
shape, timed with HIP events around HipSearchEngine.solve_device on HBM-resident torch tensors.

cells = sum over records of (L1 - L2 + 1) * L2 — the O(L1*L2) candidate cells; the
reference kernel does O(L1*L2^2) work for the same answers.

Every shape is repeated until at least --min-ms (default 60) of kernel time is measured, so launch skew
and tail effects stay small. --variants tile16,mfma runs the long-record sweep both ways (MOC_MFMA: the
matrix-core sweep, tile_mfma_kernels.hip) for an A/B on the same data; ``wire`` runs short-record shapes in
the wire formats, device-resident (solve_wire_device: P33 letters, narrow lengths, R2/R4 results).

  python tools/kernel_bench.py [--variants tile16,mfma] [--min-ms 60] [shape ...]
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: E402

from mpi_openmp_cuda_amd import HipSearchEngine, Problem, make_synthetic, search_cpu  # noqa: E402
from mpi_openmp_cuda_amd.ops.align import as_triples  # noqa: E402

# shape -> (records, Seq1 override length or None)
CASES = {"input6": (1 << 24, None), "input1": (1 << 21, None), "mid": (1 << 20, None), "heavy6": (1 << 22, None),
         "input4": (1 << 17, None), "heavy3": (1 << 13, None), "heavy4": (1 << 15, None),
         "input3": (1 << 15, None), "limits": (1 << 12, None), "heavylim": (1 << 12, None), "mid3k": (1 << 13, None),
         # long context: Seq1 beyond one LDS image -> the windowed tile16 sweep
         "long20k": (1 << 12, 20_000), "long150k": (1 << 9, 150_000)}
BASE = {"long20k": "input3", "long150k": "input3"}  # record-length distribution of the long-context shapes


def make(shape, n):
    prob = make_synthetic(BASE.get(shape, shape), n, seed=7)
    L1 = CASES[shape][1]
    if L1:
        rng = np.random.default_rng(L1)
        prob = Problem(prob.weights, rng.integers(1, 27, size=L1, dtype=np.uint8), prob.codes, prob.offsets)
    return prob


def run_wire(shape, n, min_ms, letter_format="p33"):
    """The same records in the wire formats, device-resident (P33 letters, narrow lengths, the narrowest
    results: the rccl transport's batches), through HipSearchEngine.solve_wire_device; kernel time from the
    engine's events."""
    from mpi_openmp_cuda_amd.parallel.wire import WireSlice

    prob = make(shape, n)
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    wire = WireSlice.from_csr(prob.codes, prob.offsets, letter_format=letter_format)
    res = wire.alloc_results(eng)
    dev = torch.device("cuda:0")
    letters = torch.from_numpy(wire.codes).to(dev)
    offsets = torch.from_numpy(wire.offsets).to(dev)
    lengths = torch.from_numpy(wire.lengths).to(dev) if wire.lengths is not None else None
    out = torch.zeros(res.nbytes, dtype=torch.uint8, device=dev)
    args = (letters, offsets, lengths, wire.n, out, wire.fmt, (wire.l2_min, wire.l2_max))
    kw = dict(lengths_bits=wire.len_bits or 8, lengths_base=wire.len_base, packed33=letter_format == "p33")
    eng.solve_wire_device(*args, **kw)  # warm-up
    first = max(eng.stats()["kernel_ms"], 1e-3)
    iters = max(5, math.ceil(min_ms / first))
    total = 0.0
    for _ in range(iters):
        eng.solve_wire_device(*args, **kw)
        total += eng.stats()["kernel_ms"]
    ms = total / iters
    res.view(np.uint8)[:] = out.cpu().numpy()
    nv = min(prob.n, 4000)
    ok = bool(np.array_equal(wire.triples(eng, nv), as_triples(search_cpu(prob.slice(0, nv)))))
    cells = prob.cells()
    dev_bytes = letters.numel() + (lengths.numel() if lengths is not None else 0) + out.numel()
    return {"shape": shape, "variant": f"wire-{wire.letter_format}-len{wire.len_bits}-{wire.fmt}", "records": prob.n,
            "L1": prob.L1, "letters": prob.total_chars, "cells": cells, "iters": iters, "gpu_ms": round(ms, 4),
            "timing": "kernel_events", "cells_per_s": cells / (ms / 1e3), "records_per_s": prob.n / (ms / 1e3),
            "hbm_bytes_per_record": round(dev_bytes / prob.n, 2), "kernels": eng.stats()["kernels"], "verified": ok}


def run(shape, n, variant, min_ms):
    os.environ["MOC_MFMA"] = "1" if variant == "mfma" else "0"
    prob = make(shape, n)
    eng = HipSearchEngine(device=0)
    eng.set_problem(prob.weights, prob.seq1)
    dev = torch.device("cuda:0")
    codes = torch.from_numpy(prob.codes).to(dev)
    offs = torch.from_numpy(prob.offsets).to(dev)
    out = torch.empty((prob.n, 3), dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    eng.solve_device(codes, offs, prob.offsets, out, s)  # warm-up (and host planning cache warm)
    try:
        first = eng.device_kernel_ms()
        timing = "kernel_events"
    except AttributeError:  # an older build (MOC_LIB_PATH) without the engine's kernel events
        torch.cuda.synchronize()
        first, timing = 1.0, "loop"
    iters = max(5, math.ceil(min_ms / max(first, 1e-3)))
    # kernel time: events the engine records around its launches, after the host's per-call planning
    # (plan_chunk scans every record's offsets on the host: at 16.7 M records that planning, not the
    # kernel, would set the pace of back-to-back calls)
    total = 0.0
    if timing == "kernel_events":
        for _ in range(iters):
            eng.solve_device(codes, offs, prob.offsets, out, s)
            total += eng.device_kernel_ms()
    # the same calls back to back, as a caller sees them (host planning included)
    t_host = time.perf_counter()
    e0.record(s)
    for _ in range(iters):
        eng.solve_device(codes, offs, prob.offsets, out, s)
    e1.record(s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t_host) / iters
    loop_ms = e0.elapsed_time(e1) / iters
    if timing == "loop":
        total = loop_ms * iters
    ms = total / iters
    nv = min(prob.n, 4000)
    ref = as_triples(search_cpu(prob.slice(0, nv)))
    ok = bool(np.array_equal(out[:nv].cpu().numpy(), ref))
    cells = prob.cells()
    return {"shape": shape, "variant": variant, "records": prob.n, "L1": prob.L1, "letters": prob.total_chars,
            "cells": cells, "iters": iters, "kernel_ms_total": round(total, 2), "gpu_ms": round(ms, 4),
            "loop_gpu_ms": round(loop_ms, 4), "host_wall_ms": round(wall * 1e3, 4), "timing": timing, "cells_per_s": cells / (ms / 1e3),
            "records_per_s": prob.n / (ms / 1e3), "kernels": eng.stats()["kernels"], "verified": ok}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("shapes", nargs="*")
    ap.add_argument("--variants", default="tile16")
    ap.add_argument("--min-ms", type=float, default=60.0)
    args = ap.parse_args()
    shapes = args.shapes or list(CASES)
    for shape in shapes:
        for variant in args.variants.split(","):
            if variant in ("wire", "wirebytes"):  # wirebytes: the wire lengths and results, byte letters
                print(json.dumps(run_wire(shape, CASES[shape][0], args.min_ms,
                                          "bytes" if variant == "wirebytes" else "p33")), flush=True)
            else:
                print(json.dumps(run(shape, CASES[shape][0], variant, args.min_ms)), flush=True)
