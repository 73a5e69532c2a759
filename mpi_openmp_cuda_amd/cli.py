"""Python CLI, same contract as ./final (stdin -> "#i: score: S, n: N, k: K" lines), over torch.distributed:

    python -m mpi_openmp_cuda_amd < input.txt
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m mpi_openmp_cuda_amd \
        --input input.txt

Only rank 0 reads the input and writes the output (PDF p.5).
"""
from __future__ import annotations

import argparse
import json
import sys

from .models.problem import Problem
from .models.scoring import Semantics
from .parallel import dist as D
from .parallel.search import DistributedSearch
from .utils.io import write_results


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="mpi_openmp_cuda_amd", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--input", default="-", help="input file (default: stdin)")
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "cpu"])
    ap.add_argument("--transport", default="auto", choices=["auto", "shm", "bcast"],
                    help="shm: node-shared window (one node); bcast: every record broadcast (--partition=offsets "
                         "only). Record slices between nodes: ./final --transport=rccl (the retired p2p transport "
                         "of this driver moved into ./final's device batch)")
    ap.add_argument("--partition", default="auto", choices=["auto", "records", "offsets"],
                    help="records: cost-balanced record ranges (one node); offsets: context parallel (split every "
                         "record; the only partition across nodes here). auto: records on one node, else offsets")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"])
    ap.add_argument("--semantics", default="reference", choices=["reference", "spec"])
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--strict-limits", action="store_true")
    ap.add_argument("--timing", action="store_true")
    a = ap.parse_args(argv)

    from .ops.align import device_count

    use_gpu = a.backend == "hip" or (a.backend == "auto" and device_count() > 0)
    ctx = D.init(a.dist_backend, use_gpu=use_gpu and a.dist_backend != "gloo")
    rc = 0
    problem = None
    err = ""
    if ctx.is_root:
        try:
            data = sys.stdin.buffer.read() if a.input == "-" else open(a.input, "rb").read()
            problem = Problem.parse(data, a.strict_limits)
        except Exception as e:  # report, then make every rank exit consistently
            err = str(e)
    import numpy as np

    status = D.bcast_array(ctx, np.array([1 if err else 0], np.int64) if ctx.is_root else None, 1, np.int64)
    if int(status[0]):
        if ctx.is_root:
            print(f"input error: {err}", file=sys.stderr)
        D.finalize(ctx)
        return 1
    search = DistributedSearch(ctx, backend="hip" if use_gpu else "cpu", transport=a.transport, threads=a.threads,
                               partition=a.partition)
    results = search.run(problem, Semantics.parse(a.semantics))
    if ctx.is_root:
        write_results(results)
        if a.timing:
            print(json.dumps({"timing": json.loads(search.timer.json()), "ranks": ctx.world,
                              "backend": search.backend, "transport": search.transport}), file=sys.stderr)
    D.barrier(ctx)
    D.finalize(ctx)
    return rc


if __name__ == "__main__":
    sys.exit(main())
