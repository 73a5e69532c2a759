"""Distributed search over a torch.distributed process group: the torch-facing API of the two distributed
strategies, on one node.

Reference flow (main.c:110-197): root reads, Bcast x4, Scatter fixed-stride records, per-rank GPU work,
Gather x3, root prints. Here:
  * header (weights, |Seq1|, N, semantics) + Seq1: exact-count broadcasts through the process group
    (RCCL on GPU ranks, gloo on CPU ranks);
  * cost-balanced contiguous bounds (parallel/partition.py), valid for any world size;
  * partition "records", transport "shm": the root writes the CSR batch once into a node-shared /dev/shm
    window; every rank streams its own slice to its GPU (zero-copy, the wire formats of parallel/wire.py)
    and writes its results back in place — no payload collectives at all;
  * partition "offsets" (context parallel): every rank sees every record (the shm window,
    or one broadcast with transport "bcast") and searches its share of each record's offsets; the packed
    64-bit candidate keys are combined with ONE MAX all-reduce (the Reduce the reference never had) and the
    root decodes them.
Moving record payloads between ranks (several nodes, or device-resident batches over RCCL/xGMI) is the
native driver's job, one implementation: ./final --transport=rccl (csrc/src/device_batch.cpp).
"""
from __future__ import annotations

import os
import uuid
from typing import Optional

import numpy as np

from .. import _lib
from ..models.problem import Problem
from ..models.scoring import Semantics
from ..ops.align import (HipSearchEngine, decode_keys, device_count, keys_to_ordered_int64, ordered_int64_to_keys,
                        search_cpu, search_keys_cpu)
from ..utils.timer import PhaseTimer
from . import dist as D
from .partition import CPU_COST, GPU_COST, partition
from .wire import WireSlice


class NodeWindow:
    """A /dev/shm file mapped by every rank of the node: offsets[N+1] | results[N] | codes[T]."""

    def __init__(self, name: str, n: int, total: int, create: bool):
        self.path = f"/dev/shm/{name}"
        self.n, self.total = n, total
        self.off_bytes = 8 * (n + 1)
        self.res_bytes = (12 * n + 7) & ~7
        size = max(self.off_bytes + self.res_bytes + total, 8)
        mode = "w+" if create else "r+"
        self._mm = np.memmap(self.path, dtype=np.uint8, mode=mode, shape=(size,))
        self.offsets = self._mm[:self.off_bytes].view(np.int64)
        self.results = self._mm[self.off_bytes:self.off_bytes + 12 * n].view(_lib.RESULT_DTYPE)
        self.codes = self._mm[self.off_bytes + self.res_bytes:self.off_bytes + self.res_bytes + total]

    def close(self, unlink: bool):
        self._mm._mmap.close() if getattr(self._mm, "_mmap", None) is not None else None
        if unlink:
            try:
                os.unlink(self.path)
            except OSError:
                pass


class DistributedSearch:
    def __init__(self, ctx: D.DistContext, backend: str = "auto", transport: str = "auto", threads: int = 0,
                 device: Optional[int] = None, partition: str = "auto"):
        self.ctx = ctx
        if partition == "auto":  # record slices need the node-shared window; across nodes split offsets
            partition = "records" if (ctx.single_node and transport in ("auto", "shm")) else "offsets"
        if partition not in ("records", "offsets"):
            raise ValueError("partition must be auto|records|offsets")
        self.partition = partition
        if backend == "auto":
            backend = "hip" if device_count() > 0 else "cpu"
        self.backend = backend
        if transport == "auto":
            transport = "shm" if ctx.single_node else "bcast"
        if transport not in ("shm", "bcast"):
            raise ValueError("transport must be shm|bcast")
        if transport == "shm" and not ctx.single_node:
            raise ValueError("transport=shm needs every rank on one node")
        if partition == "records" and transport != "shm":
            raise ValueError("record slices move between ranks in ./final (--transport=rccl); the Python driver "
                             "runs them through a node-shared window (transport=shm, one node)")
        self.transport = transport
        self.threads = threads
        if backend == "hip" and device is None:
            device = ctx.local_rank % max(device_count(), 1)  # node-local rank -> GPU (ranks may share one)
        self.engine = HipSearchEngine(device) if backend == "hip" else None
        self.timer = PhaseTimer()
        if partition == "offsets" and ctx.distributed:
            # GPU ranks split tile lists, CPU ranks offset ranges: one engine kind for the whole group
            kinds = D.allreduce_max_int64(ctx, np.array([1 if self.engine else 0, 0 if self.engine else 1]))
            if kinds[0] and kinds[1]:
                raise ValueError("partition=offsets needs the same backend on every rank")

    def _compute(self, prob: Problem, sem: Semantics, codes, offsets, out):
        if self.engine is not None:
            # GPU ranks: the slice in the wire formats ./final's parser writes and bench.py streams
            # (parallel/wire.py), page-locked, searched zero-copy, decoded into the R12 result window
            ws = WireSlice.from_csr(codes, offsets)
            ws.alloc_results(self.engine)
            with _lib.Pinned(*ws.arrays()):
                ws.solve(self.engine)
            out.view(np.int32).reshape(-1, 3)[:] = ws.triples(self.engine)
        else:
            sub = Problem(prob.weights, prob.seq1, codes[offsets[0]:offsets[-1]], offsets - offsets[0])
            out[:] = search_cpu(sub, sem, self.threads)

    def run(self, problem: Optional[Problem], semantics=Semantics.REFERENCE) -> Optional[np.ndarray]:
        ctx, T = self.ctx, self.timer
        sem = Semantics.parse(semantics)
        with T.phase("bcast"):
            if ctx.is_root:
                hdr = np.array(problem.weights.as_list() + [problem.L1, problem.n, problem.total_chars, int(sem)],
                               np.int64)
            else:
                hdr = None
            hdr = D.bcast_array(ctx, hdr, 8, np.int64)
            w, L1, n, total, sem = list(hdr[:4]), int(hdr[4]), int(hdr[5]), int(hdr[6]), Semantics(int(hdr[7]))
            seq1 = D.bcast_array(ctx, problem.seq1 if ctx.is_root else None, L1, np.uint8)
            prob = Problem(w, seq1)
            if self.engine is not None:
                self.engine.set_problem(w, seq1, sem)
            bounds = partition(problem.lengths, L1, ctx.world, GPU_COST if self.backend == "hip" else CPU_COST) \
                if ctx.is_root else None
            bounds = D.bcast_array(ctx, bounds, ctx.world + 1, np.int64)
        b, e = int(bounds[ctx.rank]), int(bounds[ctx.rank + 1])
        if self.partition == "offsets":
            return self._run_offsets(problem, prob, sem, n, total)
        return self._run_shm(problem, prob, sem, n, total, b, e)

    def _run_shm(self, problem, prob, sem, n, total, b, e):
        ctx, T = self.ctx, self.timer
        with T.phase("distribute"):
            name_arr = None
            if ctx.is_root:  # fixed 20-byte name: "moc_win_" + 12 hex digits
                name_arr = np.frombuffer(f"moc_win_{uuid.uuid4().hex[:12]}".encode(), np.uint8)
            name = bytes(D.bcast_array(ctx, name_arr, 20, np.uint8)).decode()
            win = None
            if ctx.is_root:
                win = NodeWindow(name, n, total, create=True)
                win.offsets[:] = problem.offsets
                win.codes[:] = problem.codes
                win._mm.flush()
            D.barrier(ctx)
            if not ctx.is_root:
                win = NodeWindow(name, n, total, create=False)
        with T.phase("compute"):
            if e > b:
                self._compute(prob, sem, win.codes, win.offsets[b:e + 1], win.results[b:e])
        with T.phase("gather"):
            D.barrier(ctx)
            out = np.array(win.results) if ctx.is_root else None
            D.barrier(ctx)
            win.close(unlink=ctx.is_root)
        return out

    def _keys(self, prob: Problem, sem: Semantics, codes, offsets) -> np.ndarray:
        if self.engine is not None:
            return self.engine.search_keys(codes, offsets, self.ctx.rank, self.ctx.world)
        sub = Problem(prob.weights, prob.seq1, codes[offsets[0]:offsets[-1]], offsets - offsets[0])
        return search_keys_cpu(sub, self.ctx.rank, self.ctx.world, sem, self.threads)

    def _run_offsets(self, problem, prob, sem, n, total):
        ctx, T = self.ctx, self.timer
        with T.phase("distribute"):  # every rank needs every record
            if self.transport == "shm":
                name_arr = None
                if ctx.is_root:
                    name_arr = np.frombuffer(f"moc_win_{uuid.uuid4().hex[:12]}".encode(), np.uint8)
                name = bytes(D.bcast_array(ctx, name_arr, 20, np.uint8)).decode()
                win = None
                if ctx.is_root:
                    win = NodeWindow(name, n, total, create=True)
                    win.offsets[:] = problem.offsets
                    win.codes[:] = problem.codes
                    win._mm.flush()
                D.barrier(ctx)
                if not ctx.is_root:
                    win = NodeWindow(name, n, total, create=False)
                codes, offsets = win.codes, win.offsets
            else:
                win = None
                offsets = D.bcast_array(ctx, problem.offsets if ctx.is_root else None, n + 1, np.int64)
                codes = D.bcast_array(ctx, problem.codes if ctx.is_root else None, total, np.uint8)
        with T.phase("compute"):
            keys = self._keys(prob, sem, np.asarray(codes), np.asarray(offsets)) if n else np.zeros(0, np.uint64)
        with T.phase("gather"):
            best = ordered_int64_to_keys(D.allreduce_max_int64(ctx, keys_to_ordered_int64(keys)))
            out = decode_keys(best, Problem(prob.weights, prob.seq1, np.asarray(codes), np.asarray(offsets))) \
                if ctx.is_root else None
            if win is not None:
                D.barrier(ctx)
                win.close(unlink=ctx.is_root)
        return out
