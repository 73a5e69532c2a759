"""torch.distributed plumbing: one process per GPU, RCCL ("nccl") on GPUs, gloo on CPU.

The torch-side twin of csrc/src/comm/comm.cpp (MPI + RCCL for the native CLI). Rendezvous comes from
the torch.distributed.run environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT);
use 127.0.0.1 as master address on single hosts.
"""
from __future__ import annotations

import os
import socket
from dataclasses import dataclass
from typing import List, Optional

import numpy as np


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: str = "none"  # nccl | gloo | none
    device: Optional[object] = None  # torch.device used for collectives
    single_node: bool = True

    @property
    def distributed(self) -> bool:
        return self.world > 1

    @property
    def is_root(self) -> bool:
        return self.rank == 0


def comm_timeout_s() -> float:
    """The job's deadline for any wait on another rank (seconds): MOC_COMM_TIMEOUT, as `./final
    --comm-timeout` (csrc/include/moc/runtime/watchdog.hpp), default 300; <= 0 leaves torch's own default."""
    try:
        return float(os.environ.get("MOC_COMM_TIMEOUT", "300"))
    except ValueError:
        return 300.0


def pg_timeout_kwargs() -> dict:
    """init_process_group's `timeout=`: a collective stuck on a peer raises (RCCL: the process group's
    watchdog aborts the communicator) instead of hanging the job (reference: a failing rank exit(1)s and
    its peers block forever, /root/reference/cudaFunctions.cu:15-33)."""
    import datetime

    t = comm_timeout_s()
    return {"timeout": datetime.timedelta(seconds=t)} if t > 0 else {}


def init(backend: str = "auto", use_gpu: Optional[bool] = None) -> DistContext:
    """Initialises the default process group from the environment (no-op for a single process)."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    if backend == "auto":
        backend = "nccl" if use_gpu else "gloo"
    dev = torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1)) if backend == "nccl" else \
        torch.device("cpu")
    if backend == "nccl":
        torch.cuda.set_device(dev)
    ctx = DistContext(rank, world, local_rank, backend if world > 1 else "none", dev)
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": dev} if backend == "nccl" else {}
        kw.update(pg_timeout_kwargs())
        # gloo prints its connection banner on stdout; stdout must carry results only (main.c:204), so
        # the native banner goes to stderr while the group is set up.
        import sys

        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(backend, **kw)
            if backend == "gloo":
                dist.barrier()  # connections are established lazily on the first collective
        finally:
            os.dup2(saved, 1)
            os.close(saved)
    if world > 1:
        hosts: List[str] = [None] * world  # type: ignore
        dist.all_gather_object(hosts, socket.gethostname())
        ctx.single_node = len(set(hosts)) == 1
    return ctx


def finalize(ctx: DistContext):
    import torch.distributed as dist

    if ctx.distributed and dist.is_initialized():
        dist.destroy_process_group()


def barrier(ctx: DistContext):
    import torch.distributed as dist

    if ctx.distributed:
        if ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.device.index])
        else:
            dist.barrier()


def bcast_array(ctx: DistContext, arr: Optional[np.ndarray], count: int, dtype, src: int = 0) -> np.ndarray:
    """Broadcasts a 1-D numpy array through the process group (device tensor on nccl)."""
    import torch
    import torch.distributed as dist

    if not ctx.distributed:
        return np.asarray(arr, dtype=dtype)
    tdt = {np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32, np.dtype(np.uint8): torch.uint8}[
        np.dtype(dtype)]
    if ctx.rank == src:
        t = torch.from_numpy(np.array(arr, dtype=dtype, copy=True)).to(ctx.device)
        assert t.numel() == count, f"broadcast size mismatch: {t.numel()} vs {count}"
    else:
        t = torch.empty(count, dtype=tdt, device=ctx.device)
    if count:
        dist.broadcast(t, src=src)
    return t.cpu().numpy()


def send_array(ctx: DistContext, arr: np.ndarray, dst: int):
    import torch
    import torch.distributed as dist

    if arr.size:
        dist.send(torch.from_numpy(np.ascontiguousarray(arr)).to(ctx.device), dst=dst)


def recv_array(ctx: DistContext, count: int, dtype, src: int) -> np.ndarray:
    import torch
    import torch.distributed as dist

    tdt = {np.dtype(np.int64): torch.int64, np.dtype(np.int32): torch.int32, np.dtype(np.uint8): torch.uint8}[
        np.dtype(dtype)]
    t = torch.empty(count, dtype=tdt, device=ctx.device)
    if count:
        dist.recv(t, src=src)
    return t.cpu().numpy()


def allreduce_max(ctx: DistContext, x: float) -> float:
    import torch
    import torch.distributed as dist

    if not ctx.distributed:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_max_int64(ctx: DistContext, arr: np.ndarray) -> np.ndarray:
    """Element-wise MAX of an int64 array over all ranks (RCCL on GPU ranks, gloo on CPU)."""
    import torch
    import torch.distributed as dist

    arr = np.ascontiguousarray(arr, dtype=np.int64)
    if not ctx.distributed or arr.size == 0:
        return arr
    t = torch.from_numpy(arr.copy()).to(ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.cpu().numpy()
