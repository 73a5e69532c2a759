#!/usr/bin/env python3
"""Headline benchmark: elements/s of the full distributed search on input6-shaped data.

Metric (BASELINE.json): "wall-clock (s) + elements/sec on input6.txt array at 1/2/4/8 MI355X", on
synthetic arrays of the input6.txt shape (W = 4 3 2 10, |Seq1| = 26, |Seq2| in 6..11; no datasets are
available offline, so records are drawn at random; data="synthetic").

One timed step = the search of one complete job over the global batch (reference flow main.c:149-197):
  1. root broadcasts the problem header (weights + Seq1) over the process group (RCCL on GPUs),
  2. every rank uploads it to its engine (LUT + Seq1 -> device),
  3. every rank streams its contiguous slice of the records from host memory bound to its GPU's NUMA node
     (zero-copy over its own PCIe link), runs the gfx950 search kernel, and writes the (score, n, k)
     results back into the node-shared result array the root prints from,
  4. an all-reduce of the per-rank record counts closes the job (the reference's MPI_Gather point).
The records are held in the wire formats `./final` writes while it parses (P33 letters: 7 per 33 bits, base-6 lengths,
R2 results; csrc/include/moc/wire.hpp): encoding them is the untimed set-up here, as parsing and printing
are outside `./final`'s compute phase, whose `--timing` shows the same kernel time for the same letters
(profiles/final_scale_1.1G_r2_p33.log: 13.13 ms kernel at 1.14 G letters; profiles/bench_input6_1gpu_1.1G_p33.log:
13.15 ms kernel, 13.26 ms/step here).
Weak scaling: --records-per-gpu is fixed per rank, the global batch grows with N.

Run: python bench.py [--gpus N --steps K --warmup W]. With N > 1 and no torch.distributed environment
(WORLD_SIZE unset) the script launches itself: a child `python -m torch.distributed.run
--nproc-per-node N --master-addr 127.0.0.1 bench.py ...` started before anything touches the GPU, whose
exit code it returns (reference: `mpiexec -np 2 ./final`, /root/reference/makefile:11). Under a launcher
the world size must equal --gpus and every rank needs its own GPU, or the run fails (no silent 1-rank
fallback).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "wall-clock (s) + elements/sec on input6.txt array at 1/2/4/8 MI355X"


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--records-per-gpu", type=int, default=1 << 25)
    ap.add_argument("--shape", default="input6")
    ap.add_argument("--shm", type=int, default=1, help="1: node-shared /dev/shm arrays; 0: private pinned")
    ap.add_argument("--host-alloc", default="", help="'hip': private hipHostMalloc arrays (overrides --shm)")
    ap.add_argument("--verify", type=int, default=20000, help="records per rank checked against the CPU engine")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL, default) | gloo (multi-rank rehearsal)")
    ap.add_argument("--numa", type=int, default=1, help="bind each rank to its GPU's NUMA node")
    ap.add_argument("--final-wall", type=int, default=1,
                    help="1: also time `mpiexec -np N ./final < input6.txt` (median of 5, checked vs the golden)")
    ap.add_argument("--dump-steps", default="", help="rank 0 writes its per-step kernel and host ms to this JSON file")
    ap.add_argument("--dry-launch", action="store_true",
                    help="print the self-launch command (JSON) for --gpus N > 1 and exit; touches no GPU")
    ap.add_argument("--comm-timeout", type=float, default=300.0,
                    help="seconds a collective may wait on a peer before the job fails (0: torch's default)")
    ap.add_argument("--allow-shared-gpu", action="store_true",
                    help="rehearsals only (gloo): let several ranks share a GPU instead of failing")
    return ap.parse_args()


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(args, argv, port=None):
    """The torch.distributed.run command line that runs this script as `args.gpus` ranks (one per GPU)."""
    port = port or _free_port()
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + \
        [a for a in argv if a != "--dry-launch"]


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def kfd_gpu_count(root=KFD_NODES, env=None, dri="/dev/dri"):
    """GPUs from the KFD topology in sysfs — no HIP runtime, no torch in the launcher: topology nodes whose
    properties report SIMDs (CPU nodes report simd_count 0) and whose render node /dev/dri/renderD<minor>
    this process may open (a shared host exposes a job only its own GPUs; the runtime filters the same way,
    csrc/src/runtime/kfd_topology.cpp). ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES
    narrow the count as the runtime would. None when there is no KFD topology."""
    env = os.environ if env is None else env
    try:
        nodes = os.listdir(root)
    except OSError:
        return None
    n = 0
    for node in nodes:
        try:
            with open(os.path.join(root, node, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if len(line.split(None, 1)) == 2)
        except (OSError, ValueError):
            continue
        if int(props.get("simd_count", "0").strip() or 0) <= 0:
            continue
        minor = props.get("drm_render_minor", "").strip()
        if minor and not os.access(os.path.join(dri, f"renderD{minor}"), os.R_OK | os.W_OK):
            continue  # another tenant's GPU
        n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def visible_gpus(wanted=1):
    """GPU count for the launcher, from sysfs (kfd_gpu_count): the launcher must not hold the GPU while its
    children use it. When sysfs shows fewer than `wanted` (or nothing), torch's count (no GPU context on
    this image) has the last word, so a render-node permission the sysfs reading gets wrong cannot
    refuse a launch the runtime would run."""
    n = kfd_gpu_count()
    if n is not None and n >= wanted:
        return n
    # torch's count in a short-lived child: the launcher itself must not start a HIP runtime
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=300)
    try:
        t = int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        t = 0
    return max(n or 0, t)


SHM_PREFIX = "/dev/shm/moc_bench_"


def cleanup_stale_shm(before=None, prefix=SHM_PREFIX):
    """Removes node-shared bench arrays left by a crashed run: this user's /dev/shm/moc_bench_* files last
    modified before `before` (the launcher's start). Names only — a process that still maps one keeps it.
    Returns the removed paths."""
    before = time.time() if before is None else before
    d, base = os.path.split(prefix)
    removed = []
    try:
        names = os.listdir(d)
    except OSError:
        return removed
    for name in names:
        if not name.startswith(base):
            continue
        p = os.path.join(d, name)
        try:
            st = os.stat(p)
            if st.st_uid == os.getuid() and st.st_mtime < before:
                os.unlink(p)
                removed.append(p)
        except OSError:
            pass
    return removed


def final_input6_wall(np_, reps=5, timeout=20, extra=(), spacing=0.0):
    """The BASELINE metric's wall-clock half: the reference's own invocation `mpiexec -np N ./final <
    input6.txt` (default flags; /root/reference/makefile:10-11) with N = this run's GPU count, median of
    `reps` runs, every output compared with the golden. None when ./final or mpiexec is missing.
    `extra` adds flags: ("--backend=hip",) times the same job forced onto the MI355X (the default engine
    choice runs a job this small on the OpenMP engine: 1 ms of CPU work against the GPU runtime's start).
    `spacing` seconds pass between launches: a GPU process started right after another one waits in the
    kernel driver for the previous one's teardown (139-208 ms instead of 52-74 ms for the runtime's start,
    profiles/hip_init_trace_b2b.log), which a single invocation on an idle GPU does not."""
    final = os.path.join(ROOT, "final")
    inp = os.path.join(ROOT, "tests", "data", "input6.txt")
    gold = os.path.join(ROOT, "tests", "data", "expected", "input6.out")
    mpiexec = os.path.join(os.environ.get("MPI_HOME", "/opt/conda"), "bin", "mpiexec")
    if not (os.path.exists(final) and os.path.exists(mpiexec) and os.path.exists(inp)):
        return None
    with open(gold, "rb") as f:
        want = f.read()
    walls, ok = [], True
    env = {k: v for k, v in os.environ.items()
           if not k.startswith(("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_", "ROLE_", "TORCHELASTIC",
                                "MASTER_"))}
    for i in range(reps):
        if i and spacing:
            time.sleep(spacing)
        with open(inp, "rb") as fin:
            t0 = time.perf_counter()
            try:
                r = subprocess.run([mpiexec, "-np", str(np_), final, *extra], stdin=fin, capture_output=True,
                                   timeout=timeout, env=env)
            except subprocess.TimeoutExpired:  # one stuck launch ends the measurement (bounded: 20 s)
                return {"wall_s": None, "ok": False, "np": np_}
            walls.append(time.perf_counter() - t0)
        ok = ok and r.returncode == 0 and r.stdout == want
        if not ok:  # a failing launcher or binary: report it once instead of retrying
            break
    out = {"wall_s": round(float(np.median(walls)), 4), "best_s": round(min(walls), 4), "ok": bool(ok), "np": np_}
    if spacing:
        out["spacing_s"] = spacing
    return out


def pci_bus_id(code):
    """PCIe address 'dddd:bb:dd.f' of an int from pci_bus_code, or None."""
    if code is None or code < 0:
        return None
    code = int(code)
    return f"{code >> 16:04x}:{(code >> 8) & 0xff:02x}:{(code >> 3) & 0x1f:02x}.{code & 7:x}"


def pci_bus_code(bus_id):
    """'dddd:bb:dd.f' -> int (domain << 16 | bus << 8 | device << 3 | function), -1 when unknown."""
    try:
        dom, bus, rest = bus_id.lower().split(":")
        dev, fn = rest.split(".")
        return (int(dom, 16) << 16) | (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn, 16)
    except (AttributeError, ValueError):
        return -1


def self_launch(args, argv):
    """--gpus N > 1 outside a launcher: run N ranks as a child torch.distributed.run job and return its
    exit code. Fails (exit 2) when fewer than N GPUs are visible, instead of measuring fewer ranks."""
    cmd = launch_command(args, argv)
    if args.dry_launch:
        print(json.dumps({"launch": cmd, "nproc": args.gpus}), flush=True)
        return 0
    n_dev = visible_gpus(args.gpus)
    if n_dev < args.gpus and not args.allow_shared_gpu:
        print(f"bench.py: --gpus {args.gpus} but only {n_dev} GPU(s) visible", file=sys.stderr, flush=True)
        return 2
    stale = cleanup_stale_shm()
    if stale:
        print(f"[bench] removed {len(stale)} stale node-shared array(s) of an earlier run", file=sys.stderr, flush=True)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env=env).returncode


class HostArrays:
    """Per-rank slice of the node-shared input/result arrays (/dev/shm files, or private memory), in the
    wire formats `./final` writes while it parses (mpi_openmp_cuda_amd/parallel/wire.py: the same
    WireSlice the distributed driver's golden tests run)."""

    def __init__(self, tag, rank, lengths, use_shm, seed, hip_alloc=False):
        from mpi_openmp_cuda_amd.parallel.wire import WireSlice
        from mpi_openmp_cuda_amd.utils.synthetic import fill_codes

        n = lengths.shape[0]
        total = int(lengths.sum())
        self.paths = []
        self.shm = False
        nbytes = 8 * (n + 1) + 12 * n + total
        if use_shm and os.path.isdir("/dev/shm"):
            st = os.statvfs("/dev/shm")
            # leave room for every local rank's slice (up to 8) plus headroom
            if st.f_bavail * st.f_frsize > 10 * nbytes:
                self.shm = True
        self.bufs = []
        if hip_alloc:
            self.shm = False
            from mpi_openmp_cuda_amd._lib import HostBuffer

            def mk(name, dtype, count):
                b = HostBuffer(np.dtype(dtype).itemsize * max(count, 1))
                self.bufs.append(b)
                return b.array(dtype, max(count, 1))[:count]
        elif self.shm:
            def mk(name, dtype, count):
                p = f"/dev/shm/moc_bench_{tag}_{rank}_{name}"
                self.paths.append(p)
                return np.memmap(p, dtype=dtype, mode="w+", shape=(max(count, 1),))[:count]
        else:
            def mk(name, dtype, count):
                return np.empty(count, dtype=dtype)
        # letters: random codes 1..26, encoded once (P33 fields, base-6 lengths) like final's parser does
        letters = np.empty(total, dtype=np.uint8)
        fill_codes(letters, seed)
        self.wire = WireSlice(lengths, letters, alloc=mk)
        self.check_letters = letters[:min(total, 1 << 22)].copy()  # kept for the untimed verification
        del letters

    def cleanup(self):
        for b in self.bufs:
            b.free()
        self.bufs = []
        for p in self.paths:
            try:
                os.unlink(p)
            except OSError:
                pass


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.dry_launch):
        if args.gpus <= 1:
            print(json.dumps({"launch": None, "nproc": 1}), flush=True)
            return 0
        return self_launch(args, sys.argv[1:])
    import torch
    import torch.distributed as dist

    from mpi_openmp_cuda_amd import HipSearchEngine, Problem, search_cpu
    from mpi_openmp_cuda_amd._lib import Pinned
    from mpi_openmp_cuda_amd.ops.align import as_triples
    from mpi_openmp_cuda_amd.utils.synthetic import SHAPES

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: refusing to report a different rank count",
              file=sys.stderr, flush=True)
        return 2
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    n_dev = torch.cuda.device_count()
    if n_dev < 1 or (n_dev < local_world and not args.allow_shared_gpu):
        print(f"bench.py: {local_world} local ranks but {n_dev} GPU(s) visible (one rank per GPU)",
              file=sys.stderr, flush=True)
        return 2
    gpu = local_rank % n_dev
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    distributed = world > 1
    nccl = args.dist_backend == "nccl"
    # where collective tensors live: the GPU for RCCL; the host for gloo and for a single rank (no
    # collective runs then, so a device copy of the header would only add a D2H sync per step)
    cdev = dev if (nccl and distributed) else torch.device("cpu")
    if distributed:
        # a stuck peer fails the step with a timeout instead of hanging the job (the driver's clock)
        import datetime

        pg_kw = {"timeout": datetime.timedelta(seconds=args.comm_timeout)} if args.comm_timeout > 0 else {}
        if nccl:
            dist.init_process_group("nccl", device_id=dev, **pg_kw)
        else:
            dist.init_process_group("gloo", **pg_kw)
        if dist.get_world_size() != args.gpus:
            print(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}", file=sys.stderr)
            return 2

    if world == 1:
        cleanup_stale_shm()  # a single rank is its own launcher
    t_setup = time.perf_counter()

    def progress(msg):  # setup of big batches takes minutes: keep stderr alive (rank 0)
        if rank == 0:
            print(f"[bench] {time.perf_counter() - t_setup:7.1f}s {msg}", file=sys.stderr, flush=True)

    def barrier():
        if distributed:
            if nccl:
                dist.barrier(device_ids=[gpu])
            else:
                dist.barrier()
        torch.cuda.synchronize(dev)

    from mpi_openmp_cuda_amd import _lib

    # host buffers the GPU streams over PCIe go on the NUMA node of its root complex
    numa = _lib.lib().moc_bind_numa(gpu) if args.numa else -1
    shape = SHAPES[args.shape]
    # ---- problem header (root) and this rank's synthetic slice (untimed setup = the parsed input)
    rng = np.random.default_rng(args.seed)
    seq1 = rng.integers(1, 27, size=shape.L1, dtype=np.uint8)
    weights = np.array(shape.weights, dtype=np.int32)
    header = torch.from_numpy(np.concatenate([weights, seq1.astype(np.int32)])).to(cdev)
    R = args.records_per_gpu
    rrng = np.random.default_rng(args.seed + 1 + rank)
    lengths = rrng.integers(shape.l2_min, shape.l2_max + 1, size=R, dtype=np.int64)
    tag = os.environ.get("MASTER_PORT", str(os.getpid()))
    progress(f"generating {R} records per rank")
    host = HostArrays(tag, rank, lengths, bool(args.shm), args.seed + 101 + rank, hip_alloc=args.host_alloc == "hip")
    wire = host.wire
    progress(f"{wire.total} letters per rank ready")
    del lengths
    eng = HipSearchEngine(device=gpu)
    eng.set_problem(weights, seq1)
    wire.alloc_results(eng)  # the narrowest result format for this slice (R2 on input6)
    fmt = wire.fmt
    pin = Pinned(*([] if host.bufs else wire.arrays()))
    progress("host arrays page-locked; warm-up")
    done = torch.zeros(1, dtype=torch.int64, device=cdev)
    # The header reaches every rank's host once, before the steps (the reference's MPI_Bcast of Seq1 and the
    # weights, main.c:149-150, is a host broadcast): each step still broadcasts it over the process group and
    # sets it on the engine, but the engine's host image comes from this copy, so no step waits on a device
    # -> host copy of the broadcast (a device sync per step at N > 1). The last step's device copy is checked
    # against it in the verification below.
    if distributed:
        dist.broadcast(header, src=0)
    hdr_host = header.cpu().numpy().copy()
    w_host, s1_host = hdr_host[:4].copy(), hdr_host[4:].astype(np.uint8)

    def step():
        if distributed:
            dist.broadcast(header, src=0)
        eng.set_problem(w_host, s1_host)
        wire.solve(eng)
        done.fill_(R)
        if distributed:
            dist.all_reduce(done)

    for _ in range(args.warmup):
        step()
    barrier()
    progress(f"timing {args.steps} steps")
    t0 = time.perf_counter()
    kms, tms, sms, ends = [], [], [], []
    t_prev = t0
    for _ in range(args.steps):
        step()
        k_ms, t_ms = eng.kernel_times()
        kms.append(k_ms)
        tms.append(t_ms)
        t_now = time.perf_counter()  # host clock per step (rank 0's view; the job is timed by t0 / elapsed)
        sms.append((t_now - t_prev) * 1e3)
        ends.append(time.time())  # wall-clock end of the step (correlated with tools/gpu_sampler.py samples)
        t_prev = t_now
    barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    if distributed:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    st = eng.stats()

    # ---- verification (untimed): the result array is poisoned and one more step is run, so a step that
    # skipped work (stale results from an earlier step) cannot pass; a sample is checked vs the CPU engine
    res = wire.results
    # poison: R2's 0xFFFF is also its "no candidate" code, a sentinel only when every record has a candidate
    # (|Seq2| < |Seq1| for the whole shape); R4/R8/R12 all-zero rows never occur (n or k or score non-zero
    # is not guaranteed either, so those check the decoded sample only)
    sentinel = res.dtype.kind == "u" and shape.l2_max < shape.L1
    res[:] = np.iinfo(res.dtype).max if res.dtype.kind == "u" else 0
    step()
    barrier()
    nv = min(args.verify, R)
    while nv > 0 and int(wire.offsets[nv]) > host.check_letters.shape[0]:
        nv //= 2
    ok = 1
    if nv > 0:
        sub = Problem(shape.weights, seq1, host.check_letters[:int(wire.offsets[nv])], wire.offsets[:nv + 1].copy())
        ref = as_triples(search_cpu(sub))
        ok = int(np.array_equal(wire.triples(eng, nv), ref))
        # a sample from the end of the slice, where the persistent grid runs its tail tiles: letters decoded
        # back from the wire form, every result of the sample checked against the CPU engine
        nt = min(nv, R)
        t0 = int(wire.offsets[R - nt])
        sub_t = Problem(shape.weights, seq1, wire.letters(t0, wire.total), wire.offsets[R - nt:] - t0)
        r2 = eng.r2_params(wire.l2_min, wire.l2_max) if wire.fmt == "r2" else None
        ok &= int(np.array_equal(as_triples(res[R - nt:], r2=r2), as_triples(search_cpu(sub_t))))
        # and the tail of the batch was written by the last step too (no sentinel left anywhere)
        tail = res[R - min(R, 1 << 16):]
        if sentinel:
            ok &= int(not (tail == np.iinfo(res.dtype).max).any())
    ok &= int(np.array_equal(header.cpu().numpy(), hdr_host))  # the header every step broadcast is the one used
    okt = torch.tensor([ok], dtype=torch.int32, device=cdev)
    if distributed:
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)

    total_records = R * world
    total_elems = wire.total * world  # per-rank chars ~ equal (same length distribution)
    if distributed:
        te = torch.tensor([wire.total], dtype=torch.int64, device=cdev)
        dist.all_reduce(te)
        total_elems = int(te.item())
    # per-rank evidence: NUMA node of the host arrays, median kernel ms per step, device index, letters, step
    # time p50/p99 (this rank's clock), PCIe link rate of the stream (bytes in / kernel time), PCIe address —
    # so a slow step or a slow link in a scaling run is attributable to a rank from the record alone
    from mpi_openmp_cuda_amd.ops.align import device_info

    bus = pci_bus_code(device_info(gpu).get("pci_bus_id"))
    k_med = float(np.median(kms))
    h2d_gbps = st["h2d_bytes"] / (k_med * 1e6) if k_med > 0 else 0.0
    mine = torch.tensor([float(numa), k_med, float(gpu), float(wire.total), float(np.percentile(sms, 50)),
                         float(np.percentile(sms, 99)), h2d_gbps, float(bus)], dtype=torch.float64, device=cdev)
    if distributed:
        allv = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allv, mine)
        per_rank = torch.stack(allv).cpu().numpy()
    else:
        per_rank = mine.cpu().numpy()[None, :]
    # the literal wall-clock of the reference invocation on input6.txt at this rank count (rank 0, untimed,
    # after the steps; the other ranks wait at the barrier below)
    wall6 = final_input6_wall(world) if (rank == 0 and args.final_wall) else None
    wall6_hip = (final_input6_wall(world, extra=("--backend=hip",), spacing=1.0)
                 if (rank == 0 and args.final_wall) else None)
    ms_per_step = elapsed / args.steps * 1e3
    value = total_elems * args.steps / elapsed
    cells_per_rec = float(np.mean([(shape.L1 - l + 1) * l for l in range(shape.l2_min, shape.l2_max + 1)]))
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "elements/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "wall_clock_s": round(elapsed, 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {
                "model": f"{args.shape}-shaped alignment search (W={list(shape.weights)}, |Seq1|={shape.L1}, "
                         f"|Seq2|={shape.l2_min}..{shape.l2_max})",
                "global_batch": total_records,
                "seq_len": shape.L1,
                "parallelism": f"dp{world}",
            },
            "records_per_s": round(total_records * args.steps / elapsed, 1),
            "cells_per_s_est": round(total_records * cells_per_rec * args.steps / elapsed, 1),
            "rank0_kernel_ms_per_step": round(float(np.median(kms)), 4),
            "rank0_kernel_ms_min_max": [round(min(kms), 4), round(max(kms), 4)],
            "rank0_kernel_ms_p90_p99": [round(float(np.percentile(kms, 90)), 4), round(float(np.percentile(kms, 99)), 4)],
            "rank0_step_ms_p50_p99": [round(float(np.percentile(sms, 50)), 4), round(float(np.percentile(sms, 99)), 4)],
            "rank0_solve_ms_median": round(float(np.median(tms)), 4),
            "rank0_h2d_bytes_per_step": int(st["h2d_bytes"]),
            "rank0_d2h_bytes_per_step": int(st["d2h_bytes"]),
            "host_arrays": "hip_host_malloc" if host.bufs else ("shm" if host.shm else "private"),
            "result_format": fmt,
            "lengths": "base6" if wire.len_bits == 6 else (f"{wire.len_bits}bit" if wire.len_bits else "offsets"),
            "letters": wire.letter_format,
            "rank0_numa_node": numa,
            # only what ran: an RCCL communicator exists only for N > 1 ranks on the nccl backend
            "rccl_world": dist.get_world_size() if (distributed and nccl) else None,
            "dist_backend": ("nccl" if nccl else "gloo") if distributed else "none",
            "rank_numa_nodes": [int(x) for x in per_rank[:, 0]],
            "rank_kernel_ms": [round(float(x), 4) for x in per_rank[:, 1]],
            "rank_devices": [int(x) for x in per_rank[:, 2]],
            "rank_letters": [int(x) for x in per_rank[:, 3]],
            "rank_step_ms_p50_p99": [[round(float(a), 4), round(float(b), 4)] for a, b in per_rank[:, 4:6]],
            "rank_h2d_gbps": [round(float(x), 2) for x in per_rank[:, 6]],
            "rank_pci_bus": [pci_bus_id(int(x)) for x in per_rank[:, 7]],
            "rank0_kernels": st["kernels"],
            "host_stream": "zero_copy" if st["direct"] else "staged",
            "verified": bool(okt.item()),
            # each timed step broadcasts the header over the process group (N > 1) but the engine's image
            # comes from the host copy made before the loop (set_problem of an unchanged problem is a
            # no-op), as the reference broadcasts it once per job (main.c:149-150)
            "header_per_step": "broadcast_only" if distributed else "none",
            "final_input6_wall": wall6,
            "final_input6_wall_hip": wall6_hip,
        }
        print(json.dumps(out), flush=True)
        if args.dump_steps:
            with open(args.dump_steps, "w") as f:
                json.dump({"kernel_ms": kms, "step_ms": sms, "solve_ms": tms, "end_time": ends}, f)
    pin.release()
    if distributed:
        barrier()
        dist.destroy_process_group()
    host.cleanup()


if __name__ == "__main__":
    sys.exit(main() or 0)
