"""Multi-process torch.distributed path on CPU (gloo, world_size 2-3): the Python driver (parallel/search.py)
must reproduce the goldens with its record slices (node-shared window) and its context-parallel split
(window or broadcast), for any world size."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT, expected, input_path

def _free_port():
    # an OS-assigned port: fixed counters collide across pytest-xdist workers (EADDRINUSE)
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def torchrun(nproc, args, timeout=180):
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "mpi_openmp_cuda_amd"] + args
    return subprocess.run(cmd, capture_output=True, timeout=timeout, env=env, cwd="/tmp")


@pytest.mark.parametrize("transport", ["shm"])
@pytest.mark.parametrize("i,nproc", [(3, 2), (6, 3), (2, 2)])
def test_gloo_goldens(transport, i, nproc):
    r = torchrun(nproc, ["--backend=cpu", "--dist-backend=gloo", f"--transport={transport}",
                         f"--input={input_path(i)}"])
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert r.stdout.decode() == expected(i)


@pytest.mark.parametrize("transport", ["shm", "bcast"])
@pytest.mark.parametrize("i,nproc", [(3, 2), (2, 3), (4, 2)])
def test_gloo_context_parallel(transport, i, nproc):
    # --partition=offsets: every rank searches a share of every record; MAX all-reduce of packed keys
    r = torchrun(nproc, ["--backend=cpu", "--dist-backend=gloo", f"--transport={transport}", "--partition=offsets",
                         f"--input={input_path(i)}"])
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert r.stdout.decode() == expected(i)


def test_record_slices_between_ranks_belong_to_final():
    # one distributed implementation per transport: payload sends between ranks are ./final's (rccl)
    r = torchrun(2, ["--backend=cpu", "--dist-backend=gloo", "--transport=bcast", "--partition=records",
                     f"--input={input_path(1)}"], timeout=120)
    assert r.returncode != 0 and b"--transport=rccl" in r.stderr


def test_bcast_transport_defaults_to_offsets_partition():
    # the default partition (auto) with the transport that crosses nodes splits offsets, so a multi-node
    # launch on default flags runs instead of failing the records/bcast check
    r = torchrun(2, ["--backend=cpu", "--dist-backend=gloo", "--transport=bcast", f"--input={input_path(3)}"])
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    assert r.stdout.decode() == expected(3)


def test_process_group_timeout_from_env(monkeypatch):
    import datetime

    from mpi_openmp_cuda_amd.parallel import dist as D

    monkeypatch.setenv("MOC_COMM_TIMEOUT", "7.5")
    assert D.pg_timeout_kwargs() == {"timeout": datetime.timedelta(seconds=7.5)}
    monkeypatch.setenv("MOC_COMM_TIMEOUT", "0")
    assert D.pg_timeout_kwargs() == {}
    monkeypatch.delenv("MOC_COMM_TIMEOUT")
    assert D.comm_timeout_s() == 300.0


def test_single_process_cli_stdin():
    with open(input_path(1), "rb") as f:
        r = subprocess.run([sys.executable, "-m", "mpi_openmp_cuda_amd", "--backend=cpu"], stdin=f,
                           capture_output=True, env=dict(os.environ, PYTHONPATH=ROOT), cwd="/tmp", timeout=120)
    assert r.returncode == 0 and r.stdout.decode() == expected(1)


def test_input_error_all_ranks_exit():
    bad = os.path.join("/tmp", "moc_bad_input.txt")
    with open(bad, "w") as f:
        f.write("1 2 3 4\nAB1\n1\nA\n")
    r = torchrun(2, ["--backend=cpu", "--dist-backend=gloo", f"--input={bad}"], timeout=120)
    assert r.returncode != 0 and b"non-letter" in r.stderr
