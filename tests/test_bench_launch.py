"""bench.py launcher contract (CPU only, no GPU touched): --gpus N > 1 outside torch.distributed launches
N ranks itself, and a rank count that does not match --gpus fails instead of reporting fewer GPUs."""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def run(args, env_extra=None, timeout=120):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, timeout=timeout, env=env, cwd="/tmp")


def test_dry_launch_builds_torchrun_command():
    r = run(["--gpus", "8", "--steps", "7", "--warmup", "2", "--dry-launch"])
    assert r.returncode == 0, r.stderr.decode()
    d = json.loads(r.stdout.decode().strip().splitlines()[-1])
    cmd = d["launch"]
    assert d["nproc"] == 8
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd and "--master-addr=127.0.0.1" in cmd
    assert any(a.startswith("--master-port=") for a in cmd)
    # the child re-runs this script with the same arguments, minus --dry-launch
    i = cmd.index(BENCH)
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "7", "--warmup", "2"]


def test_single_gpu_command_line_unchanged():
    r = run(["--dry-launch"])
    assert r.returncode == 0
    assert json.loads(r.stdout.decode().strip())["launch"] is None


def test_launch_refuses_without_enough_gpus():
    # this container has no GPU: a real 2-GPU launch must fail loudly, not fall back to one rank
    r = run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2
    assert b"GPU(s) visible" in r.stderr
    assert not r.stdout.strip()


def test_rank_refuses_world_mismatch():
    r = run(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert b"refusing to report a different rank count" in r.stderr
