"""bench.py launcher contract (CPU only, no GPU touched): --gpus N > 1 outside torch.distributed launches
N ranks itself, and a rank count that does not match --gpus fails instead of reporting fewer GPUs."""
import json
import os
import subprocess
import sys
import types

import pytest

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


def _bench_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_kfd_gpu_count_from_sysfs(tmp_path):
    # the launcher counts GPUs from the KFD topology (no HIP runtime, no torch): nodes with SIMDs are GPUs,
    # the *_VISIBLE_DEVICES variables narrow the count, a missing topology gives None (torch fallback)
    b = _bench_module()
    nodes = tmp_path / "nodes"
    for i, simds in enumerate([0, 0, 1024, 1024, 1024]):  # two CPU nodes, three GPUs
        (nodes / str(i)).mkdir(parents=True)
        (nodes / str(i) / "properties").write_text(f"cpu_cores_count 64\nsimd_count {simds}\ngfx_target_version 90500\n")
    (nodes / "9").mkdir()  # a node without properties is skipped
    assert b.kfd_gpu_count(str(nodes), env={}) == 3
    assert b.kfd_gpu_count(str(nodes), env={"HIP_VISIBLE_DEVICES": "0,2"}) == 2
    assert b.kfd_gpu_count(str(nodes), env={"ROCR_VISIBLE_DEVICES": ""}) == 0
    assert b.kfd_gpu_count(str(tmp_path / "absent"), env={}) is None
    # this container: no GPU nodes (or no KFD at all) -> the 2-GPU launch refusal above comes from sysfs
    assert b.kfd_gpu_count(env={}) in (None, 0)


def test_kfd_gpu_count_8gpu_node(tmp_path):
    # the 8-GPU, two-socket node of a SCALE run (csrc/tests/test_core.cpp test_kfd_topology_8gpu: the same
    # tree): 8 GPUs, narrowed by the visibility lists; a box exposing one render node counts 1
    b = _bench_module()
    nodes, dri = tmp_path / "nodes", tmp_path / "dri"
    dri.mkdir()
    for cpu in range(2):
        (nodes / str(cpu)).mkdir(parents=True)
        (nodes / str(cpu) / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    for g in range(8):
        (nodes / str(2 + g)).mkdir()
        (nodes / str(2 + g) / "properties").write_text(f"simd_count 1024\ndrm_render_minor {128 + g}\n")
        (dri / f"renderD{128 + g}").write_text("")
    assert b.kfd_gpu_count(str(nodes), env={}, dri=str(dri)) == 8
    assert b.kfd_gpu_count(str(nodes), env={"ROCR_VISIBLE_DEVICES": "4,5,6,7,0,1,2,3"}, dri=str(dri)) == 8
    assert b.kfd_gpu_count(str(nodes), env={"HIP_VISIBLE_DEVICES": "0,2,4,6"}, dri=str(dri)) == 4
    for g in range(8):
        if g != 5:
            (dri / f"renderD{128 + g}").unlink()
    assert b.kfd_gpu_count(str(nodes), env={"HIP_VISIBLE_DEVICES": "0", "ROCR_VISIBLE_DEVICES": "0"},
                           dri=str(dri)) == 1
    # one visible GPU: the 8-rank launch is refused unless it is a shared-GPU rehearsal
    args = types.SimpleNamespace(gpus=8, dry_launch=False, allow_shared_gpu=False)
    orig = b.visible_gpus
    b.visible_gpus = lambda wanted=1: 1
    try:
        assert b.self_launch(args, ["--gpus", "8"]) == 2
    finally:
        b.visible_gpus = orig


def test_stale_shm_cleanup(tmp_path):
    # arrays of a crashed run (older than the launcher) are removed; newer ones and other names are kept
    import time

    b = _bench_module()
    prefix = str(tmp_path / "moc_bench_")
    old = tmp_path / "moc_bench_1234_0_letters"
    new = tmp_path / "moc_bench_5678_0_letters"
    other = tmp_path / "unrelated"
    for p in (old, new, other):
        p.write_bytes(b"x")
    t = time.time()
    os.utime(old, (t - 100, t - 100))
    os.utime(other, (t - 100, t - 100))
    removed = b.cleanup_stale_shm(before=t - 10, prefix=prefix)
    assert removed == [str(old)] and not old.exists() and new.exists() and other.exists()


def test_pci_bus_code_roundtrip():
    b = _bench_module()
    for bus in ("0000:0d:00.0", "0001:8e:1f.7"):
        assert b.pci_bus_id(b.pci_bus_code(bus)) == bus
    assert b.pci_bus_code("") == -1 and b.pci_bus_id(-1) is None


@pytest.mark.parametrize("np_", [1, 2])
def test_final_input6_wall(np_):
    # the BASELINE metric's wall-clock half, reported by every bench run: the reference invocation on
    # input6.txt at the run's rank count, each output checked against the golden
    import bench

    r = bench.final_input6_wall(np_, reps=2)
    if r is None:
        pytest.skip("./final or mpiexec not built here")
    assert r["ok"] and r["np"] == np_ and 0 < r["best_s"] <= r["wall_s"] < 60
