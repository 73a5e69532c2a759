import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "tests", "data")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

MPIEXEC = os.environ.get("MOC_MPIEXEC", "/opt/conda/bin/mpiexec")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


_built = {"done": False}


def source_hash():
    """The hash `make` bakes into libmoc.so and ./final: every file under csrc/ plus the Makefile, sorted."""
    import glob
    import hashlib

    pats = ["csrc/*", "csrc/*/*", "csrc/*/*/*", "csrc/*/*/*/*", "csrc/*/*/*/*/*"]
    files = sorted([f for p in pats for f in glob.glob(p, root_dir=ROOT) if os.path.isfile(os.path.join(ROOT, f))]
                   + ["Makefile"])
    h = hashlib.sha1()
    for f in files:
        with open(os.path.join(ROOT, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:12]


def _products_current():
    """libmoc.so and ./final carry this tree's source hash and the ./final GPU plugin was linked after the
    library: the products of these sources, whatever the object files' state (a gpurun box gets the
    products without build/obj, where `make` would rebuild every object)."""
    lib = os.path.join(ROOT, "mpi_openmp_cuda_amd", "lib", "libmoc.so")
    plugin = os.path.join(ROOT, "mpi_openmp_cuda_amd", "lib", "libmoc_final_gpu.so")
    final = os.path.join(ROOT, "final")
    if not all(os.path.isfile(p) for p in (lib, plugin, final)) or os.path.getmtime(plugin) < os.path.getmtime(lib):
        return False
    tag = ("src=" + source_hash()).encode()
    for p in (lib, final):
        with open(p, "rb") as fh:
            if tag not in fh.read():
                return False
    return True


def ensure_built():
    """Builds libmoc.so and ./final in-tree once per session if they are missing or stale. pytest-xdist
    workers take turns (file lock): concurrent makes would relink ./final under tests that run it."""
    import fcntl

    if _built["done"]:
        return
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    with open(os.path.join(ROOT, "build", ".make.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        if not _products_current():
            subprocess.run(["make", "-C", ROOT, f"-j{min(16, os.cpu_count() or 8)}", "build"], check=True,
                           stdout=subprocess.DEVNULL)
    _built["done"] = True


@pytest.fixture(scope="session", autouse=True)
def _native_build():
    ensure_built()


def input_path(i):
    return os.path.join(DATA, f"input{i}.txt")


def expected(i):
    with open(os.path.join(DATA, "expected", f"input{i}.out")) as f:
        return f.read()


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def run_final(args, stdin_path=None, stdin_bytes=None, np_=1, env=None, timeout=120):
    """Runs ./final under mpiexec (MPICH). Returns CompletedProcess."""
    e = dict(os.environ)
    e.setdefault("OMP_NUM_THREADS", "2")
    if env:
        e.update(env)
    cmd = [MPIEXEC, "-np", str(np_), os.path.join(ROOT, "final")] + list(args)
    data = stdin_bytes
    if stdin_path is not None:
        with open(stdin_path, "rb") as f:
            data = f.read()
    return subprocess.run(cmd, input=data, capture_output=True, timeout=timeout, env=e)
