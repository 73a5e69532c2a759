"""Host sanitizer builds of ./final: ASan/UBSan and TSan (LLVM libomp + Archer) on the
CPU backend, multi-rank (the sliced shm path, mpi transport, the rccl driver over MPI: bulk text batch and
streamed with the print thread), streaming and context-parallel paths — no
reports allowed. ASan runs with LeakSanitizer on: every allocation of a job must be released by exit (the
reference frees nothing, bug B7, main.c:213-240)."""
import os
import subprocess

import pytest

from conftest import MPIEXEC, ROOT, expected, input_path


def _run(binary, args, i, np_, env):
    e = dict(os.environ, OMP_NUM_THREADS="4", **env)
    with open(input_path(i), "rb") as f:
        return subprocess.run([MPIEXEC, "-np", str(np_), os.path.join(ROOT, binary), "--backend=cpu"] + args,
                              stdin=f, capture_output=True, timeout=300, env=e)


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_sanitized_final(kind):
    r = subprocess.run(["make", "-C", ROOT, "-s", kind], capture_output=True, timeout=900)
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    env = {"ASAN_OPTIONS": "detect_leaks=1:halt_on_error=1"} if kind == "asan" else {
        "TSAN_OPTIONS": f"suppressions={ROOT}/tools/tsan.supp halt_on_error=1",
        "OMP_TOOL_LIBRARIES": "/opt/rocm/lib/llvm/lib/libarcher.so"}
    for args, i, np_ in ((["--transport=shm"], 3, 2), (["--transport=shm"], 4, 3),
                         (["--transport=mpi", "--batch-records=2"], 1, 3), (["--partition=offsets"], 4, 2),
                         (["--batch-records=2"], 6, 2), (["--transport=rccl-emul"], 6, 3),
                         (["--transport=rccl-emul", "--batch-records=2"], 3, 2)):
        res = _run(f"final_{kind}", args, i, np_, env)
        err = res.stderr.decode()
        assert res.returncode == 0, err[-3000:]
        assert "ERROR: AddressSanitizer" not in err and "WARNING: ThreadSanitizer" not in err, err[-3000:]
        assert "LeakSanitizer" not in err, err[-3000:]
        assert "runtime error" not in err, err[-3000:]
        assert res.stdout.decode() == expected(i)
