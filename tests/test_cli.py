"""CLI behaviour: determinism, semantics flag, error handling, fault injection (no hangs: every run is
bounded by a timeout), input edge cases through ./final."""
import json
import re
import subprocess
import numpy as np

import pytest

from conftest import expected, input_path, run_final


@pytest.mark.parametrize("threads", ["1", "3", "8"])
def test_deterministic_over_threads(threads):
    # reference bug B2: parallel fscanf permutes rows with > 1 OpenMP thread
    r = run_final(["--backend=cpu"], stdin_path=input_path(1), np_=2, env={"OMP_NUM_THREADS": threads})
    assert r.stdout.decode() == expected(1)


def test_help_and_unknown_flag():
    r = run_final(["--help"], stdin_bytes=b"")
    assert r.returncode == 0 and b"usage" in r.stdout
    r = run_final(["--bogus=1"], stdin_bytes=b"")
    assert r.returncode == 2 and b"unknown flag" in r.stderr


def test_env_flag_override():
    r = run_final([], stdin_path=input_path(6), np_=2, env={"MOC_BACKEND": "cpu", "MOC_TRANSPORT": "mpi"})
    assert r.returncode == 0 and r.stdout.decode() == expected(6)


def test_spec_semantics_flag():
    text = b"10 2 3 4\nABCDEFGH\n1\nFGH\n"
    ref = run_final(["--backend=cpu"], stdin_bytes=text)
    spec = run_final(["--backend=cpu", "--semantics=spec"], stdin_bytes=text)
    assert ref.stdout == b"#0: score: 16, n: 4, k: 1\n"
    assert spec.stdout == b"#0: score: 30, n: 5, k: 0\n"


def test_parse_error_exit_code():
    r = run_final(["--backend=cpu"], stdin_bytes=b"1 2 3 4\nAB1\n1\nA\n", np_=3)
    assert r.returncode == 1
    assert b"non-letter" in r.stderr and r.stdout == b""


def test_edge_records_through_cli():
    text = b"1 1 1 1\nABCD\n4\nABCD\nABCDE\nA\nDCBA\n"
    r = run_final(["--backend=cpu"], stdin_bytes=text, np_=3)
    lines = r.stdout.decode().splitlines()
    assert lines[0] == "#0: score: 4, n: 0, k: 0"
    assert lines[1] == "#1: score: -2147483648, n: 0, k: 0"
    assert len(lines) == 4


def test_zero_records():
    r = run_final(["--backend=cpu"], stdin_bytes=b"1 1 1 1\nABCD\n0\n", np_=2)
    assert r.returncode == 0 and r.stdout == b""


@pytest.mark.parametrize("phase", ["parse", "bcast", "distribute", "compute", "gather"])
@pytest.mark.parametrize("rank", [0, 1])
def test_fault_injection_aborts_cleanly(phase, rank):
    # reference bug B11: exit(1) on one rank without MPI_Abort leaves the peers blocked forever
    if phase == "parse" and rank == 1:
        pytest.skip("only the root parses")
    try:
        r = run_final(["--backend=cpu", f"--inject-fault={phase}:{rank}"], stdin_path=input_path(3), np_=2,
                      timeout=60)
    except subprocess.TimeoutExpired:
        pytest.fail("fault did not abort the job (hang)")
    assert r.returncode != 0
    assert b"injected fault" in r.stderr or phase == "parse"


# ---- comm deadline: a rank that is alive but stuck ends the job with a diagnosis

@pytest.mark.parametrize("transport,flags,phase,rank", [
    ("rccl-emul", [], "distribute", 2),          # the device batch driver over MPI point-to-point
    ("rccl-emul", ["--batch-records=7"], "compute", 1),  # streamed device batches
    ("rccl-emul", ["--partition=offsets"], "compute", 2),  # context parallel: bcast + MAX all-reduce
    ("mpi", [], "compute", 1),                    # Scatterv / Gatherv flow
    ("shm", [], "compute", 2),                    # node-shared slices: host-table collectives
])
def test_comm_timeout_names_stuck_rank(transport, flags, phase, rank):
    import time

    # reference: a failing rank exit(1)s without MPI_Abort and its peers hang in the next collective
    # (/root/reference/cudaFunctions.cu:15-33, main.c:174,195-197); here a stalled rank (MOC_STALL_S: long
    # enough that only the deadline can end the job) is caught by its peers' deadline-polled waits
    t0 = time.time()
    try:
        r = run_final(["--backend=cpu", f"--transport={transport}", "--comm-timeout=2",
                       f"--inject-fault=stall:{phase}:{rank}", *flags], stdin_path=input_path(3), np_=3,
                      env={"MOC_STALL_S": "60"}, timeout=45)
    except subprocess.TimeoutExpired:
        pytest.fail("a stalled rank hung the job past its comm deadline")
    err = r.stderr.decode()
    assert r.returncode != 0, err
    assert time.time() - t0 < 30
    assert "injected rank stall" in err
    fatal = [l for l in err.splitlines() if "fatal: comm timeout" in l]
    assert fatal, err[-2000:]
    # a peer names the phase it waited in; when the wait was point-to-point, the stalled rank too
    assert all(re.search(r"in phase '\w+'", l) for l in fatal), fatal
    if transport in ("rccl-emul", "mpi") and not flags:
        assert any(f"rank {rank}" in l.split("outstanding:")[-1] for l in fatal), fatal


def test_comm_timeout_flag_in_help_and_default_jobs_unaffected():
    r = run_final(["--help"], stdin_bytes=b"")
    assert b"--comm-timeout" in r.stdout
    # a tiny deadline does not fire on a healthy job (waits that complete never see it)
    r = run_final(["--backend=cpu", "--transport=rccl-emul", "--comm-timeout=5"], stdin_path=input_path(3), np_=3)
    assert r.returncode == 0 and r.stdout.decode() == expected(3)


def test_timing_json():
    import json

    r = run_final(["--backend=cpu", "--timing"], stdin_path=input_path(4), np_=2)
    line = [l for l in r.stderr.decode().splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["records"] == 30 and d["ranks"] == 2 and "compute_ms" in d["timing"]


# ---- decomposition / streaming / resume

@pytest.mark.parametrize("i", [1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("transport", ["shm", "mpi"])
@pytest.mark.parametrize("np_", [1, 3])
def test_offsets_partition(i, transport, np_):
    # context parallel: every rank searches a share of every record's offsets, MAX-all-reduce of keys
    r = run_final(["--backend=cpu", "--partition=offsets", f"--transport={transport}"], stdin_path=input_path(i),
                  np_=np_)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == expected(i)


@pytest.mark.parametrize("batch", ["--batch-records=1", "--batch-records=4", "--batch-chars=30"])
@pytest.mark.parametrize("partition", ["cost", "offsets"])
def test_streaming_batches(batch, partition):
    for i in (1, 3, 6):
        r = run_final(["--backend=cpu", batch, f"--partition={partition}"], stdin_path=input_path(i), np_=2)
        assert r.returncode == 0, r.stderr.decode()
        assert r.stdout.decode() == expected(i)


@pytest.mark.parametrize("extra", [[], ["--batch-records=3"]])
def test_skip_records_resume(extra):
    exp = expected(1).splitlines(keepends=True)
    r = run_final(["--backend=cpu", "--skip-records=4"] + extra, stdin_path=input_path(1), np_=2)
    assert r.returncode == 0 and r.stdout.decode() == "".join(exp[4:])
    r = run_final(["--backend=cpu", "--skip-records=99"] + extra, stdin_path=input_path(1), np_=2)
    assert r.returncode == 0 and r.stdout == b""


def test_input_flag_large_file(tmp_path):
    # MPICH's hydra cannot forward a large stdin here ("reading stdin too slowly"); --input reads the file
    from mpi_openmp_cuda_amd import format_results, make_synthetic, search_cpu

    prob = make_synthetic("input6", 60000, seed=4)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    want = format_results(search_cpu(prob))
    for extra in ([], ["--batch-records=7000"], ["--partition=offsets"]):
        r = run_final(["--backend=cpu", f"--input={path}"] + extra, stdin_bytes=b"", np_=3)
        assert r.returncode == 0, r.stderr.decode()
        assert r.stdout.decode() == want



def test_gpu_prewarm_hint(tmp_path):
    # --gpu-prewarm-bytes: every rank starts the HIP runtime on a helper thread during the parse; with no
    # usable GPU (or an auto backend that then picks the OpenMP engine) the output is unchanged
    from mpi_openmp_cuda_amd import format_results, make_synthetic, search_cpu

    prob = make_synthetic("input6", 20000, seed=5)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    want = format_results(search_cpu(prob))
    for extra in ([f"--input={path}"], ["--batch-records=3000", f"--input={path}"]):
        r = run_final(["--gpu-prewarm-bytes=1", "--gpu-min-cells=1000000000000"] + extra, stdin_bytes=b"", np_=2)
        assert r.returncode == 0, r.stderr.decode()
        assert r.stdout.decode() == want
    # the hint from a redirected stdin (a regular file; singleton start, as mpiexec's proxy forwards a pipe)
    import os

    from conftest import ROOT

    with open(path, "rb") as f:
        r = subprocess.run([os.path.join(ROOT, "final"), "--gpu-prewarm-bytes=1", "--gpu-min-cells=1000000000000"],
                           stdin=f, capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == want

@pytest.mark.parametrize("mode", ["w", "a"])
def test_output_to_regular_file(tmp_path, mode):
    # stdout a regular file: the writer's parallel pwrite path (at the current offset, after text already
    # in the file) — or, opened O_APPEND (`>>`), the ordered path; both must give the rows in order
    import os

    from conftest import ROOT
    from mpi_openmp_cuda_amd import format_results, make_synthetic, search_cpu

    prob = make_synthetic("input6", 140000, seed=9)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    want = format_results(search_cpu(prob))
    out = tmp_path / "out.txt"
    out.write_text("previous line\n")
    with open(out, mode) as f:
        if mode == "w":
            f.write("header\n")
            f.flush()
        env = dict(os.environ, OMP_NUM_THREADS="4")
        # singleton MPI start (no mpiexec: its proxies would turn stdout into a pipe)
        r = subprocess.run([os.path.join(ROOT, "final"), "--backend=cpu", f"--input={path}"],
                           stdin=subprocess.DEVNULL, stdout=f, stderr=subprocess.PIPE, env=env, timeout=120)
    assert r.returncode == 0, r.stderr.decode()
    prefix = "header\n" if mode == "w" else "previous line\n"
    assert out.read_text() == prefix + want
    # --output: the root writes the file itself, also under mpiexec
    out2 = tmp_path / "out2.txt"
    # an existing longer file is overwritten and cut to the new length (opened without O_TRUNC)
    out2.write_text("stale\n" * (len(want) // 3 + 100))
    r = run_final(["--backend=cpu", f"--input={path}", f"--output={out2}"], stdin_bytes=b"", np_=2,
                  env={"OMP_NUM_THREADS": "4"})
    assert r.returncode == 0 and r.stdout == b"", r.stderr.decode()
    assert out2.read_text() == want


def test_streaming_parse_error_mid_stream():
    text = b"1 2 3 4\nABCDEFG\n5\nABC\nABD\nAB1\nAC\nAD\n"
    r = run_final(["--backend=cpu", "--batch-records=2"], stdin_bytes=text, np_=2)
    assert r.returncode == 1 and b"non-letter" in r.stderr
    # the batch before the bad record was already printed (a resume restarts at --skip-records=2)
    assert [l.split(":")[0] for l in r.stdout.decode().splitlines()] == ["#0", "#1"]


def test_length_limit_flags():
    text = b"1 1 1 1\nABCDEFG\n2\nABC\nABCDE\n"
    r = run_final(["--backend=cpu", "--max-l2=4"], stdin_bytes=text)
    assert r.returncode == 1 and b"limit is 4" in r.stderr
    r = run_final(["--backend=cpu", "--max-l1=6"], stdin_bytes=text)
    assert r.returncode == 1 and b"limit is 6" in r.stderr
    r = run_final(["--backend=cpu", "--max-l2=5", "--batch-records=1"], stdin_bytes=text)
    assert r.returncode == 0 and len(r.stdout.splitlines()) == 2


def test_timing_json_has_throughput():
    import json

    r = run_final(["--backend=cpu", "--timing", "--batch-records=3"], stdin_path=input_path(1), np_=2)
    t = json.loads(r.stderr.decode().strip().splitlines()[-1])
    assert t["records"] == 10 and t["batches"] == 4 and t["cells"] > 0 and t["cells_per_s"] > 0
    # the node's streaming flow: root cuts (count), every rank encodes its slice (fill), search, gather, print
    assert set(t["timing"]) >= {"parse_ms", "bcast_ms", "count_ms", "fill_ms", "compute_ms", "gather_ms", "print_ms"}
    assert t["rank_records"] and sum(t["rank_records"]) == 10


def test_cmake_build_matches(tmp_path):
    # the CMake build produces a working ./final and libmoc.so
    import shutil

    if not shutil.which("cmake") or not shutil.which("ninja"):
        pytest.skip("cmake/ninja not available")
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    bdir = tmp_path / "cm"
    r = subprocess.run(["cmake", "-S", root, "-B", str(bdir), "-G", "Ninja"], capture_output=True, timeout=300)
    assert r.returncode == 0, r.stderr.decode()[-2000:]
    r = subprocess.run(["cmake", "--build", str(bdir), "-j", "8", "--target", "final"], capture_output=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout.decode()[-2000:]
    from conftest import MPIEXEC

    with open(input_path(4), "rb") as f:
        out = subprocess.run([MPIEXEC, "-np", "2", str(bdir / "final"), "--backend=cpu"], input=f.read(),
                             capture_output=True, timeout=120)
    assert out.returncode == 0 and out.stdout.decode() == expected(4)


@pytest.mark.parametrize("transport", ["shm", "mpi"])
@pytest.mark.parametrize("np_", [1, 3])
def test_record_error_after_header(transport, np_):
    # with the shm transport the records are encoded straight into the shared window after the header
    # went out; a bad record must still end every rank with exit code 1 and the record's index
    text = b"1 2 3 4\nABCDEFG\n4\nABC\nABD\nAB1\nAC\n"
    r = run_final(["--backend=cpu", f"--transport={transport}"], stdin_bytes=text, np_=np_)
    assert r.returncode == 1, r.stderr.decode()
    assert b"record #2" in r.stderr and r.stdout == b""
    ok = b"1 2 3 4\nABCDEFG\n3\nAB\nABCD\nAC\n"
    r = run_final(["--backend=cpu", f"--transport={transport}", "--max-l2=2"], stdin_bytes=ok, np_=np_)
    assert r.returncode == 1 and b"record #1 has 4 letters, limit is 2" in r.stderr


def test_large_file_parallel_read(tmp_path):
    # an input file over 64 MiB is read with parallel preads into a huge-page buffer: the bulk path must
    # agree with the streaming reader (an independent tokeniser) line for line
    import os
    import sys

    from conftest import ROOT

    path = tmp_path / "big.txt"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_synthetic.py"), "--shape", "input6",
                    "--records", "7500000", "--seed", "11", "--out", str(path)], check=True, timeout=300,
                   capture_output=True)
    assert path.stat().st_size > (64 << 20)
    outs = []
    for extra in ([], ["--batch-records=2000000"]):
        out = tmp_path / f"out{len(outs)}.txt"
        r = run_final(["--backend=cpu", f"--input={path}", f"--output={out}"] + extra, stdin_bytes=b"", np_=1,
                      timeout=300)
        assert r.returncode == 0, r.stderr.decode()
        outs.append(out.read_bytes())
    assert outs[0] == outs[1]
    assert outs[0].count(b"\n") == 7500000


def test_pipe_output_double_buffered(tmp_path):
    # stdout a pipe (mpiexec's proxy) with more rows than one block (64 K rows per thread): the blocks go
    # out through the background writer, double-buffered against the formatting — order must hold, and the
    # bytes must equal the pwrite path's and the Python formatter's
    from mpi_openmp_cuda_amd import format_results, make_synthetic, search_cpu

    prob = make_synthetic("input6", 700000, seed=13)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    want = format_results(search_cpu(prob)).encode()
    r = run_final(["--backend=cpu", f"--input={path}"], stdin_bytes=b"", np_=1, env={"OMP_NUM_THREADS": "2"},
                  timeout=300)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout == want
    out = tmp_path / "out.txt"
    r = run_final(["--backend=cpu", f"--input={path}", f"--output={out}"], stdin_bytes=b"", np_=1,
                  env={"OMP_NUM_THREADS": "2"}, timeout=300)
    assert r.returncode == 0, r.stderr.decode()
    assert out.read_bytes() == want


@pytest.mark.parametrize("omp_env", [{"OMP_DYNAMIC": "true", "OMP_NUM_THREADS": "8"},
                                     {"OMP_THREAD_LIMIT": "2", "OMP_NUM_THREADS": "6"}])
def test_fewer_omp_threads_than_requested(tmp_path, omp_env):
    # parser passes, formatter and pwrite writer iterate over parts, not thread ids: a runtime that delivers
    # fewer threads than asked (OMP_DYNAMIC, OMP_THREAD_LIMIT) must still process every part
    from mpi_openmp_cuda_amd import format_results, make_synthetic, search_cpu

    prob = make_synthetic("input6", 150000, seed=12)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    want = format_results(search_cpu(prob))
    out = tmp_path / "out.txt"
    for extra in ([], [f"--output={out}"], ["--batch-records=40000"]):
        r = run_final(["--backend=cpu", f"--input={path}"] + extra, stdin_bytes=b"", np_=2, env=omp_env)
        assert r.returncode == 0, r.stderr.decode()
        got = out.read_text() if extra and extra[0].startswith("--output") else r.stdout.decode()
        assert got == want


def _source_hash():
    """The hash `make` bakes into ./final (conftest.source_hash)."""
    from conftest import source_hash

    return source_hash()


def test_build_id_matches_sources():
    # a prebuilt ./final shipped next to newer sources would print another source hash
    r = run_final(["--help"], np_=1)
    line = [l for l in r.stdout.decode().splitlines() if l.startswith("build:")][-1]
    assert f"src={_source_hash()}" in line, line


def test_library_is_the_product_build():
    # the loaded libmoc.so was built from these sources with no extra kernel defines (a `make variant` or
    # `make debug-kernels` library reports its defines and is refused by the loader)
    from mpi_openmp_cuda_amd import _lib

    info = _lib.build_info()
    assert info == {"src": _source_hash(), "defs": ""}, info


def test_variant_library_is_refused(tmp_path):
    # a library whose kernel objects carry defines must not stand in for the product: the loader refuses it
    # unless MOC_ALLOW_VARIANT_LIB=1 (built here as a one-file stand-in exporting moc_build_info)
    import os
    import sys

    from conftest import ROOT

    src = tmp_path / "v.c"
    src.write_text('const char* moc_build_info(void) { return "src=x defs=-DMOC_T16_UNROLL=8"; }\n'
                   'const char* moc_last_error(void) { return ""; }\n')
    so = tmp_path / "libv.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    code = ("import os, sys; sys.path.insert(0, %r)\n"
            "from mpi_openmp_cuda_amd import _lib\n"
            "try:\n    _lib.lib()\nexcept _lib.NativeError as e:\n    print('refused', e)\n"
            "else:\n    print('loaded', _lib.build_info())\n") % ROOT
    env = dict(os.environ, MOC_LIB_PATH=str(so))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.stdout.startswith("refused") and "MOC_T16_UNROLL" in r.stdout, (r.stdout, r.stderr)
    env["MOC_ALLOW_VARIANT_LIB"] = "1"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.stdout.startswith("loaded") and "-DMOC_T16_UNROLL=8" in r.stdout, (r.stdout, r.stderr)


@pytest.mark.parametrize("np_", [2, 3, 8])
@pytest.mark.parametrize("i", [1, 3, 4])
def test_sliced_bounds_and_timing(np_, i):
    # bulk shm jobs are "sliced": each rank encodes its own record slice from the shared text; the slices
    # tile the job in order, CPU ranks pin nothing, and the bounds equal the lengths-based cost split
    import json

    import numpy as np

    from mpi_openmp_cuda_amd import Problem
    from mpi_openmp_cuda_amd.parallel.partition import CPU_COST, partition

    r = run_final(["--backend=cpu", "--timing"], stdin_path=input_path(i), np_=np_)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == expected(i)
    d = json.loads([l for l in r.stderr.decode().splitlines() if l.startswith("{")][-1])
    assert d["sliced"] is True and d["transport"] == "shm"
    prob = Problem.read(input_path(i))
    assert sum(d["rank_records"]) == prob.n and d["elements"] == int(prob.offsets[-1])
    assert d["rank_pinned_bytes"] == [0] * np_ and d["rank_h2d_bytes"] == [0] * np_
    want = np.diff(partition(np.diff(prob.offsets), len(prob.seq1), np_, CPU_COST))
    assert d["rank_records"] == [int(x) for x in want]


# ---- the rccl transport's batch driver, run over the MPI-emulated device layer (no GPU needed)

@pytest.mark.parametrize("np_", [1, 2, 3, 8])
@pytest.mark.parametrize("partition", ["cost", "offsets"])
def test_rccl_driver_emulated(np_, partition):
    # same device_batch code as --transport=rccl: per-rank wire plans (3/4/8-bit narrow forms and the dense
    # form), chunked pipelined sends (tiny chunks force many pieces), narrow-result gather, CP MAX reduce
    for i in (1, 3, 4, 6):
        r = run_final(["--backend=cpu", "--transport=rccl-emul", f"--partition={partition}"], stdin_path=input_path(i),
                      np_=np_, env={"MOC_SEND_CHUNK": "4096"})
        assert r.returncode == 0, r.stderr.decode()
        assert r.stdout.decode() == expected(i), (i, np_, partition)


@pytest.mark.parametrize("np_", [1, 3, 8])
@pytest.mark.parametrize("stream", [False, True])
def test_rccl_transport_timing_fields(np_, stream):
    # --timing on the device transport reports what a first multi-GPU run needs: the communicator's set-up,
    # the bytes each rank put on the comm, the root's bytes to each peer and its per-peer rate
    import json

    extra = ["--batch-records=8"] if stream else []
    r = run_final(["--backend=cpu", "--transport=rccl-emul", "--timing"] + extra, stdin_path=input_path(3), np_=np_,
                  env={"MOC_SEND_CHUNK": "4096"})
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == expected(3)
    d = json.loads([l for l in r.stderr.decode().splitlines() if l.startswith("{")][-1])
    for k in ("rccl_comm_init_ms", "rccl_comm_wait_ms", "distribute_ms", "rank_sent_bytes", "peer_sent_bytes",
              "peer_distribute_gbps"):
        assert k in d, (k, d)
    assert len(d["rank_sent_bytes"]) == np_ and len(d["peer_sent_bytes"]) == np_ == len(d["peer_distribute_gbps"])
    assert d["peer_sent_bytes"][0] == 0  # the root's own slice never crosses the comm
    assert d["rank_sent_bytes"][0] == sum(d["peer_sent_bytes"])  # the root sends exactly what its peers get
    if np_ > 1:
        assert all(b > 0 for b in d["peer_sent_bytes"][1:]) and d["distribute_ms"] > 0
        assert all(b > 0 for b in d["rank_sent_bytes"][1:])  # every peer sends its results back
        assert all(g > 0 for g in d["peer_distribute_gbps"][1:])
    # the root encodes (and uploads) its own slice first, then the peers' in rank order: its search waits for
    # no encode of its own behind the last peer's pieces (device_batch.cpp, device_batch_text)
    assert d["fill_order"] == list(range(np_))


@pytest.mark.parametrize("np_", [2, 3])
def test_rccl_driver_emulated_streaming_and_synthetic(np_, tmp_path):
    # streaming batches through the device driver, and a larger mixed-length synthetic input
    from mpi_openmp_cuda_amd import format_results, search_cpu
    from mpi_openmp_cuda_amd.utils.synthetic import make_synthetic

    for i in (1, 3):
        r = run_final(["--backend=cpu", "--transport=rccl-emul", "--batch-records=4"], stdin_path=input_path(i), np_=np_)
        assert r.returncode == 0, r.stderr.decode()
        assert r.stdout.decode() == expected(i)
    prob = make_synthetic("input6", 20_000, seed=5)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    r = run_final(["--backend=cpu", "--transport=rccl-emul", f"--input={path}", "--timing"], stdin_bytes=b"", np_=np_,
                  env={"MOC_SEND_CHUNK": "65536"})
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == format_results(search_cpu(prob))


@pytest.mark.parametrize("np_", [2, 3, 8])
@pytest.mark.parametrize("i", [2, 3, 6])
def test_distributed_print_to_output_file(tmp_path, np_, i):
    # --parallel-print, several ranks + --output: every rank writes its own rows at its offset of the file (sizes all-gathered);
    # ranks without records (input2 has one) write nothing, a longer old file is cut to the new length
    out = tmp_path / "out.txt"
    out.write_text("x" * 100000)
    r = run_final(["--backend=cpu", f"--input={input_path(i)}", f"--output={out}", "--parallel-print"], stdin_bytes=b"",
                  np_=np_)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout == b"" and out.read_text() == expected(i)


# ---- the node's streaming flow (csrc/apps/flow_stream.cpp): batches cut by the root, every rank encoding its
# slice into its ring slot, printed while the next batch is searched

@pytest.mark.parametrize("np_", [1, 3, 8])
@pytest.mark.parametrize("mode", ["stdin", "input"])
def test_streaming_goldens_every_rank_count(np_, mode):
    # stdin: the root's stream buffer (copied into node-shared text slots at np > 1); input: every rank maps
    # the file. Batches of 2 / 3 records and of 40 letters, more ranks than records included.
    for i in range(1, 7):
        for b in ("--batch-records=2", "--batch-records=3", "--batch-chars=40"):
            args = ["--backend=cpu", b]
            if mode == "input":
                r = run_final(args + [f"--input={input_path(i)}"], stdin_bytes=b"", np_=np_)
            else:
                r = run_final(args, stdin_path=input_path(i), np_=np_)
            assert r.returncode == 0, (i, b, r.stderr.decode())
            assert r.stdout.decode() == expected(i), (i, b)


def test_streaming_pipe_large_singleton(tmp_path):
    # a stream (pipe) larger than the root's first probe and read buffer: many count extensions, buffer
    # compaction past the consumed batches, records cut by letters too; the same bytes as the bulk path
    import os

    from conftest import ROOT
    from mpi_openmp_cuda_amd import format_results, make_synthetic, search_cpu

    prob = make_synthetic("input6", 1_300_000, seed=21)
    text = prob.to_text().encode()
    path = tmp_path / "in.txt"
    path.write_bytes(text)
    want = format_results(search_cpu(prob)).encode()
    env = dict(os.environ, OMP_NUM_THREADS="4")
    for extra in (["--batch-records=100000"], ["--batch-chars=700000"], ["--batch-records=250000", "--skip-records=123457"]):
        r = subprocess.run([os.path.join(ROOT, "final"), "--backend=cpu"] + extra, input=text, capture_output=True,
                           timeout=300, env=env)
        assert r.returncode == 0, r.stderr.decode()
        if "--skip-records=123457" in extra:
            assert r.stdout == b"".join(want.splitlines(keepends=True)[123457:])
        else:
            assert r.stdout == want, extra
    # mapped (--input) at two ranks, batches cut mid-chunk
    r = run_final(["--backend=cpu", f"--input={path}", "--batch-records=333333"], stdin_bytes=b"", np_=2, timeout=300)
    assert r.returncode == 0 and r.stdout == want


def test_streaming_short_input_and_bad_record():
    # fewer records than announced: the batches before are printed, then the error, exit code 1
    r = run_final(["--backend=cpu", "--batch-records=2"], stdin_bytes=b"1 2 3 4\nABCDEFG\n5\nABC\nABD\nAC\n", np_=2)
    assert r.returncode == 1 and b"expected 5 Seq2 records, found only 3" in r.stderr
    assert r.stdout.decode().count("\n") == 2
    r = run_final(["--backend=cpu", "--batch-records=2"], stdin_bytes=b"1 2 3 4\nABCDEFG\n4\nABC\nABD\nA1\nAC\n",
                  np_=3)
    assert r.returncode == 1 and b"record #2 contains a non-letter" in r.stderr
    assert r.stdout.decode().count("\n") == 2


@pytest.mark.parametrize("np_", [2, 3, 8])
def test_rccl_driver_emulated_many_pieces(np_, tmp_path):
    # the root's piece pipeline (device_batch.cpp): every rank's block cut into 2640-byte pieces (P33 blocks,
    # 5-bit groups and offsets never straddle two), interleaved round-robin with the root's own, three
    # staging slots reused — narrow form (input6 shape) and dense form (input3 shape: records over 255)
    from mpi_openmp_cuda_amd import format_results, search_cpu
    from mpi_openmp_cuda_amd.utils.synthetic import make_synthetic

    for shape, n in (("input6", 20_000), ("input3", 300)):
        prob = make_synthetic(shape, n, seed=17)
        path = tmp_path / f"{shape}.txt"
        path.write_text(prob.to_text())
        r = run_final(["--backend=cpu", "--transport=rccl-emul", f"--input={path}"], stdin_bytes=b"", np_=np_,
                      env={"MOC_SEND_CHUNK": "5000"}, timeout=300)
        assert r.returncode == 0, r.stderr.decode()
        assert r.stdout.decode() == format_results(search_cpu(prob)), shape


def test_rccl_driver_pieces_smaller_than_a_record(tmp_path):
    # 8 ranks, records of 9-20 K letters (5-bit dense form: 5.6-12.5 KB each) cut into 2640-byte pieces: a
    # record spans several pieces, which arrive interleaved with the other ranks' — bulk and streamed
    from mpi_openmp_cuda_amd import Problem, format_results, search_cpu

    rng = np.random.default_rng(41)
    s1 = "".join(chr(65 + x) for x in rng.integers(0, 26, 21_000))
    recs = ["".join(chr(65 + x) for x in rng.integers(0, 26, int(n))) for n in rng.integers(9_000, 20_001, 12)]
    prob = Problem.from_strings([3, 1, 2, 1], s1, recs)
    path = tmp_path / "long.txt"
    path.write_text(prob.to_text())
    want = format_results(search_cpu(prob))
    for extra in ([], ["--batch-records=5"]):
        r = run_final(["--backend=cpu", "--transport=rccl-emul", f"--input={path}"] + extra, stdin_bytes=b"", np_=8,
                      env={"MOC_SEND_CHUNK": "2640"}, timeout=300)
        assert r.returncode == 0, (extra, r.stderr.decode())
        assert r.stdout.decode() == want, extra


@pytest.mark.parametrize("fault", ["distribute:3", "compute:5", "gather:7", "distribute:0"])
@pytest.mark.parametrize("mode", ["bulk", "streamed"])
def test_rccl_driver_fault_at_np8(tmp_path, fault, mode):
    # a rank failing inside the rccl transport's driver (device_batch_text / the streamed device flow) at
    # 8 ranks: the whole job aborts with the message, no rank hangs in a collective (reference bug B11)
    from mpi_openmp_cuda_amd.utils.synthetic import make_synthetic

    prob = make_synthetic("input6", 20_000, seed=5)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    args = ["--backend=cpu", "--transport=rccl-emul", f"--input={path}", f"--inject-fault={fault}"]
    if mode == "streamed":
        args.append("--batch-records=3000")
    try:
        r = run_final(args, stdin_bytes=b"", np_=8, env={"MOC_SEND_CHUNK": "2640"}, timeout=120)
    except subprocess.TimeoutExpired:
        pytest.fail(f"fault {fault} did not abort the job (hang)")
    assert r.returncode != 0
    assert b"injected fault" in r.stderr, r.stderr.decode()[-2000:]


# ---- bulk jobs off the shm transport start from the text (run_text_batch / device_batch_text): the root
# counts, splits and encodes every rank's slice straight into its wire block; mpi encodes one byte batch

@pytest.mark.parametrize("np_", [1, 2, 3, 8])
def test_text_batch_transports_goldens(np_):
    for tr in ("--transport=rccl-emul", "--transport=mpi"):
        for part in ("--partition=cost", "--partition=even"):
            for i in range(1, 7):
                r = run_final(["--backend=cpu", tr, part], stdin_path=input_path(i), np_=np_,
                              env={"MOC_SEND_CHUNK": "2640"})
                assert r.returncode == 0, (tr, part, i, r.stderr.decode())
                assert r.stdout.decode() == expected(i), (tr, part, i)


@pytest.mark.parametrize("np_", [2, 3])
def test_text_batch_skip_and_errors(np_, tmp_path):
    # --skip-records through the text path; an input error in a later rank's slice (found after earlier
    # slices were sent) reaches every rank: the sequential reader's first error, exit code 1, nothing printed
    for tr in ("--transport=rccl-emul", "--transport=mpi"):
        r = run_final(["--backend=cpu", tr, "--skip-records=2"], stdin_path=input_path(6), np_=np_)
        assert r.returncode == 0, r.stderr.decode()
        assert r.stdout.decode() == "".join(expected(6).splitlines(keepends=True)[2:])
        recs = ["ABCDEFGH"] * 40
        recs[31] = "ABC1DEF"
        recs[35] = "A" * 3001
        text = "1 2 3 4\nABCDEFGHIJ\n40\n" + "\n".join(recs) + "\n"
        r = run_final(["--backend=cpu", tr], stdin_bytes=text.encode(), np_=np_)
        assert r.returncode == 1 and b"record #31 contains a non-letter" in r.stderr, r.stderr.decode()
        assert r.stdout == b""
        r = run_final(["--backend=cpu", tr], stdin_bytes=b"1 2 3 4\nABCDEFGHIJ\n40\nABC\nABD\n", np_=np_)
        assert r.returncode == 1 and b"expected 40 Seq2 records, found only 2" in r.stderr, r.stderr.decode()


def test_text_batch_timing_phases(tmp_path):
    import json

    from mpi_openmp_cuda_amd.utils.synthetic import make_synthetic

    prob = make_synthetic("input6", 30_000, seed=9)
    path = tmp_path / "in.txt"
    path.write_text(prob.to_text())
    r = run_final(["--backend=cpu", "--transport=rccl-emul", f"--input={path}", "--timing"], stdin_bytes=b"", np_=3,
                  env={"MOC_SEND_CHUNK": "65536"})
    assert r.returncode == 0, r.stderr.decode()
    d = json.loads([ln for ln in r.stderr.decode().splitlines() if ln.startswith("{")][-1])
    for ph in ("count", "fill", "distribute", "compute", "gather", "print"):
        assert ph + "_ms" in d["timing"], (ph, d["timing"])
    assert "parse_ms" in d["timing"] and d["timing"]["parse_ms"] < 1000
    assert sum(d["rank_records"]) == prob.n and d["elements"] == int(prob.offsets[-1]) and d["records"] == prob.n


# ---- streamed jobs off the shm transport (flow_device_stream.cpp): the root cuts the batches from the text
# (pass 1 kept past each cut), device transports encode the ranks' slices straight into their wire blocks,
# batch b prints while batch b+1 runs; mpi scatters byte-code batches

@pytest.mark.parametrize("np_", [1, 3, 8])
@pytest.mark.parametrize("tr", ["rccl-emul", "mpi"])
def test_device_streaming_goldens(np_, tr):
    for i in range(1, 7):
        for b in ("--batch-records=2", "--batch-records=3", "--batch-chars=40"):
            for mode in ("stdin", "input"):
                args = ["--backend=cpu", f"--transport={tr}", b]
                if mode == "input":
                    r = run_final(args + [f"--input={input_path(i)}"], stdin_bytes=b"", np_=np_,
                                  env={"MOC_SEND_CHUNK": "2640"})
                else:
                    r = run_final(args, stdin_path=input_path(i), np_=np_, env={"MOC_SEND_CHUNK": "2640"})
                assert r.returncode == 0, (i, b, mode, r.stderr.decode())
                assert r.stdout.decode() == expected(i), (i, b, mode)


@pytest.mark.parametrize("tr", ["rccl-emul", "mpi"])
def test_device_streaming_large_skip_errors(tr, tmp_path):
    import json
    import os

    from conftest import ROOT

    from mpi_openmp_cuda_amd import format_results, make_synthetic, search_cpu

    prob = make_synthetic("input6", 300_000, seed=23)
    text = prob.to_text().encode()
    path = tmp_path / "in.txt"
    path.write_bytes(text)
    want = format_results(search_cpu(prob)).encode()
    lines = want.splitlines(keepends=True)
    for extra, np_ in ((["--batch-records=70000", "--timing"], 2), (["--batch-chars=500000"], 3),
                       (["--batch-records=50000", "--skip-records=123457"], 2)):
        for src in ("stdin", "input"):
            args = ["--backend=cpu", f"--transport={tr}"] + extra
            if src == "input":
                r = run_final(args + [f"--input={path}"], stdin_bytes=b"", np_=np_, timeout=300)
            else:  # one singleton rank: mpiexec's stdin forwarding aborts on MBs of input at np > 1
                r = subprocess.run([os.path.join(ROOT, "final")] + args, input=text, capture_output=True, timeout=300)
            assert r.returncode == 0, (extra, src, r.stderr.decode())
            assert r.stdout == (b"".join(lines[123457:]) if "--skip-records=123457" in extra else want), (extra, src)
            if "--timing" in extra:
                d = json.loads([ln for ln in r.stderr.decode().splitlines() if ln.startswith("{")][-1])
                assert d["batches"] == 5 and d["records"] == prob.n and d["elements"] == int(prob.offsets[-1])
                if tr != "mpi":
                    assert sum(d["rank_records"]) == prob.n
    # a bad record in the third batch: the first two batches print, then the error
    recs = ["ABCDEFGH"] * 12
    recs[9] = "ABC1DEF"
    bad = ("1 2 3 4\nABCDEFGHIJ\n12\n" + "\n".join(recs) + "\n").encode()
    r = run_final(["--backend=cpu", f"--transport={tr}", "--batch-records=4"], stdin_bytes=bad, np_=3)
    assert r.returncode == 1 and b"record #9 contains a non-letter" in r.stderr, r.stderr.decode()
    assert r.stdout.decode().count("\n") == 8
    r = run_final(["--backend=cpu", f"--transport={tr}", "--batch-records=2"],
                  stdin_bytes=b"1 2 3 4\nABCDEFG\n5\nABC\nABD\nAC\n", np_=2)
    assert r.returncode == 1 and b"expected 5 Seq2 records, found only 3" in r.stderr
    assert r.stdout.decode().count("\n") == 2


def _hwloc_components(stderr):
    # every rank prints its list; with several ranks their stderr lines can interleave mid-line, so match
    # the lists anywhere and take the components of all of them
    found = re.findall(r"Final list of enabled discovery components:\s*([A-Za-z0-9_]+(?:,[A-Za-z0-9_]+)*)",
                       stderr.decode(errors="replace"))
    return set(",".join(found).split(",")) if found else None


@pytest.mark.parametrize("np_", [1, 2])
def test_mpi_topology_lean_vs_full(np_):
    # MPI_Init's host discovery (MPICH's embedded hwloc): lean keeps only the flat no_os topology
    # (profiles/mpi_init_floor_box.log: 226 -> 2.3 ms on the MI355X box), full keeps MPI's default, and a
    # HWLOC_COMPONENTS the user set wins; the results are the same either way
    verbose = {"HWLOC_COMPONENTS_VERBOSE": "1"}
    lean = run_final(["--backend=cpu"], stdin_path=input_path(6), np_=np_, env=verbose)
    full = run_final(["--backend=cpu", "--mpi-topology=full"], stdin_path=input_path(6), np_=np_, env=verbose)
    user = run_final(["--backend=cpu"], stdin_path=input_path(6), np_=np_,
                     env=dict(verbose, HWLOC_COMPONENTS="-linuxio"))
    for r in (lean, full, user):
        assert r.returncode == 0 and r.stdout.decode() == expected(6), r.stderr[-400:]
    cl, cf, cu = (_hwloc_components(r.stderr) for r in (lean, full, user))
    if cf is None:
        pytest.skip("this MPI does not report its hwloc discovery components")
    assert "x86" in cf and "linuxio" in cf
    assert cl == {"no_os"}
    assert "x86" in cu and "linuxio" not in cu
    bad = run_final(["--mpi-topology=fast"], stdin_path=input_path(6))
    assert bad.returncode == 2 and b"--mpi-topology" in bad.stderr


def test_timing_exit_line():
    # --timing-exit: the teardown after the job, as the last stderr line (--timing's JSON stays the last
    # line without it)
    r = run_final(["--backend=cpu", "--timing", "--timing-exit"], stdin_path=input_path(6))
    assert r.returncode == 0 and r.stdout.decode() == expected(6)
    lines = [l for l in r.stderr.decode().splitlines() if l.startswith("{")]
    last = json.loads(lines[-1])
    assert set(last["exit_timing_ms"]) == {"job_done", "job_teardown", "mpi_finalize", "releaser_drain"}
    assert last["since_process_start_ms"] > 0 and "timing" in json.loads(lines[-2])
    r = run_final(["--backend=cpu", "--timing"], stdin_path=input_path(6))
    assert "timing" in json.loads(r.stderr.decode().strip().splitlines()[-1])


@pytest.mark.parametrize("quick", ["0", "1"])
def test_quick_exit_flushes_everything(tmp_path, quick):
    # --quick-exit=1 (default) ends with _Exit after the outputs are closed: stdout and --output files
    # must be complete either way
    r = run_final(["--backend=cpu", f"--quick-exit={quick}"], stdin_path=input_path(3), np_=2)
    assert r.returncode == 0 and r.stdout.decode() == expected(3)
    out = tmp_path / "o.txt"
    r = run_final(["--backend=cpu", f"--quick-exit={quick}", f"--output={out}"], stdin_path=input_path(1), np_=2)
    assert r.returncode == 0 and out.read_text() == expected(1)


@pytest.mark.parametrize("mode", ["auto", "0", "1"])
def test_gpu_isolate_flag_on_cpu_ranks(mode):
    # --gpu-isolate is decided before MPI_Init from the flags and the driver's topology; CPU ranks (and a
    # host without GPUs) leave the environment alone and print the golden
    r = run_final(["--backend=cpu", f"--gpu-isolate={mode}", "--log-level=info"], stdin_path=input_path(6), np_=2)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == expected(6)
    assert "runtime isolated" not in r.stderr.decode()
