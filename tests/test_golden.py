"""Golden outputs (race-free reference semantics) — byte-exact, any rank count.

The reference has no expected outputs of its own; these goldens were produced by the survey's brute-force
emulator of cudaFunctions.cu and its independent prefix-sum oracle, which agree.
"""
import pytest

from conftest import expected, input_path, run_final
from mpi_openmp_cuda_amd import Problem, format_results, search_cpu
from mpi_openmp_cuda_amd.models.reference import solve_problem

INPUTS = [1, 2, 3, 4, 5, 6]


@pytest.mark.parametrize("i", INPUTS)
def test_cpu_engine_golden(i):
    prob = Problem.read(input_path(i))
    assert format_results(search_cpu(prob)) == expected(i)


@pytest.mark.parametrize("i", [1, 2, 5, 6])
def test_python_oracle_golden(i):
    prob = Problem.read(input_path(i))
    from mpi_openmp_cuda_amd.utils.io import format_results_py

    assert format_results_py(solve_problem(prob)) == expected(i)


@pytest.mark.parametrize("i", INPUTS)
@pytest.mark.parametrize("np_", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("transport", ["mpi", "shm"])
def test_final_cpu_any_np(i, np_, transport):
    # reference fails at p=8 on input2/5/6 (abort) and prints INT_MIN rows for p > rows (bugs B4/B5)
    r = run_final(["--backend=cpu", f"--transport={transport}"], stdin_path=input_path(i), np_=np_)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == expected(i)


@pytest.mark.parametrize("i", [3, 4])
def test_final_even_partition(i):
    r = run_final(["--backend=cpu", "--partition=even"], stdin_path=input_path(i), np_=3)
    assert r.returncode == 0, r.stderr.decode()
    assert r.stdout.decode() == expected(i)
