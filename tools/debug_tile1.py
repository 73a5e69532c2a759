import os, sys
sys.path.insert(0, ".")
import numpy as np
from mpi_openmp_cuda_amd import HipSearchEngine, Problem
p = Problem.read("tests/data/input3.txt").slice(0, 1)
e = HipSearchEngine(0)
e.set_problem(p.weights, p.seq1)
print(e.solve(p.codes, p.offsets))
print("codes", p.codes[:8].tolist(), "L2", p.n and p.lengths[0])
