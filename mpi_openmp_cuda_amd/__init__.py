"""MI355X-native hybrid MPI + OpenMP + HIP sequence-alignment search framework.

Same capabilities as nmiz1987/MPI-OPENMP-CUDA (CLI ``./final``, stdin format, output lines), rebuilt
for gfx950: an O(L1*L2) diagonal-sweep HIP kernel, a chunked pinned-DMA pipeline per GPU, cost-balanced
decomposition over ranks, RCCL (torch.distributed "nccl") / MPI collectives and a node-shared input
window. See README.md and SURVEY.md.
"""
from .models.problem import Problem
from .models.scoring import PairClass, Semantics, Weights
from .ops.align import (HipSearchEngine, align_search, align_search_device, brute_force_native, decode_keys,
                        device_count, search_cpu, search_hip, search_keys_cpu)
from .utils.io import format_results, write_results
from .utils.synthetic import make_synthetic

__version__ = "0.1.0"
__all__ = [
    "Problem", "PairClass", "Semantics", "Weights", "HipSearchEngine", "align_search", "align_search_device",
    "brute_force_native", "device_count", "search_cpu", "search_hip", "format_results", "write_results",
    "make_synthetic", "search_keys_cpu", "decode_keys",
]
