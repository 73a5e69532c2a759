#!/bin/bash
# Round 4 GPU call D: swipe fixes re-checked, device-resident counters of the old and new swipe kernels,
# then call C's rehearsal / RCCL trace / step variance.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_steps.sh \
 "r4d_gpu_tests:400:python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu.py -k 'swipe or wire or packed5 or r2 or host_stream or short or kernel_selection or group_coded or stdin'" \
 "pmc_swipe_ab_r4:500:TAG=r4 LIBS='build/ab_base/libmoc.so mpi_openmp_cuda_amd/lib/libmoc.so' SHAPES='input6 input1' bash tools/pmc_ab.sh" || exit 1
bash tools/gpu_r4_c.sh
