#!/bin/bash
# Round 4 GPU call: swipe kernel checks + device-resident A/B against the saved baseline build, the HIP
# wall-clock of the reference inputs (spaced launches), the headline bench.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_steps.sh \
 "r4_gpu_swipe_tests:400:python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu.py -k 'swipe or wire or stdin or streaming or group_coded or packed5 or r2 or host_stream or goldens or random_shapes or zero_copy or mixed or brute'" \
 "kernel_bench_r4_ab:400:for lib in build/ab_base/libmoc.so mpi_openmp_cuda_amd/lib/libmoc.so; do echo \"# lib \$lib\"; MOC_LIB_PATH=\$PWD/\$lib timeout -k 5 150 python tools/kernel_bench.py --min-ms 80 input6 input1 || exit 1; done" \
 "final_walltime_hip_r4b_spaced:300:NPS='1 2' INPUTS='6 3' REPS=5 SPACING=2 HELLO=0 TIMING=1 EXTRA='--backend=hip --device=0 --log-level=debug' bash tools/final_walltime.sh" \
 "bench_r4b:300:python bench.py --steps 20 --warmup 5"
