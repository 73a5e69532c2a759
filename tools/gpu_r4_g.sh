#!/bin/bash
# Round 4 GPU call G: device-resident kernel throughput timed by the engine's own kernel events (the host's
# per-call planning out of the interval), the old and new swipe kernels' durations from a kernel trace, then
# call F (CPU share, 1e10 stream at np 1/2/4, smoke).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_steps.sh \
 "kernel_bench_r4g:400:timeout -k 10 350 python3 tools/kernel_bench.py --min-ms 60 input6 input1 input3 input4" \
 "kernel_trace_ab_r4g:400:for i in 0 1; do lib=\$( [ \$i = 0 ] && echo build/ab_base/libmoc.so || echo mpi_openmp_cuda_amd/lib/libmoc.so ); MOC_LIB_PATH=\$PWD/\$lib timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ktrace_ab_\$i -o k -- python3 tools/kernel_bench.py --min-ms 30 input6 input1 || exit 1; done" || exit 1
bash tools/gpu_r4_f.sh
