#!/bin/bash
# Round 4 GPU call I: where `mpiexec -np N ./final --backend=hip < input6.txt` spends its wall-clock, next to
# the floor of any MPI program that runs one kernel (tools/hip_hello.hip): spaced launches at np 1/2 with
# --timing, then a HIP API + kernel + copy trace of one singleton launch of each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hip_wall_trace
bash tools/gpu_steps.sh \
 "final_walltime_hip_r4i:400:NPS='1 2' INPUTS='6 1 3' REPS=7 SPACING=1 HELLO=1 TIMING=1 EXTRA='--backend=hip --log-level=debug' bash tools/final_walltime.sh" \
 "hip_wall_trace_final:120:cd /tmp && timeout -k 10 100 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/hip_wall_trace -o final -- $GRAFT_REPO_ROOT/final --backend=hip --timing --quick-exit=0 < $GRAFT_REPO_ROOT/tests/data/input6.txt" \
 "hip_wall_trace_hello:120:cd /tmp && timeout -k 10 100 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/hip_wall_trace -o hello -- $GRAFT_REPO_ROOT/build/hip_hello"
