#!/bin/bash
# Round 4 GPU call K: swipe instances split into one code object per (letter form, NOFF); staged batches of
# one chunk on the compute stream alone. GPU tier, headline bench, --backend=hip wall-clock at np 1/2 and
# API traces of input6 (swipe, direct) and input3 (tile16, staged).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=gpurun_out/hip_wall_trace_k
mkdir -p $T
bash tools/gpu_steps.sh \
 "gpu_tests_r4k:600:python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu" \
 "bench_r4k:300:python bench.py --steps 50 --warmup 5" \
 "final_walltime_hip_r4k:300:NPS='1 2' INPUTS='6 1 3' REPS=7 SPACING=1 HELLO=1 TIMING=1 EXTRA='--backend=hip --log-level=debug' bash tools/final_walltime.sh" \
 "trace_k_input6:120:cd /tmp && timeout -k 10 100 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$T -o input6 -- $GRAFT_REPO_ROOT/final --backend=hip --timing --quick-exit=0 < $GRAFT_REPO_ROOT/tests/data/input6.txt" \
 "trace_k_input3:120:cd /tmp && timeout -k 10 100 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$T -o input3 -- $GRAFT_REPO_ROOT/final --backend=hip --timing --quick-exit=0 < $GRAFT_REPO_ROOT/tests/data/input3.txt"
