#!/bin/bash
# Round 4 GPU call M: small host<->device copies on a copy kernel (no SDMA start-up inside short jobs).
# GPU tier (with the new preload / staging / copy tests), --backend=hip wall-clock np 1/2 on input 6/1/3/4,
# API trace of input3 and input4 (staged tile16), headline bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T=gpurun_out/hip_wall_trace_m
mkdir -p $T
bash tools/gpu_steps.sh \
 "gpu_tests_r4m:600:python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu" \
 "final_walltime_hip_r4m:300:NPS='1 2' INPUTS='6 1 3 4' REPS=7 SPACING=1 HELLO=0 TIMING=1 EXTRA='--backend=hip --log-level=debug' bash tools/final_walltime.sh" \
 "trace_m_input3:120:cd /tmp && timeout -k 10 100 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$T -o input3 -- $GRAFT_REPO_ROOT/final --backend=hip --timing --quick-exit=0 < $GRAFT_REPO_ROOT/tests/data/input3.txt" \
 "trace_m_input4:120:cd /tmp && timeout -k 10 100 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$T -o input4 -- $GRAFT_REPO_ROOT/final --backend=hip --timing --quick-exit=0 < $GRAFT_REPO_ROOT/tests/data/input4.txt" \
 "bench_r4m:300:python bench.py --steps 50 --warmup 5"
