#!/bin/bash
# Round 4 GPU call J: the --backend=hip launch after the image upload moved to a page-locked staging buffer,
# with the kernel preload set varied (MOC_PRELOAD none / the swipe files / all), and its API trace again.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hip_wall_trace_j
W="NPS=1 INPUTS='6 1 3' REPS=7 SPACING=1 HELLO=0 TIMING=1 EXTRA='--backend=hip --log-level=debug' bash tools/final_walltime.sh"
bash tools/gpu_steps.sh \
 "gpu_tests_r4j:600:python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu" \
 "wall_preload_none:200:MOC_PRELOAD=none $W" \
 "wall_preload_swipe:200:MOC_PRELOAD=swipe $W" \
 "wall_preload_all:200:MOC_PRELOAD=all $W" \
 "wall_hello:200:NPS=1 INPUTS=6 REPS=7 SPACING=1 HELLO=1 EXTRA='--backend=hip' bash tools/final_walltime.sh" \
 "hip_wall_trace_j:120:cd /tmp && timeout -k 10 100 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/hip_wall_trace_j -o final -- $GRAFT_REPO_ROOT/final --backend=hip --timing --quick-exit=0 < $GRAFT_REPO_ROOT/tests/data/input6.txt"
