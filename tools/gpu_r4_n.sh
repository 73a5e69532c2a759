#!/bin/bash
# Round 4 GPU call N: per-rank GPU isolation (--gpu-isolate) on the box, and the GPU tier.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_steps.sh \
 "gpu_tests_r4n:600:python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu" \
 "wall_isolate_r4n:200:NPS='1 2' INPUTS='6' REPS=7 SPACING=1 HELLO=0 TIMING=1 EXTRA='--backend=hip --gpu-isolate=1 --log-level=info' bash tools/final_walltime.sh"
