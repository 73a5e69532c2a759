#!/bin/bash
# Round 4 GPU call H: the tree as it stands — GPU tier, smoke, headline bench, its kernel trace, and the
# reference invocation's wall-clock (default engine) at 1/2/4 ranks.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_steps.sh \
 "gpu_tests_r4h:900:python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu" \
 "smoke_r4h:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "bench_r4h:300:python bench.py --steps 50 --warmup 5" \
 "bench_trace_r4h:300:timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bench_trace_r4 -o b -- python3 bench.py --steps 20 --warmup 5 --final-wall 0" \
 "final_walltime_r4h:400:NPS='1 2 4' REPS=7 HELLO=1 bash tools/final_walltime.sh"
