#!/bin/bash
# Round 4 GPU call E: the whole GPU tier, the RCCL transport traced at one rank (--quick-exit=0: rocprofv3
# writes its files from exit handlers that _Exit skips), the HIP wall-clock of the reference inputs, the
# host phases of the 1e10-letter stream by thread count, the bench.
set -o pipefail
mkdir -p gpurun_out
python3 tools/gen_synthetic.py --shape input6 --records 8000000 --jobs 16 --out /tmp/rccl_in.txt > /dev/null || exit 1
bash tools/gpu_steps.sh \
 "gpu_tests_r4e:900:python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu" \
 "rccl_np1_trace_r4e:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/rccl_np1_prof -o rccl -- ./final --backend=hip --transport=rccl --device=0 --input=/tmp/rccl_in.txt --output=/dev/null --timing --quick-exit=0" \
 "final_walltime_hip_r4e:400:NPS='1 2' REPS=5 SPACING=1 HELLO=0 TIMING=1 EXTRA='--backend=hip --device=0' bash tools/final_walltime.sh" \
 "final_1e10_threads_r4e:900:THREADS='1 2 4 8 16' NPS=1 KEEP=1 bash tools/final_1e10_threads.sh && THREADS='8' NPS=2 KEEP=1 bash tools/final_1e10_threads.sh && THREADS='4' NPS=4 bash tools/final_1e10_threads.sh" \
 "bench_r4e:300:python bench.py --steps 20 --warmup 5"
rm -f /tmp/rccl_in.txt /tmp/moc_1e10.txt
