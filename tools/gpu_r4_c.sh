#!/bin/bash
# Round 4 GPU call C: multi-rank rehearsal (8 bench ranks over gloo on the one GPU; ./final np 1/4/8 at
# 1.14 G letters, md5-equal), the RCCL transport at one rank under rocprofv3 (kernel trace), step variance.
set -o pipefail
mkdir -p gpurun_out
python3 tools/gen_synthetic.py --shape input6 --records 8000000 --jobs 16 --out /tmp/rccl_in.txt > /dev/null || exit 1
bash tools/gpu_steps.sh \
 "rehearse_8ranks_r4:900:NR=8 NPS='1 4 8' bash tools/rehearse_ranks.sh" \
 "rccl_np1_trace_r4:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/rccl_np1_prof -o rccl -- ./final --backend=hip --transport=rccl --device=0 --input=/tmp/rccl_in.txt --output=/dev/null --timing" \
 "step_variance_r4:400:STEPS=2000 bash tools/step_variance.sh"
rm -f /tmp/rccl_in.txt
