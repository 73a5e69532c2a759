#!/bin/bash
# Round 4 GPU call F: the box's CPU share (cores vs SMT siblings), the 1e10-letter stream at np 1/2/4 with
# the root formatting on the node's thread budget, smoke().
set -o pipefail
mkdir -p gpurun_out
bash tools/cpu_topology.sh > gpurun_out/cpu_topology_box.log 2>&1; cat gpurun_out/cpu_topology_box.log
bash tools/gpu_steps.sh \
 "final_1e10_np_r4f:900:THREADS='16' NPS=1 KEEP=1 bash tools/final_1e10_threads.sh && THREADS='8' NPS=2 KEEP=1 bash tools/final_1e10_threads.sh && THREADS='4' NPS=4 bash tools/final_1e10_threads.sh" \
 "smoke_r4f:300:python -c 'import __graft_entry__ as g; g.smoke()'"
rm -f /tmp/moc_1e10.txt
