# round 5: two workgroups per CU as the sliding-window default — bench shapes and the tile tests
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 240 python -u tools/kernel_bench.py limits long20k long150k heavylim mid3k > gpurun_out/r5/kb_wgd.log 2>&1 || { tail -20 gpurun_out/r5/kb_wgd.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r5/kb_wgd.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'], d['kernels'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile16 or extreme or long or keys or selection or tiles or window or context" > gpurun_out/r5/pytest_wgd.log 2>&1; rc=$?; tail -5 gpurun_out/r5/pytest_wgd.log; exit $rc
