# round 5: the int16 tile16 profile for weights past the byte pairs (heavy3 / heavy4), then the tile tests
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u tools/kernel_bench.py heavy3 heavy4 input3 input4 > gpurun_out/r5/kb_r.log 2>&1 || { tail -20 gpurun_out/r5/kb_r.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r5/kb_r.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'], d['kernels'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile16 or extreme or long or selection or tiles or keys" > gpurun_out/r5/pytest_r.log 2>&1; rc=$?; tail -3 gpurun_out/r5/pytest_r.log; exit $rc
