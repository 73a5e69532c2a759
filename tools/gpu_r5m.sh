# round 5: tile16 32-bit selection keys — throughput, then the tile16 / extremes GPU tests
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 200 python -u tools/kernel_bench.py input3 limits input4 long20k > gpurun_out/r5/kb_m.log 2>&1 || { tail -20 gpurun_out/r5/kb_m.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r5/kb_m.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile16 or extreme or long" > gpurun_out/r5/pytest_m.log 2>&1; rc=$?; tail -3 gpurun_out/r5/pytest_m.log; exit $rc
