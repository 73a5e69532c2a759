# round 5: P33 wire batches through the wave-autonomous swipe kernel — throughput vs bytes, then the tests
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u tools/kernel_bench.py input6 input1 --variants tile16,wire,wirebytes > gpurun_out/r5/kb_j.log 2>&1 || { tail -20 gpurun_out/r5/kb_j.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r5/kb_j.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d['variant'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "wire_device or wire_p33" > gpurun_out/r5/pytest_j.log 2>&1; rc=$?; tail -3 gpurun_out/r5/pytest_j.log; exit $rc
