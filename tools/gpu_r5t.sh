# round 5: P33 field decode and base-6 length digits on 24-bit multiplies (device-resident wire batches)
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u tools/kernel_bench.py input6 input1 --variants wire,wirebytes,tile16 > gpurun_out/r5/kb_t2.log 2>&1 || { tail -20 gpurun_out/r5/kb_t2.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r5/kb_t2.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d['variant'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'], d['kernels'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "wire or p33 or extreme or swipe or base6 or len6" > gpurun_out/r5/pytest_t2.log 2>&1; rc=$?; tail -3 gpurun_out/r5/pytest_t2.log; exit $rc
