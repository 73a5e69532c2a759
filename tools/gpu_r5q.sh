# round 5: swipe for records of 65..128 letters (24 / 32 record words) — the mid shape, regressions, tests
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u tools/kernel_bench.py mid input6 input1 heavy6 > gpurun_out/r5/kb_q.log 2>&1 || { tail -20 gpurun_out/r5/kb_q.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r5/kb_q.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'], d['kernels'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "selection or extreme or swipe or wire or short" > gpurun_out/r5/pytest_q.log 2>&1; rc=$?; tail -3 gpurun_out/r5/pytest_q.log; exit $rc
