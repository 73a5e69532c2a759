# round 5: the swipe kernel without the obsolete W <= 127 rule — heavy-weight short records, then the tests
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u tools/kernel_bench.py heavy6 input6 input1 > gpurun_out/r5/kb_p.log 2>&1 || { tail -20 gpurun_out/r5/kb_p.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r5/kb_p.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'], d['kernels'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "selection or extreme or swipe or wire" > gpurun_out/r5/pytest_p.log 2>&1; rc=$?; tail -3 gpurun_out/r5/pytest_p.log; exit $rc
