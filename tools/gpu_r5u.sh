# round 5: P33 next-tile field prefetch + faster digit decode (wire batches); tile16 epilogue (interleaved
# DPP scans, full-tile fast path) — bench shapes and the affected tests
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u tools/kernel_bench.py input6 input1 --variants wire,wirebytes > gpurun_out/r5/kb_u1.log 2>&1 || { tail -20 gpurun_out/r5/kb_u1.log; exit 1; }
timeout -k 10 300 python -u tools/kernel_bench.py input4 heavy4 input3 limits long20k heavy3 > gpurun_out/r5/kb_u2.log 2>&1 || { tail -20 gpurun_out/r5/kb_u2.log; exit 1; }
python3 -c "
import json
for f in ('kb_u1.log','kb_u2.log'):
  for l in open('gpurun_out/r5/'+f):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d['variant'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'], d['kernels'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "wire or p33 or extreme or swipe or base6 or tile16 or long or keys or selection or tiles" > gpurun_out/r5/pytest_u.log 2>&1; rc=$?; tail -3 gpurun_out/r5/pytest_u.log; exit $rc
