# round 5: run lists (LPT) for imbalanced whole-image tile16 splits, A/B against the contiguous split
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u tools/kernel_bench.py limits input3 heavy3 > gpurun_out/r5/kb_s.log 2>&1 || { tail -20 gpurun_out/r5/kb_s.log; exit 1; }
MOC_TILE16_LISTS=0 timeout -k 10 300 python -u tools/kernel_bench.py limits input3 heavy3 > gpurun_out/r5/kb_s0.log 2>&1 || { tail -20 gpurun_out/r5/kb_s0.log; exit 1; }
python3 -c "
import json
for f in ('kb_s.log','kb_s0.log'):
  for l in open('gpurun_out/r5/'+f):
    if l.startswith('{'):
        d=json.loads(l); print(f, d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'], d['kernels'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile16 or extreme or long or selection or tiles or keys" > gpurun_out/r5/pytest_s.log 2>&1; rc=$?; tail -3 gpurun_out/r5/pytest_s.log; exit $rc
