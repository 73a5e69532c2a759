# round 5: sliding widened windows for long records past the widened image (limits, heavylim, mid3k),
# A/B against the previous plans (MOC_TILE16_SLIDE=0), then the tile tests
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 240 python -u tools/kernel_bench.py limits heavylim mid3k input3 input4 > gpurun_out/r5/kb_x1.log 2>&1 || { tail -20 gpurun_out/r5/kb_x1.log; exit 1; }
MOC_TILE_U=2 timeout -k 10 240 python -u tools/kernel_bench.py limits heavylim mid3k > gpurun_out/r5/kb_x0.log 2>&1 || { tail -20 gpurun_out/r5/kb_x0.log; exit 1; }
MOC_TILE_U=8 timeout -k 10 240 python -u tools/kernel_bench.py limits heavylim mid3k > gpurun_out/r5/kb_x4.log 2>&1 || { tail -20 gpurun_out/r5/kb_x4.log; exit 1; }
python3 -c "
import json
for f in ('kb_x1.log','kb_x0.log','kb_x4.log'):
  for l in open('gpurun_out/r5/'+f):
    if l.startswith('{'):
        d=json.loads(l); print(f, d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'], d['kernels'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile16 or extreme or long or keys or selection or tiles" > gpurun_out/r5/pytest_x.log 2>&1; rc=$?; tail -5 gpurun_out/r5/pytest_x.log; exit $rc
