# round 5: int16 windows staged 8 entries per load (heavylim, heavy4), and sliding windows in place of byte-pair
# windows on L1 past one byte image (MOC_TILE16_SLIDE=2: long20k, long150k), then the tile tests
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 240 python -u tools/kernel_bench.py heavylim heavy4 limits long20k long150k > gpurun_out/r5/kb_y1.log 2>&1 || { tail -20 gpurun_out/r5/kb_y1.log; exit 1; }
MOC_TILE16_SLIDE=2 timeout -k 10 240 python -u tools/kernel_bench.py long20k long150k > gpurun_out/r5/kb_y2.log 2>&1 || { tail -20 gpurun_out/r5/kb_y2.log; exit 1; }
python3 -c "
import json
for f in ('kb_y1.log','kb_y2.log'):
  for l in open('gpurun_out/r5/'+f):
    if l.startswith('{'):
        d=json.loads(l); print(f, d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'], d['kernels'])"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile16 or extreme or long or keys or selection or tiles" > gpurun_out/r5/pytest_y.log 2>&1; rc=$?; tail -5 gpurun_out/r5/pytest_y.log; exit $rc
