# round 5 A/B: sliding windows with two workgroups per CU (half-LDS windows, MOC_TILE16_SLIDE_WG=2), U = 4 and 2
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 240 python -u tools/kernel_bench.py limits long20k heavylim > gpurun_out/r5/kb_wg1.log 2>&1 || { tail -20 gpurun_out/r5/kb_wg1.log; exit 1; }
MOC_TILE16_SLIDE_WG=2 timeout -k 10 240 python -u tools/kernel_bench.py limits long20k heavylim > gpurun_out/r5/kb_wg2.log 2>&1 || { tail -20 gpurun_out/r5/kb_wg2.log; exit 1; }
MOC_TILE16_SLIDE_WG=2 MOC_TILE_U=2 timeout -k 10 240 python -u tools/kernel_bench.py limits long20k heavylim > gpurun_out/r5/kb_wg2u2.log 2>&1 || { tail -20 gpurun_out/r5/kb_wg2u2.log; exit 1; }
python3 -c "
import json
for f in ('kb_wg1.log','kb_wg2.log','kb_wg2u2.log'):
  for l in open('gpurun_out/r5/'+f):
    if l.startswith('{'):
        d=json.loads(l); print(f, d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"
