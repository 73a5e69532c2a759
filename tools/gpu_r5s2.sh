# round 5 A/B: sliding windows forced on the shapes that fit the widened image or widened windows
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 240 python -u tools/kernel_bench.py input3 heavy3 input4 heavy4 > gpurun_out/r5/kb_f0.log 2>&1 || { tail -20 gpurun_out/r5/kb_f0.log; exit 1; }
MOC_TILE16_SLIDE=2 timeout -k 10 240 python -u tools/kernel_bench.py input3 heavy3 input4 heavy4 > gpurun_out/r5/kb_f2.log 2>&1 || { tail -20 gpurun_out/r5/kb_f2.log; exit 1; }
MOC_TILE16_SLIDE=2 MOC_TILE_U=8 timeout -k 10 240 python -u tools/kernel_bench.py input3 input4 > gpurun_out/r5/kb_f8.log 2>&1 || { tail -20 gpurun_out/r5/kb_f8.log; exit 1; }
python3 -c "
import json
for f in ('kb_f0.log','kb_f2.log','kb_f8.log'):
  for l in open('gpurun_out/r5/'+f):
    if l.startswith('{'):
        d=json.loads(l); print(f, d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'], d['kernels'])"
