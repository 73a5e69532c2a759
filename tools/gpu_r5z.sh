# round 5: sliding windows by default for long records on windowed plans too, with the group-fill rule;
# bench shapes and the tile / long-context tests
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 240 python -u tools/kernel_bench.py limits heavylim mid3k long20k long150k input3 input4 > gpurun_out/r5/kb_z1.log 2>&1 || { tail -20 gpurun_out/r5/kb_z1.log; exit 1; }
python3 -c "
import json
for f in ('kb_z1.log',):
  for l in open('gpurun_out/r5/'+f):
    if l.startswith('{'):
        d=json.loads(l); print(f, d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'], d['kernels'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile16 or extreme or long or keys or selection or tiles or window or context" > gpurun_out/r5/pytest_z.log 2>&1; rc=$?; tail -5 gpurun_out/r5/pytest_z.log; exit $rc
