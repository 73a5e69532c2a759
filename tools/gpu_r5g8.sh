# round 5 A/B: sliding-window kernel with 8 steps per read group at U = 4 (build/variant_g8) against the default 4
set -o pipefail
mkdir -p gpurun_out/r5
for i in 1 2; do
  timeout -k 10 240 python -u tools/kernel_bench.py limits long20k heavylim > gpurun_out/r5/kb_g_def$i.log 2>&1 || { tail -20 gpurun_out/r5/kb_g_def$i.log; exit 1; }
  env MOC_LIB_PATH=$PWD/build/variant_g8/libmoc.so MOC_ALLOW_VARIANT_LIB=1 timeout -k 10 240 python -u tools/kernel_bench.py limits long20k heavylim > gpurun_out/r5/kb_g_g8$i.log 2>&1 || { tail -20 gpurun_out/r5/kb_g_g8$i.log; exit 1; }
done
python3 -c "
import json
for f in ('kb_g_def1.log','kb_g_g81.log','kb_g_def2.log','kb_g_g82.log'):
  for l in open('gpurun_out/r5/'+f):
    if l.startswith('{'):
        d=json.loads(l); print(f, d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"
