# round 5 timing-only A/B (throwaway variant libraries, wrong results by construction): the sliding-window
# kernel without restaging after the first window (build/variant_nostage, barriers kept) and without the
# barriers too (build/variant_nobar) — the upper bound of what staging and its barriers cost
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 240 python -u tools/kernel_bench.py limits long20k > gpurun_out/r5/kb_ns_def.log 2>&1 || { tail -20 gpurun_out/r5/kb_ns_def.log; exit 1; }
env MOC_LIB_PATH=$PWD/build/variant_nostage/libmoc.so MOC_ALLOW_VARIANT_LIB=1 timeout -k 10 240 python -u tools/kernel_bench.py limits long20k > gpurun_out/r5/kb_ns_ns.log 2>&1 || { tail -20 gpurun_out/r5/kb_ns_ns.log; exit 1; }
env MOC_LIB_PATH=$PWD/build/variant_nobar/libmoc.so MOC_ALLOW_VARIANT_LIB=1 timeout -k 10 240 python -u tools/kernel_bench.py limits long20k > gpurun_out/r5/kb_ns_nb.log 2>&1 || { tail -20 gpurun_out/r5/kb_ns_nb.log; exit 1; }
python3 -c "
import json
for f in ('kb_ns_def.log','kb_ns_ns.log','kb_ns_nb.log'):
  for l in open('gpurun_out/r5/'+f):
    if l.startswith('{'):
        d=json.loads(l); print(f, d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"
