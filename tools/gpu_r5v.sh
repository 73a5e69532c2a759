# round 5: A/B of the tile16 epilogue (interleaved DPP scans + full-tile path) against the previous kernel
# (build/variant_old16: make variant NAME=old16 from the previous tile16_kernels.hip), interleaved
set -o pipefail
mkdir -p gpurun_out/r5
OLD="MOC_LIB_PATH=$PWD/build/variant_old16/libmoc.so MOC_ALLOW_VARIANT_LIB=1"
for i in 1 2; do
  timeout -k 10 300 python -u tools/kernel_bench.py input4 heavy4 input3 > gpurun_out/r5/kb_v_new$i.log 2>&1 || { tail -20 gpurun_out/r5/kb_v_new$i.log; exit 1; }
  env MOC_LIB_PATH=$PWD/build/variant_old16/libmoc.so MOC_ALLOW_VARIANT_LIB=1 timeout -k 10 300 python -u tools/kernel_bench.py input4 heavy4 input3 > gpurun_out/r5/kb_v_old$i.log 2>&1 || { tail -20 gpurun_out/r5/kb_v_old$i.log; exit 1; }
done
python3 -c "
import json
for f in ('kb_v_new1.log','kb_v_old1.log','kb_v_new2.log','kb_v_old2.log'):
  for l in open('gpurun_out/r5/'+f):
    if l.startswith('{'):
        d=json.loads(l); print(f, d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"
