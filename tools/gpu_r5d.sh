# round 5: tile16 occupancy (two workgroups per CU where the image fits half the LDS) + sub-tile A/B
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "tile16 or long or extreme or random or golden or mfma or context or windowed" > gpurun_out/r5/gputest_d.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5/gputest_d.log; tail -3 gpurun_out/r5/gputest_d.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kernel_bench.py input3 input4 limits long20k > gpurun_out/r5/kb_d.log 2>&1 || exit 1
MOC_TILE_U=4 timeout -k 10 200 python -u tools/kernel_bench.py input3 limits > gpurun_out/r5/kb_d_u4.log 2>&1 || exit 1
MOC_TILE_U=1 timeout -k 10 200 python -u tools/kernel_bench.py input3 limits > gpurun_out/r5/kb_d_u1.log 2>&1 || exit 1
for f in kb_d kb_d_u4 kb_d_u1; do echo "== $f"; python3 -c "
import json,sys
for l in open('gpurun_out/r5/$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"; done
