# round 5: tile16 widened entries (A/B MOC_TILE16_WIDE) — correctness then throughput
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "tile16 or long or extreme or random or golden or mfma or context or windowed or kernel_selection or mixed" > gpurun_out/r5/gputest_e.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5/gputest_e.log; tail -3 gpurun_out/r5/gputest_e.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/kernel_bench.py input3 input4 limits > gpurun_out/r5/kb_e_wide.log 2>&1 || exit 1
MOC_TILE16_WIDE=0 timeout -k 10 200 python -u tools/kernel_bench.py input3 > gpurun_out/r5/kb_e_narrow.log 2>&1 || exit 1
for f in kb_e_wide kb_e_narrow; do echo "== $f"; python3 -c "
import json,sys
for l in open('gpurun_out/r5/$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"; done
