# round 5: tile16 LDS entry forms A/B — byte pairs, widened pairs, int16 columns (unaligned dword reads)
set -o pipefail
mkdir -p gpurun_out/r5
run() { echo "== $1"; shift; env "$@" timeout -k 10 200 python -u tools/kernel_bench.py input3 limits input4 long20k > gpurun_out/r5/kb_i.log 2>&1 || { tail -20 gpurun_out/r5/kb_i.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r5/kb_i.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"; }
run default MOC_X=0
run half MOC_TILE16_FORM=half
run pairs MOC_TILE16_FORM=pairs
MOC_TILE16_FORM=half timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile16 or extreme or long" > gpurun_out/r5/pytest_i.log 2>&1; rc=$?; tail -3 gpurun_out/r5/pytest_i.log; exit $rc
