# round 5: tile16 work list (largest tiles first, persistent waves) vs the static split
set -o pipefail
mkdir -p gpurun_out/r5
run() { echo "== $1"; shift; env "$@" timeout -k 10 200 python -u tools/kernel_bench.py limits input3 input4 long20k > gpurun_out/r5/kb_n.log 2>&1 || { tail -20 gpurun_out/r5/kb_n.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r5/kb_n.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"; }
run queue MOC_X=0
run static MOC_TILE16_QUEUE=0
run queue_u4 MOC_TILE_U=4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile16 or extreme or long or keys" > gpurun_out/r5/pytest_n.log 2>&1; rc=$?; tail -3 gpurun_out/r5/pytest_n.log; exit $rc
