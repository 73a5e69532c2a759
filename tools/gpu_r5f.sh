# round 5: tile16 sub-tiles per wave A/B on the widened sweep (input3) and limits
set -o pipefail
mkdir -p gpurun_out/r5
run() { echo "== $1"; shift; env "$@" timeout -k 10 200 python -u tools/kernel_bench.py input3 limits input4 > gpurun_out/r5/kb_f.log 2>&1 || exit 1
  python3 -c "
import json
for l in open('gpurun_out/r5/kb_f.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"; }
run default MOC_X=0
run u4 MOC_TILE_U=4
run u1 MOC_TILE_U=1
