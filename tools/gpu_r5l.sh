# round 5: limits / input3 — whole byte-pair image vs forced byte-pair windows (A/B)
set -o pipefail
mkdir -p gpurun_out/r5
run() { echo "== $1"; shift; env "$@" timeout -k 10 200 python -u tools/kernel_bench.py limits input3 > gpurun_out/r5/kb_l.log 2>&1 || { tail -20 gpurun_out/r5/kb_l.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r5/kb_l.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"; }
run whole MOC_X=0
run win2976 MOC_TILE16_WINDOW=2976 MOC_TILE16_WIDE=0
run win2976_u2 MOC_TILE16_WINDOW=2976 MOC_TILE_U=2
run win2976_u1 MOC_TILE16_WINDOW=2976 MOC_TILE_U=1
