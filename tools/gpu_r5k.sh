# round 5: widened windows for short records on L1 ~ 1500..3050 (input4) vs the whole byte-pair image
set -o pipefail
mkdir -p gpurun_out/r5
run() { echo "== $1"; shift; env "$@" timeout -k 10 200 python -u tools/kernel_bench.py input4 limits input3 long20k > gpurun_out/r5/kb_k.log 2>&1 || { tail -20 gpurun_out/r5/kb_k.log; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/r5/kb_k.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], round(d['cells_per_s']/1e12,2), d['gpu_ms'], d['verified'])"; }
run winwide MOC_X=0
run whole MOC_TILE16_WINWIDE=0
run winwide_u4 MOC_TILE16_WIN_U8=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile16 or extreme or long" > gpurun_out/r5/pytest_kk.log 2>&1; rc=$?; tail -3 gpurun_out/r5/pytest_kk.log; exit $rc
