#!/bin/bash
# The kernel tests on the device-bounds-checked library (make debug-kernels; copy build/debug/libmoc.so to
# build/dbgk/ — build/debug stays out of a gpurun upload). MOC_DCHECK reports print per lane, so the output is
# folded into one "COUNT n <report>" line per distinct check (0 lines: no report).
#   bash tools/dcheck.sh 'wire or swipe or tile16'     (a pytest -k expression; default: every kernel test)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=${DBG_LIB:-$PWD/build/dbgk/libmoc.so}
[ -f "$LIB" ] || { echo "no bounds-checked library at $LIB (make debug-kernels, then copy it there)"; exit 2; }
MOC_LIB_PATH=$LIB MOC_ALLOW_VARIANT_LIB=1 timeout -k 10 ${SECS:-800} \
  python -u -m pytest -s -q --timeout 120 --timeout-method thread tests/test_gpu.py -m gpu \
  -k "${1:-wire or swipe or tile16 or slide or extreme or keys or long or device or golden or context}" 2>&1 |
  awk '/MOC_DCHECK/ {sub(/block [0-9]+ thread [0-9]+/, ""); c[$0]++; next} {print} END {for (k in c) print "COUNT", c[k], k}'
