#!/bin/bash
# Round 4 GPU call O: where the swipe kernel's device-resident time goes — the build before the anchor LUT was
# stored by Seq1 letter (ab_prev), the current one, and A/B builds that drop the per-lane anchor LUT read (ab1), read one profile row for every lane (ab2), or both (ab3). Timing only: the variants'
# results are wrong by construction ("verified": false expected for them).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/swipe_ab_r4o.log
: > $out
for lib in build/ab_prev/libmoc.so mpi_openmp_cuda_amd/lib/libmoc.so build/variant_ab1/libmoc.so build/variant_ab2/libmoc.so build/variant_ab3/libmoc.so; do
  echo "# $lib" >> $out
  MOC_LIB_PATH=$PWD/$lib timeout -k 10 200 python tools/kernel_bench.py input6 input1 >> $out 2>&1 || exit 1
done
cat $out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu > gpurun_out/gpu_tests_r4o.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests_r4o.log; exit $rc
