#!/bin/bash
# GPU call: the restored tree end to end on one MI355X — full GPU test tier, smoke(), the default bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_r3_full2.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r3_full2.log; exit 1; }
tail -3 gpurun_out/gpu_tests_r3_full2.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_r3_2.log 2>&1 || { cat gpurun_out/smoke_r3_2.log; exit 1; }
cat gpurun_out/smoke_r3_2.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r3_2.log 2>&1 || { tail -20 gpurun_out/bench_r3_2.log; exit 1; }
tail -2 gpurun_out/bench_r3_2.log
