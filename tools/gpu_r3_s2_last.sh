#!/bin/bash
# GPU call: the round's last tree — full GPU tier, smoke(), the default bench (what the driver runs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_r3_last.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r3_last.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r3_last.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_r3_last.log 2>&1 || { cat gpurun_out/smoke_r3_last.log; exit 1; }
tail -1 gpurun_out/smoke_r3_last.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r3_last.log 2>&1 || { tail -20 gpurun_out/bench_r3_last.log; exit 1; }
tail -1 gpurun_out/bench_r3_last.log | cut -c1-300
