#!/bin/bash
# GPU call: the bench with the input6 wall-clock field, at 1 rank and as a 2-rank gloo rehearsal on one GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r3_wall6.log 2> gpurun_out/bench_r3_wall6.err || { tail -5 gpurun_out/bench_r3_wall6.err; exit 1; }
tail -1 gpurun_out/bench_r3_wall6.log
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --allow-shared-gpu --records-per-gpu 8388608 --steps 10 --warmup 2 \
  > gpurun_out/bench_r3_gloo2_wall6.log 2> gpurun_out/bench_r3_gloo2_wall6.err || { tail -5 gpurun_out/bench_r3_gloo2_wall6.err; exit 1; }
tail -1 gpurun_out/bench_r3_gloo2_wall6.log
