#!/bin/bash
# GPU call: parser throughput on the box's CPU, ./final bulk vs streaming at 1.14 G letters, 1e10 letters
# streamed, the reference invocation's wall-clock on inputs 1-6, and the bench's per-rank fields (2-rank gloo).
set -o pipefail
mkdir -p gpurun_out
make -s build/fill_bench || exit 1
(grep -m1 "model name" /proc/cpuinfo; grep -o -w 'avx512_vbmi2\|avx512bw' /proc/cpuinfo | sort -u | tr '\n' ' '; echo) > gpurun_out/fill_bench_box.log
for t in 16 8 1; do OMP_NUM_THREADS=$t timeout -k 5 120 build/fill_bench 40000000 >> gpurun_out/fill_bench_box.log 2>&1 || exit 1; done
MODES="--output=/tmp/moc_big6.out|--output=/tmp/moc_big6.out --batch-records=16777216" NPS="1" timeout -k 10 600 bash tools/final_scale.sh > gpurun_out/final_scale_r3b.log 2>&1 || { tail -5 gpurun_out/final_scale_r3b.log; exit 1; }
head -3 gpurun_out/final_scale_r3b.log | cut -c1-400
timeout -k 10 1000 bash tools/final_1e10.sh > gpurun_out/final_1e10.log 2>&1 || { tail -5 gpurun_out/final_1e10.log; exit 1; }
cut -c1-600 gpurun_out/final_1e10.log | tail -2
timeout -k 10 300 bash tools/final_walltime_r3.sh > gpurun_out/final_walltime_r3.log 2>&1 || { tail -5 gpurun_out/final_walltime_r3.log; exit 1; }
cat gpurun_out/final_walltime_r3.log
