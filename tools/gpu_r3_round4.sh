#!/bin/bash
# GPU call: the rccl transport at 1.14 G letters (1 rank) after the warm-up / scratch / huge-page changes, the
# box's pack33 rate, and a short GPU test subset.
set -o pipefail
mkdir -p gpurun_out
make -s build/fill_bench || exit 1
OMP_NUM_THREADS=16 timeout -k 5 120 build/fill_bench 40000000 > gpurun_out/fill_bench_box2.log 2>&1 || exit 1
grep pack33 gpurun_out/fill_bench_box2.log
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F || exit 1
for mode in "--transport=rccl" "--transport=rccl --batch-records=33554432" "--collectives=rccl" "--batch-records=16777216"; do
  rm -f /tmp/moc_big6.out
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np 1 ./final --timing --device=0 --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_mode_timing.txt || { tail -5 gpurun_out/r3_mode_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "mode='$mode' wall_ms=$(( (e - s) / 1000000 )) out_bytes=$(stat -c %s /tmp/moc_big6.out) $(tail -1 gpurun_out/r3_mode_timing.txt)"
done > gpurun_out/final_modes_r3b.log
cut -c1-900 gpurun_out/final_modes_r3b.log
rm -f $F /tmp/moc_big6.out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "rccl or tail or streaming or final_cli" > gpurun_out/gpu_tests_r3_sub.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r3_sub.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r3_sub.log
