#!/bin/bash
# GPU call: the parser with per-block record bookkeeping (fill_bench on the box's CPU), then ./final at
# 1.14 G letters (bulk, streamed) and 1e10 letters, then the GPU tests of the CLI paths.
set -o pipefail
mkdir -p gpurun_out
make -s build/fill_bench || exit 1
OMP_NUM_THREADS=16 timeout -k 5 120 build/fill_bench 40000000 > gpurun_out/fill_bench_box_r3c.log 2>&1 || exit 1
grep -E "count|pack=33|pack_lengths" gpurun_out/fill_bench_box_r3c.log | head -8
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F || exit 1
for mode in "" "" "--batch-records=16777216" "--transport=rccl"; do
  rm -f /tmp/moc_big6.out
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np 1 ./final --timing --device=0 --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_mode_timing.txt || { tail -5 gpurun_out/r3_mode_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "mode='$mode' wall_ms=$(( (e - s) / 1000000 )) out_bytes=$(stat -c %s /tmp/moc_big6.out) md5=$(md5sum < /tmp/moc_big6.out | cut -c1-12) $(tail -1 gpurun_out/r3_mode_timing.txt)"
done > gpurun_out/final_modes_r3h.log
cut -c1-900 gpurun_out/final_modes_r3h.log
rm -f $F /tmp/moc_big6.out
bash tools/final_1e10.sh > gpurun_out/final_1e10_r3d.log 2>&1 || { tail -5 gpurun_out/final_1e10_r3d.log; exit 1; }
tail -1 gpurun_out/final_1e10_r3d.log | cut -c1-700
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "final_cli or streaming or narrow or rccl" > gpurun_out/gpu_tests_r3_sub7.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r3_sub7.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r3_sub7.log
