#!/bin/bash
# GPU call: the node streaming flow with prefaulted ring slots (print on the main thread) — 1.14 G letters (batches of 16.7 M / 67 M
# records vs bulk) and BASELINE config 5 (1e10 letters) through ./final; then the streaming GPU tests.
set -o pipefail
mkdir -p gpurun_out
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F || exit 1
for mode in "" "--batch-records=16777216" "--batch-records=67108864" "--batch-records=16777216" "--transport=rccl --batch-records=16777216"; do
  rm -f /tmp/moc_big6.out
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np 1 ./final --timing --device=0 --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_mode_timing.txt || { tail -5 gpurun_out/r3_mode_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "mode='$mode' wall_ms=$(( (e - s) / 1000000 )) out_bytes=$(stat -c %s /tmp/moc_big6.out) md5=$(md5sum < /tmp/moc_big6.out | cut -c1-12) $(tail -1 gpurun_out/r3_mode_timing.txt)"
done > gpurun_out/final_modes_r3g.log
cut -c1-1000 gpurun_out/final_modes_r3g.log
rm -f $F /tmp/moc_big6.out
bash tools/final_1e10.sh > gpurun_out/final_1e10_r3c.log 2>&1 || { tail -5 gpurun_out/final_1e10_r3c.log; exit 1; }
tail -1 gpurun_out/final_1e10_r3c.log | cut -c1-900
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "streaming or narrow" > gpurun_out/gpu_tests_r3_sub6.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r3_sub6.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r3_sub6.log
