#!/bin/bash
# GPU call: engine start-up overlapped with the encode and the pins — final CLI GPU tests, then 1.14 G
# letters bulk/streamed and 1e10 letters streamed (engine_wait, ring_pin, wall).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "final or rccl or cli or stream or host_stream" > gpurun_out/gpu_tests_r3_populate.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r3_populate.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r3_populate.log
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F > /dev/null || exit 1
for mode in "" "" "--batch-records=16777216" "--batch-records=16777216"; do
  sleep 3
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np 1 ./final --timing --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "1.14G mode='$mode' wall_ms=$(( (e - s) / 1000000 )) md5=$(md5sum < /tmp/moc_big6.out | cut -c1-12) $(tail -1 gpurun_out/r3_timing.txt)"
  rm -f /tmp/moc_big6.out
done > gpurun_out/final_modes_1.1G_r3r_populate.log
grep -o "1.14G mode='[^']*' wall_ms=[0-9]* md5=[0-9a-f]*\|\"engine_wait_ms\": [0-9.]*\|\"pin_ms\": [0-9.]*\|\"ring_pin\": [0-9.]*\|\"wall_s\": [0-9.]*" gpurun_out/final_modes_1.1G_r3r_populate.log
rm -f $F
F=/tmp/moc_1e10.txt
timeout -k 10 900 python3 tools/gen_synthetic.py --shape input6 --records 1176470589 --jobs 16 --out $F > /dev/null || exit 1
for r in 1 2 3; do
  sleep 3
  s=$(date +%s%N)
  timeout -k 10 600 /opt/conda/bin/mpiexec -np 1 ./final --timing --input=$F --batch-records=16777216 \
    --output=/dev/null 2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "1e10 run=$r wall_ms=$(( (e - s) / 1000000 )) $(tail -1 gpurun_out/r3_timing.txt)"
done > gpurun_out/final_1e10_stream_r3j_populate.log
grep -o "1e10 run=[0-9]* wall_ms=[0-9]*\|\"wall_s\": [0-9.]*\|\"ring_pin\": [0-9.]*\|\"count_ahead\": [0-9.]*\|\"count_ms\": [0-9.]*" gpurun_out/final_1e10_stream_r3j_populate.log
rm -f $F
