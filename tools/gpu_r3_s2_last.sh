#!/bin/bash
# GPU call: the round's last tree — full GPU tier, smoke(), the default bench (what the driver runs).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_r3_last2.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r3_last2.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r3_last2.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_r3_last2.log 2>&1 || { cat gpurun_out/smoke_r3_last2.log; exit 1; }
tail -1 gpurun_out/smoke_r3_last2.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r3_last2.log 2>&1 || { tail -20 gpurun_out/bench_r3_last2.log; exit 1; }
tail -1 gpurun_out/bench_r3_last2.log | cut -c1-300
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
done > gpurun_out/final_modes_1.1G_r3s_preload.log
grep -o "1.14G mode='[^']*' wall_ms=[0-9]* md5=[0-9a-f]*\|\"pin_ms\": [0-9.]*\|\"compute_ms\": [0-9.]*\|\"wall_s\": [0-9.]*" gpurun_out/final_modes_1.1G_r3s_preload.log
rm -f $F
