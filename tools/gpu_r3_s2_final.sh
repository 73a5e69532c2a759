#!/bin/bash
# GPU call: the session's final tree on one MI355X — full GPU tier, smoke(), bench, ./final at 1.14 G and
# 1.0e10 letters, the reference invocation on inputs 1-6 at 1/2/4 ranks.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/gpu_tests_r3_final2.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r3_final2.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r3_final2.log
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke_r3_final2.log 2>&1 || { cat gpurun_out/smoke_r3_final2.log; exit 1; }
tail -1 gpurun_out/smoke_r3_final2.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_r3_final2.log 2>&1 || { tail -20 gpurun_out/bench_r3_final2.log; exit 1; }
tail -1 gpurun_out/bench_r3_final2.log | cut -c1-200
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F > /dev/null || exit 1
for mode in "" "" "--batch-records=16777216" "--batch-records=16777216"; do
  sleep 2
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np 1 ./final --timing --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "1.14G mode='$mode' wall_ms=$(( (e - s) / 1000000 )) md5=$(md5sum < /tmp/moc_big6.out | cut -c1-12) $(tail -1 gpurun_out/r3_timing.txt)"
  rm -f /tmp/moc_big6.out
done > gpurun_out/final_modes_1.1G_r3_final2.log
grep -o "1.14G mode='[^']*' wall_ms=[0-9]* md5=[0-9a-f]*" gpurun_out/final_modes_1.1G_r3_final2.log
rm -f $F
F=/tmp/moc_1e10.txt
timeout -k 10 900 python3 tools/gen_synthetic.py --shape input6 --records 1176470589 --jobs 16 --out $F > /dev/null || exit 1
for r in 1 2 3; do
  sleep 2
  s=$(date +%s%N)
  timeout -k 10 600 /opt/conda/bin/mpiexec -np 1 ./final --timing --input=$F --batch-records=16777216 \
    --output=/dev/null 2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "1e10 run=$r wall_ms=$(( (e - s) / 1000000 )) $(tail -1 gpurun_out/r3_timing.txt)"
done > gpurun_out/final_1e10_stream_r3_final2.log
grep -o "1e10 run=[0-9]* wall_ms=[0-9]*\|\"wall_s\": [0-9.]*" gpurun_out/final_1e10_stream_r3_final2.log
rm -f $F
bash tools/final_walltime_r3b.sh > gpurun_out/final_walltime_r3_final2.log 2>&1 || exit 1
grep "input6\|hello" gpurun_out/final_walltime_r3_final2.log
