#!/bin/bash
# GPU call: where `final`'s ~125-175 ms outside its job goes (--timing-exit), 1.14 G letters bulk/streamed.
set -o pipefail
mkdir -p gpurun_out
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F > /dev/null || exit 1
for mode in "--quick-exit=0" "" "--quick-exit=0" "" "--quick-exit=0 --batch-records=16777216" "--batch-records=16777216"; do
  sleep 3
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np 1 ./final --timing --timing-exit --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "1.14G mode='$mode' wall_ms=$(( (e - s) / 1000000 )) $(grep '"wall_s"' gpurun_out/r3_timing.txt | grep -o '"wall_s": [0-9.]*') $(tail -1 gpurun_out/r3_timing.txt)"
  rm -f /tmp/moc_big6.out
done > gpurun_out/final_exit_1.1G_r3c_leave.log
cat gpurun_out/final_exit_1.1G_r3c_leave.log
rm -f $F
timeout -k 10 800 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "final or rccl or cli" > gpurun_out/gpu_tests_r3_exit.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r3_exit.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r3_exit.log
