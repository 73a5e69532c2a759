#!/bin/bash
# GPU call: the lean MPI start-up at scale — final CLI GPU tests, then 1.14 G and 1.0e10 input6-shaped
# letters through ./final (bulk and streamed) with the lean and the full MPI topology.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "final_cli or rccl" \
  > gpurun_out/gpu_tests_r3_final_cli.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r3_final_cli.log; exit 1; }
tail -1 gpurun_out/gpu_tests_r3_final_cli.log
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F > /dev/null || exit 1
for mode in "--mpi-topology=full" "" "--mpi-topology=full --batch-records=16777216" "--batch-records=16777216"; do
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np 1 ./final --timing --device=0 --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "1.14G mode='$mode' wall_ms=$(( (e - s) / 1000000 )) md5=$(md5sum < /tmp/moc_big6.out | cut -c1-12) $(tail -1 gpurun_out/r3_timing.txt)"
  rm -f /tmp/moc_big6.out
done > gpurun_out/final_modes_1.1G_r3j_kfd.log
grep -o "1.14G mode='[^']*' wall_ms=[0-9]* md5=[0-9a-f]*" gpurun_out/final_modes_1.1G_r3j_kfd.log
rm -f $F
F=/tmp/moc_1e10.txt
timeout -k 10 900 python3 tools/gen_synthetic.py --shape input6 --records 1176470589 --jobs 16 --out $F > /dev/null || exit 1
for mode in "" "" ""; do
  s=$(date +%s%N)
  timeout -k 10 600 /opt/conda/bin/mpiexec -np 1 ./final --timing --device=0 --input=$F --batch-records=16777216 \
    --output=/dev/null $mode 2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "1e10 mode='$mode' wall_ms=$(( (e - s) / 1000000 )) $(tail -1 gpurun_out/r3_timing.txt)"
done > gpurun_out/final_1e10_stream_r3f_kfd.log
grep -o "1e10 mode='[^']*' wall_ms=[0-9]*\|\"wall_s\": [0-9.]*" gpurun_out/final_1e10_stream_r3f_kfd.log
rm -f $F
