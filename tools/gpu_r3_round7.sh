#!/bin/bash
# GPU call: the rccl transport at 1.14 G letters on 1 rank — bulk text batch (prefaulted registered staging)
# and streamed through the text cutter (flow_device_stream.cpp) — then the GPU tests of the CLI paths.
set -o pipefail
mkdir -p gpurun_out
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F || exit 1
for mode in "--transport=rccl" "--transport=rccl" "--transport=rccl --batch-records=33554432" "--transport=rccl --batch-records=16777216" "--batch-records=16777216"; do
  rm -f /tmp/moc_big6.out
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np 1 ./final --timing --device=0 --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_mode_timing.txt || { tail -5 gpurun_out/r3_mode_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "mode='$mode' wall_ms=$(( (e - s) / 1000000 )) out_bytes=$(stat -c %s /tmp/moc_big6.out) md5=$(md5sum < /tmp/moc_big6.out | cut -c1-12) $(tail -1 gpurun_out/r3_mode_timing.txt)"
done > gpurun_out/final_modes_r3e.log
cut -c1-1000 gpurun_out/final_modes_r3e.log
rm -f $F /tmp/moc_big6.out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "rccl or final_cli or streaming" > gpurun_out/gpu_tests_r3_sub4.log 2>&1 || { tail -30 gpurun_out/gpu_tests_r3_sub4.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r3_sub4.log
