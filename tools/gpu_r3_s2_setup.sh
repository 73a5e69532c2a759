#!/bin/bash
# GPU call: where `final`'s setup phase waits after the kfd start-up (gpu count / rank create / reduce),
# 1.14 G input6-shaped letters, bulk and streamed.
set -o pipefail
mkdir -p gpurun_out
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F > /dev/null || exit 1
for mode in "" "" "--batch-records=16777216" "--gpu-prewarm-bytes=0"; do
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np 1 ./final --timing --device=0 --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "1.14G mode='$mode' wall_ms=$(( (e - s) / 1000000 )) md5=$(md5sum < /tmp/moc_big6.out | cut -c1-12) $(tail -1 gpurun_out/r3_timing.txt)"
  rm -f /tmp/moc_big6.out
done > gpurun_out/final_modes_1.1G_r3k_setup.log
grep -o "1.14G mode='[^']*' wall_ms=[0-9]*\|\"setup_ms\": [0-9.]*\|\"rank0_setup_split_ms\": {[^}]*}\|\"engine_wait_ms\": [0-9.]*" gpurun_out/final_modes_1.1G_r3k_setup.log
rm -f $F
