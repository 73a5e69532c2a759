#!/bin/bash
# GPU call: where the node streaming flow's fill time goes (ring allocation / encode / lengths), for
# 16.7 M- and 67 M-record batches at 1.14 G letters.
set -o pipefail
mkdir -p gpurun_out
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F || exit 1
for mode in "" "--batch-records=16777216" "--batch-records=16777216" "--batch-records=4194304"; do
  rm -f /tmp/moc_big6.out
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np 1 ./final --timing --device=0 --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_mode_timing.txt || { tail -5 gpurun_out/r3_mode_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "mode='$mode' wall_ms=$(( (e - s) / 1000000 )) out_bytes=$(stat -c %s /tmp/moc_big6.out) md5=$(md5sum < /tmp/moc_big6.out | cut -c1-12) $(tail -1 gpurun_out/r3_mode_timing.txt)"
done > gpurun_out/final_modes_r3k.log
grep -o "mode='[^']*'\|\"fill_ms\": [0-9.]*\|\"count_ms\": [0-9.]*\|\"rank0_fill_split_ms\": {[^}]*}\|\"pin_ms\": [0-9.]*\|\"wall_s\": [0-9.]*" gpurun_out/final_modes_r3k.log
rm -f $F /tmp/moc_big6.out
