#!/bin/bash
# GPU call: two ranks on the one GPU (--device=0) at 1.14 G letters, bulk and streamed, output checked
# against the 1-rank run's md5 (the kfd start-up, the overlapped engine and quick exit at np 2).
set -o pipefail
F=/tmp/moc_big6.txt
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F > /dev/null || exit 1
for run in "1|" "2|" "2|--batch-records=16777216" "2|--parallel-print"; do
  np=${run%%|*}; mode=${run#*|}
  sleep 3
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np $np ./final --timing --device=0 --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "np=$np mode='$mode' wall_ms=$(( (e - s) / 1000000 )) md5=$(md5sum < /tmp/moc_big6.out | cut -c1-12) $(tail -1 gpurun_out/r3_timing.txt)"
  rm -f /tmp/moc_big6.out
done > gpurun_out/final_np2_1.1G_r3.log
grep -o "np=[0-9] mode='[^']*' wall_ms=[0-9]* md5=[0-9a-f]*" gpurun_out/final_np2_1.1G_r3.log
rm -f $F
