#!/bin/bash
# GPU call: does the HIP runtime's start-up (on a helper thread) lose its CPU to the 16 OpenMP threads of the
# read/count/encode? 1.14 G letters bulk and streamed at 16 vs 15 threads (pin_ms / ring_pin = the wait).
set -o pipefail
mkdir -p gpurun_out
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F > /dev/null || exit 1
for mode in ${MODES:-"--threads=16" "--threads=15" "--threads=16" "--threads=15" "--threads=16 --batch-records=16777216" "--threads=15 --batch-records=16777216" "--threads=16 --batch-records=16777216" "--threads=15 --batch-records=16777216"}; do
  sleep 3
  s=$(date +%s%N)
  timeout -k 10 300 env $ENVS /opt/conda/bin/mpiexec -np 1 ./final --timing --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "1.14G mode='$mode' wall_ms=$(( (e - s) / 1000000 )) $(tail -1 gpurun_out/r3_timing.txt)"
  rm -f /tmp/moc_big6.out
done > gpurun_out/${OUT:-final_modes_1.1G_r3n_threads.log}
python3 - <<'PY'
import json
for line in open('gpurun_out/${OUT:-final_modes_1.1G_r3n_threads.log}'):
    head, rest = line.split(' {', 1)
    js = json.loads('{' + rest)
    t = js['timing']
    keys = ['read_ms', 'count_ms', 'fill_ms', 'pin_ms', 'compute_ms', 'print_ms']
    print(head, {k: round(t[k], 1) for k in keys if k in t}, 'ring', js.get('rank0_fill_split_ms', {}).get('ring_pin'), 'wall_s', js['wall_s'])
PY
rm -f $F
