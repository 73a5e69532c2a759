#!/bin/bash
# GPU call: 16 vs 15 OpenMP threads again (bulk, 4 pairs), and 16 threads with a passive wait policy.
set -o pipefail
F=/tmp/moc_big6.txt
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F > /dev/null || exit 1
run() {  # run <label> <env> <flags>
  sleep 3
  s=$(date +%s%N)
  timeout -k 10 300 env $2 /opt/conda/bin/mpiexec -np 1 ./final --timing --input=$F --output=/tmp/moc_big6.out $3 \
    2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "$1 wall_ms=$(( (e - s) / 1000000 )) $(tail -1 gpurun_out/r3_timing.txt)"
  rm -f /tmp/moc_big6.out
}
for r in 1 2 3 4; do
  run "t16" "X=1" "--threads=16"
  run "t15" "X=1" "--threads=15"
  run "t16passive" "OMP_WAIT_POLICY=passive" "--threads=16"
done > gpurun_out/final_modes_1.1G_r3o_threads2.log
python3 - <<'PY'
import json
for line in open('gpurun_out/final_modes_1.1G_r3o_threads2.log'):
    head, rest = line.split(' {', 1)
    t = json.loads('{' + rest)['timing']
    print(head, {k: round(t[k], 1) for k in ['fill_ms', 'pin_ms', 'compute_ms', 'print_ms'] if k in t})
PY
rm -f $F
