#!/bin/bash
# GPU call: when does the HIP runtime come up inside ./final (runtime_up_since_start_ms), and does malloc's
# mmap/munmap churn (glibc's mmap threshold) slow it? 1.14 G letters bulk + streamed, interleaved.
set -o pipefail
F=/tmp/moc_big6.txt
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F > /dev/null || exit 1
TUNE="GLIBC_TUNABLES=glibc.malloc.mmap_threshold=33554432:glibc.malloc.trim_threshold=4294967296"
run() {  # run <label> <env> <flags>
  sleep 3
  s=$(date +%s%N)
  timeout -k 10 300 env $2 /opt/conda/bin/mpiexec -np 1 ./final --timing --input=$F --output=/tmp/moc_big6.out $3 \
    2> gpurun_out/r3_timing.txt || { tail -5 gpurun_out/r3_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "$1 wall_ms=$(( (e - s) / 1000000 )) $(tail -1 gpurun_out/r3_timing.txt)"
  rm -f /tmp/moc_big6.out
}
for r in 1 2 3; do
  run "bulk default" "X=1" ""
  run "bulk mmapthr" "$TUNE" ""
  run "stream default" "X=1" "--batch-records=16777216"
  run "stream mmapthr" "$TUNE" "--batch-records=16777216"
done > gpurun_out/final_modes_1.1G_r3p_rtup.log
python3 - <<'PY'
import json
for line in open('gpurun_out/final_modes_1.1G_r3p_rtup.log'):
    head, rest = line.split(' {', 1)
    js = json.loads('{' + rest)
    t = js['timing']
    print(head, 'rt_up', js.get('runtime_up_since_start_ms'), {k: round(t[k], 1) for k in ['read_ms', 'count_ms', 'fill_ms', 'pin_ms', 'compute_ms', 'print_ms'] if k in t}, 'ring_pin', js.get('rank0_fill_split_ms', {}).get('ring_pin'))
PY
rm -f $F
