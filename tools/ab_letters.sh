#!/bin/bash
# Interleaved A/B of the bench's letter codes (P33 vs P24) on one GPU: REPS rounds of each, STEPS timed
# steps per run; prints the JSON fields that decide it (value, ms/step, kernel median and range, H2D bytes).
mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-3}); do
  for L in p33 p24; do
    timeout -k 10 120 python bench.py --steps ${STEPS:-200} --warmup 20 --letters $L ${EXTRA:-} > gpurun_out/ab_letters_run.json 2> /dev/null || exit 1
    python - "$L" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_letters_run.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]} value={d['value'] / 1e9:.2f}G ms/step={d['ms_per_step']:.4f} kernel_med={d['rank0_kernel_ms_per_step']:.4f} "
      f"kernel_min_max={d['rank0_kernel_ms_min_max']} h2d={d['rank0_h2d_bytes_per_step']} verified={d['verified']}", flush=True)
PY
  done
done
