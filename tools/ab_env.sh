#!/bin/bash
# Interleaved bench.py A/B of one environment setting and/or extra arguments: REPS rounds of "A" (defaults)
# and "B" ($AB_ENV set, $AB_ARGS appended), STEPS
# timed steps each; prints value, mean and p50/p99 step ms, kernel median.
mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-3}); do
  for side in A B; do
    if [ $side = A ]; then envs=""; args=""; else envs="$AB_ENV"; args="${AB_ARGS:-}"; fi
    env $envs timeout -k 10 120 python bench.py --steps ${STEPS:-500} --warmup 20 $args > gpurun_out/ab_env_run.json 2> /dev/null || exit 1
    python - "$side ${envs:-default} $args" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_env_run.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]}: value={d['value'] / 1e9:.2f}G ms/step={d['ms_per_step']:.4f} step_p50_p99={d['rank0_step_ms_p50_p99']} "
      f"kernel_med={d['rank0_kernel_ms_per_step']:.4f} kernel_p90_p99={d['rank0_kernel_ms_p90_p99']}", flush=True)
PY
  done
done
