#!/bin/bash
# Per-step variance of the headline bench with the GPU's clocks / power / temperature sampled alongside
# (tools/gpu_sampler.py) and the host's memory-management state recorded before and after, so slow steps
# can be attributed to the link, the GPU's clocks or the host's pages. STEPS timed steps (default 2000).
set -o pipefail
mkdir -p gpurun_out
STEPS=${STEPS:-2000}
OUT=gpurun_out/step_variance
mkdir -p $OUT
host_state() {
  for f in /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag \
           /proc/sys/kernel/numa_balancing /sys/kernel/mm/transparent_hugepage/khugepaged/defrag; do
    echo "$f: $(cat $f 2>/dev/null)"
  done
  grep -E "^(numa_hint_faults|numa_pages_migrated|pgmigrate_success|thp_fault_alloc|thp_collapse_alloc|compact_stall|pgfault|pgmajfault) " /proc/vmstat
  grep -E "MHz" /proc/cpuinfo | awk '{s+=$4; n++} END {printf "cpu MHz mean over %d cpus: %.0f\n", n, s/n}'
}
host_state > $OUT/host_before.txt
BUS=$(python3 -c "
import os,glob
for d in sorted(glob.glob('/sys/class/drm/card*/device')):
    if os.path.exists(os.path.join(d,'pp_dpm_sclk')):
        print(os.path.basename(os.path.realpath(d))); break")
timeout -k 5 $((STEPS / 100 + 200)) python3 tools/gpu_sampler.py --bus "$BUS" --period 0.01 --out $OUT/gpu_samples.jsonl &
SAMPLER=$!
timeout -k 10 $((STEPS / 100 + 180)) python3 bench.py --steps $STEPS --warmup 20 --final-wall 0 --dump-steps $OUT/steps.json \
  > $OUT/bench.json 2> $OUT/bench.err
rc=$?
kill $SAMPLER 2>/dev/null; wait $SAMPLER 2>/dev/null
host_state > $OUT/host_after.txt
cat $OUT/bench.json
python3 tools/step_variance_report.py $OUT
exit $rc
