#!/bin/bash
# Runs GPU steps in order on a gpurun box; stops at the first fatal status (fault/abort/segv/timeout)
# so nothing else touches a GPU that may be in a bad state. Usage: tools/gpu_steps.sh "name:secs:cmd" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 15 "gpurun_out/$name.log"
  case $rc in
    124|134|137|139|143) echo "FATAL status $rc in step $name: stopping"; exit $rc;;
  esac
done
exit 0
