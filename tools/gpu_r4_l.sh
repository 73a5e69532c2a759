#!/bin/bash
# Round 4 GPU call L: the first host->device copy's cost by size and copy path (tools/copy_path_probe.hip),
# each size in a fresh process, with SDMA allowed and with HSA_ENABLE_SDMA=0.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/copy_path_probe.log
: > $out
for b in 4096 65536 131072 1048576 16777216; do
  timeout -k 10 30 build/copy_path_probe $b >> $out 2>&1 || exit 1
  HSA_ENABLE_SDMA=0 timeout -k 10 30 build/copy_path_probe $b >> $out 2>&1 || exit 1
done
cat $out
