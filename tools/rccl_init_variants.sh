#!/bin/bash
# RCCL start-up variants (tools/rccl_init_probe.cpp): load order, a warm-up communicator on a helper thread,
# teardown by destroy / abort / process exit. Warm page cache (one run first).
set -o pipefail
P=build/rccl_init_probe
timeout -k 10 90 $P > /dev/null || exit 1
for args in "" "--dlopen-first" "--warm" "--warm --dlopen-first" "--teardown=abort" "--teardown=none"; do
  echo "== $args"
  s=$(date +%s%N)
  timeout -k 10 90 $P $args || exit 1
  e=$(date +%s%N)
  echo "process wall (incl. exit) $(( (e - s) / 1000000 )) ms"
done
