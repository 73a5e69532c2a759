#!/bin/bash
# Root cause of RCCL communicator start-up on the MI355X box (one rank, one GPU): phase timings of a bare
# probe (tools/rccl_init_probe.cpp), the same with a busy OpenMP team on other threads (./final's
# connect-overlaps-parse case), RCCL's own INIT log with timestamps, and a rocprofv3 HIP API trace of the
# probe (which runtime calls the time goes to). Output: gpurun_out/rccl_rootcause/*.
set -o pipefail
O=gpurun_out/rccl_rootcause
mkdir -p $O
P=build/rccl_init_probe
export TMPDIR=/tmp
echo "== cold (first run on the box)"; timeout -k 10 90 $P || exit 1
echo "== warm"; timeout -k 10 90 $P || exit 1
echo "== busy team of 16 spinning"; timeout -k 10 120 $P --busy=16 || exit 1
echo "== busy team of 16, 1 ms sleeps"; timeout -k 10 120 $P --busy=16 --passive || exit 1
echo "== busy team of 8"; timeout -k 10 120 $P --busy=8 || exit 1
echo "== HIP_ENABLE_DEFERRED_LOADING=0"; HIP_ENABLE_DEFERRED_LOADING=0 timeout -k 10 120 $P || exit 1
echo "== NCCL_MAX_NCHANNELS=1"; NCCL_MAX_NCHANNELS=1 timeout -k 10 90 $P || exit 1
echo "== INIT log with timestamps"
NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,ENV,GRAPH,ALLOC NCCL_DEBUG_TIMESTAMP_LEVELS=ALL \
  NCCL_DEBUG_TIMESTAMP_FORMAT="[%T.%6f] " timeout -k 10 90 $P > $O/debug_stdout.txt 2> $O/debug_stderr.txt || exit 1
cat $O/debug_stdout.txt
grep -c . $O/debug_stderr.txt
echo "== rocprofv3 HIP API + kernel trace"
cd /tmp && timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o probe \
  -- $GRAFT_REPO_ROOT/$P > $GRAFT_REPO_ROOT/$O/prof_stdout.txt 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof_stdout.txt; exit 1; }
cd $GRAFT_REPO_ROOT
grep -v '^$' $O/prof_stdout.txt | grep -E "ms$|TOTAL" || true
find $O/prof -name '*stats*.csv' | head
