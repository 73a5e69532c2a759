#!/bin/bash
# RCCL communicator start-up cost inside ./final's sliced path (--collectives=rccl), one rank, one GPU.
# fill_ms holds the wait for ncclCommInitRank (started on a helper thread at set-up); the same job with
# MPI collectives has fill_ms ~0.5. Each variant is one env setting for RCCL (channel caps, topology).
mkdir -p gpurun_out
run() {
  local s e t
  s=$(date +%s%N)
  env "$@" timeout -k 10 60 /opt/conda/bin/mpiexec -np 1 ./final --backend=hip --collectives=${COLL:-rccl} --timing \
    --input=tests/data/input6.txt > /dev/null 2> gpurun_out/rccl_probe_timing.txt || { echo "FAILED: $*"; tail -5 gpurun_out/rccl_probe_timing.txt; return 1; }
  e=$(date +%s%N)
  t=$(tail -1 gpurun_out/rccl_probe_timing.txt)
  echo "$* wall_ms=$(( (e - s) / 1000000 )) $(grep -o '"fill_ms": [0-9.]*' <<< "$t") $(grep -o '"collectives": "[a-z]*"' <<< "$t")"
}
COLL=mpi run X=1 || exit 1
run X=1 || exit 1
run NCCL_MAX_NCHANNELS=2 || exit 1
run NCCL_MAX_NCHANNELS=2 NCCL_MIN_NCHANNELS=1 NCCL_IB_DISABLE=1 || exit 1
run NCCL_MAX_NCHANNELS=2 NCCL_IB_DISABLE=1 NCCL_SOCKET_IFNAME=lo RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0 || exit 1
run NCCL_MAX_NCHANNELS=2 NCCL_IB_DISABLE=1 NCCL_SOCKET_IFNAME=lo NCCL_RAS_ENABLE=0 NCCL_PROXY_APPEND_BATCH_SIZE=1 || exit 1
run NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,ENV NCCL_MAX_NCHANNELS=2 NCCL_IB_DISABLE=1 NCCL_SOCKET_IFNAME=lo || exit 1
grep -E "Init (START|COMPLETE)|init.cc.*ms|Time" gpurun_out/rccl_probe_timing.txt | cut -c1-200 | tail -20
