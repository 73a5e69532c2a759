# SQ counters of the swipe kernel, device-resident (tools/kernel_bench.py input6) and streaming from host
# memory (bench.py): one rocprofv3 pass of <= 8 SQ counters each.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_swipe_dev -o p \
  -- python3 tools/kernel_bench.py --min-ms 20 input6 > gpurun_out/pmc_swipe_dev.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS \
  SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/pmc_swipe_dev2 -o p \
  -- python3 tools/kernel_bench.py --min-ms 20 input6 > gpurun_out/pmc_swipe_dev2.log 2>&1
