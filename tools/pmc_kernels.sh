# SQ counters of the device-resident kernels (tools/kernel_bench.py), one rocprofv3 pass per shape set.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
  SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_kernels -o k \
  -- python3 tools/kernel_bench.py ${SHAPES:-input6 input1} > gpurun_out/pmc_kernels.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES \
  GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_kernels2 -o k \
  -- python3 tools/kernel_bench.py ${SHAPES:-input6 input1} > gpurun_out/pmc_kernels2.log 2>&1
