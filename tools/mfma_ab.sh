# A/B of the long-record sweep: packed-int16 VALU (tile16) vs matrix cores (MOC_MFMA=1), device-resident
# (tools/kernel_bench.py, >= 60 ms of kernel time per shape), then SQ counters of each variant in passes
# of <= 8 SQ counters (rocprofv3 --pmc; no tracing domains mixed in).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
SHAPES=${SHAPES:-input3 input4}
timeout -k 10 300 python3 tools/kernel_bench.py --variants tile16,mfma $SHAPES > gpurun_out/mfma_ab_bench.log 2>&1
for v in tile16 mfma; do
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d gpurun_out/mfma_pmc_$v -o p1 \
    -- python3 tools/kernel_bench.py --variants $v --min-ms 5 $SHAPES > gpurun_out/mfma_pmc_$v.log 2>&1
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
    --output-format csv -d gpurun_out/mfma_pmc2_$v -o p2 \
    -- python3 tools/kernel_bench.py --variants $v --min-ms 5 $SHAPES > gpurun_out/mfma_pmc2_$v.log 2>&1
done
