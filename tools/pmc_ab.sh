#!/bin/bash
# SQ counters of the device-resident kernels (tools/kernel_bench.py) for one or more builds of libmoc.so
# (MOC_LIB_PATH), two rocprofv3 passes of <= 8 SQ counters each per build.
#   LIBS="build/ab_base/libmoc.so mpi_openmp_cuda_amd/lib/libmoc.so"  SHAPES="input6 input1"  TAG=r4
#   VARIANTS=tile16,wire (kernel_bench --variants: the byte and P33 wire forms of each shape)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LIBS=${LIBS:-mpi_openmp_cuda_amd/lib/libmoc.so}
i=0
for lib in $LIBS; do
  d=gpurun_out/pmc_${TAG:-ab}_$i
  echo "# lib $i: $lib -> $d"
  MOC_LIB_PATH=$PWD/$lib timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d $d/p1 -o k \
    -- python3 tools/kernel_bench.py --min-ms 20 ${VARIANTS:+--variants $VARIANTS} ${SHAPES:-input6 input1} > $d.p1.log 2>&1 || exit 1
  MOC_LIB_PATH=$PWD/$lib timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_LDS \
    SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY --output-format csv -d $d/p2 -o k \
    -- python3 tools/kernel_bench.py --min-ms 20 ${VARIANTS:+--variants $VARIANTS} ${SHAPES:-input6 input1} > $d.p2.log 2>&1 || exit 1
  python3 tools/pmc_summary.py $d/p1 $d/p2
  i=$((i + 1))
done
