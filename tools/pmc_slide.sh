#!/bin/bash
# Round-5 roofline rows of the sliding-window tile16 kernel (profiles/roofline_r5.md): throughput, then the
# two SQ counter sets per shape, one shape per pass (the three shapes run the same kernel instance).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5roof
mkdir -p $OUT
timeout -k 10 300 python3 tools/kernel_bench.py limits long20k heavylim long150k --variants slide > $OUT/kb_slide.log 2>&1 || { tail -5 $OUT/kb_slide.log; exit 1; }
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE")
i=10
for shape in limits long20k heavylim; do
  for j in 0 1; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc ${SETS[$j]} --output-format csv -d $OUT/pmc_$i -o k \
      -- python3 tools/kernel_bench.py --min-ms 15 --variants slide $shape > $OUT/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pmc_$i.log; exit 1; }
    echo "pass $i ok ($shape, set $j)"
  done
done
for k in 11 13 15; do python3 tools/pmc_summary.py --tag p$(((k+1)/2)) $OUT/pmc_$k $OUT/pmc_$((k+1)); done > $OUT/pmc_summary_slide.jsonl
cat $OUT/kb_slide.log | grep '^{' | cut -c1-160
