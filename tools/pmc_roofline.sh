#!/bin/bash
# The roofline (profiles/roofline_r5.md, profiles/roofline_r6.md): the instruction-rate probe, plain throughput of every search
# kernel (tools/kernel_bench.py, device-resident), then SQ counters in passes of their own, each with its own
# time limit. Shapes run in separate passes so each kernel instance's counters belong to one shape.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${OUT:-gpurun_out/roofline}
mkdir -p $OUT
timeout -k 10 180 build/isa_peak 20000 > $OUT/isa_peak.log 2>&1 || { tail -5 $OUT/isa_peak.log; exit 1; }
timeout -k 10 300 python3 tools/kernel_bench.py input6 input1 mid input3 limits input4 long20k heavy3 heavy4 heavylim > $OUT/kb_all.log 2>&1 || { tail -5 $OUT/kb_all.log; exit 1; }
timeout -k 10 200 python3 tools/kernel_bench.py input6 input1 --variants wire >> $OUT/kb_all.log 2>&1 || { tail -5 $OUT/kb_all.log; exit 1; }
SETS=("SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE")
i=0
for args in "input6 input1 mid" "input3 limits" "input4 long20k" "input6 input1 --variants wire" "heavy3 heavy4" "heavylim"; do
  for j in 0 1; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc ${SETS[$j]} --output-format csv -d $OUT/pmc_$i -o k \
      -- python3 tools/kernel_bench.py --min-ms 15 $args > $OUT/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/pmc_$i.log; exit 1; }
    echo "pass $i ok ($args, set $j)"
  done
done
for k in 1 3 5 7 9 11; do python3 tools/pmc_summary.py --tag p$(((k+1)/2)) $OUT/pmc_$k $OUT/pmc_$((k+1)); done > $OUT/pmc_summary.jsonl
python3 tools/roofline.py $OUT/pmc_summary.jsonl $OUT/kb_all.log > $OUT/roofline.md
cat $OUT/roofline.md
