#!/bin/bash
# Round-5 roofline counters (profiles/roofline_r5.md): SQ counters of every search kernel, device-resident
# (tools/kernel_bench.py), one rocprofv3 pass per counter set, each with its own time limit.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5
SHAPES=${SHAPES:-"input6 input1 mid input3 input4 long20k"}
# plain throughput first (no counters), every shape
timeout -k 10 300 python3 tools/kernel_bench.py $SHAPES > gpurun_out/r5/kb_all.log 2>&1 || { tail -5 gpurun_out/r5/kb_all.log; exit 1; }
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/r5/pmc_avail.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" gpurun_out/r5/pmc_avail.txt | sort -u | tr '\n' ' ' | head -c 4000 > gpurun_out/r5/pmc_sq_names.txt
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/r5/pmc_$i -o k \
    -- python3 tools/kernel_bench.py --min-ms 15 $SHAPES > gpurun_out/r5/pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/r5/pmc_$i.log; exit 1; }
  echo "pass $i ok"
done
python3 tools/pmc_summary.py gpurun_out/r5/pmc_1 gpurun_out/r5/pmc_2 > gpurun_out/r5/pmc_summary.jsonl
python3 tools/roofline.py gpurun_out/r5/pmc_summary.jsonl gpurun_out/r5/pmc_1.log gpurun_out/r5/kb_all.log \
  > gpurun_out/r5/roofline.md
cat gpurun_out/r5/roofline.md
