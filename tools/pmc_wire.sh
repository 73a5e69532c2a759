# round 5: counters of the P33 lane-direct swipe kernel against the byte-letter one (input6, wire lengths/results)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5w
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY \
  --output-format csv -d gpurun_out/r5w/p1 -o k -- python3 tools/kernel_bench.py --min-ms 15 input6 --variants wire,wirebytes > gpurun_out/r5w/p1.log 2>&1 || { tail -5 gpurun_out/r5w/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/r5w/p2 -o k -- python3 tools/kernel_bench.py --min-ms 15 input6 --variants wire,wirebytes > gpurun_out/r5w/p2.log 2>&1 || { tail -5 gpurun_out/r5w/p2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/r5w/p1 gpurun_out/r5w/p2 > gpurun_out/r5w/summary.jsonl
python3 - <<'PY'
import json
for l in open("gpurun_out/r5w/summary.jsonl"):
    d = json.loads(l)
    if "swipe_direct" in d["kernel"]:
        n = d["dispatches"]
        print(d["kernel"].split("(")[0], {k: round(v / n / 1e6, 3) for k, v in d.items() if isinstance(v, (int, float)) and k != "dispatches" and v})
PY
