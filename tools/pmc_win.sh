# round 5: counters of the widened-window tile16 sweep against the whole byte-pair image (input4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r5win
mkdir -p $OUT
for mode in 1 0; do
  MOC_TILE16_WINWIDE=$mode timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_SMEM \
    --output-format csv -d $OUT/p$mode -o k -- python3 tools/kernel_bench.py --min-ms 15 input4 > $OUT/p$mode.log 2>&1 || { tail -5 $OUT/p$mode.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/p$mode > $OUT/s$mode.jsonl
  python3 - $OUT/s$mode.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    n = d["dispatches"]
    print(d["kernel"].split("(")[0][-60:], n, {k: round(v / n / 1e6, 3) for k, v in d.items() if isinstance(v, (int, float)) and k not in ("dispatches",) and not k.endswith("cycle") and v})
PY
done
