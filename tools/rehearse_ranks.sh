#!/bin/bash
# Multi-rank rehearsal on the one MI355X of a gpurun box, before any 8-GPU node runs it:
#   1. bench.py --gpus $NR --allow-shared-gpu --dist-backend gloo at the default per-rank size (NR x 285 M
#      letters): the self-launch, the per-rank fields of the scaling record, the verification at NR ranks.
#   2. ./final at 1.14 G letters (134 M input6-shaped records, 1.28 GB of text) on NPS ranks, all on
#      --device=0, bulk and streamed (--batch-records=16777216): output md5 against np 1, per-rank --timing.
# FINAL_WALL=1 keeps the bench's ./final wall-clock fields (np = NR ranks on the same GPU: NR <= 4 here, the
# box allows 16 GPU processes). STEP=bench|final|all (default all). Every GPU step has its own time limit; the script stops at the first
# failure.
set -o pipefail
mkdir -p gpurun_out
NR=${NR:-8}
NPS=${NPS:-"1 4 8"}
STEP=${STEP:-all}
if [ "$STEP" = all ] || [ "$STEP" = bench ]; then
  echo "=== bench.py --gpus $NR (gloo, shared GPU)"
  timeout -k 10 600 python3 bench.py --gpus $NR --allow-shared-gpu --dist-backend gloo --steps ${STEPS:-20} \
    --warmup 3 --final-wall ${FINAL_WALL:-0} > gpurun_out/rehearse_bench_$NR.json 2> gpurun_out/rehearse_bench_$NR.err || {
    tail -20 gpurun_out/rehearse_bench_$NR.err; exit 1; }
  cat gpurun_out/rehearse_bench_$NR.json
fi
[ "$STEP" = bench ] && exit 0
F=/tmp/moc_big6.txt
O=/tmp/moc_big6.out
timeout -k 10 600 python3 tools/gen_synthetic.py --shape input6 --records ${RECORDS:-134217728} --jobs 16 --out $F || exit 1
ref=""
for np in $NPS; do
  for mode in "" "--batch-records=16777216"; do
    rm -f $O
    s=$(date +%s%N)
    timeout -k 10 300 /opt/conda/bin/mpiexec -np $np ./final --timing --device=0 --input=$F --output=$O $mode \
      2> gpurun_out/rehearse_final_timing.txt
    rc=$?
    e=$(date +%s%N)
    [ $rc = 0 ] || { tail -20 gpurun_out/rehearse_final_timing.txt; rm -f $F $O; exit $rc; }
    sum=$(md5sum $O | cut -c1-32)
    [ -z "$ref" ] && ref=$sum
    same=$([ "$sum" = "$ref" ] && echo md5_equal || echo MD5_DIFFERS)
    echo "np=$np mode='${mode:-bulk}' rc=$rc wall_ms=$(( (e - s) / 1000000 )) md5=$sum $same $(grep '^{' gpurun_out/rehearse_final_timing.txt | tail -1)"
  done
done
rm -f $F $O
