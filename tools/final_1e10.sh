#!/bin/bash
# BASELINE config 5 through the product: 1.0e10 input6-shaped letters (1.18 G records, 11.2 GB of text)
# streamed through ./final on one GPU in batches of --batch-records (persistent page-locked rings,
# csrc/apps/flow_stream.cpp), rows formatted and written to /dev/null (40 GB of text would not fit the
# box's /tmp). One line: wall ms + the --timing JSON.
set -o pipefail
mkdir -p gpurun_out
F=/tmp/moc_1e10.txt
RECORDS=${RECORDS:-1176470589}
timeout -k 10 900 python3 tools/gen_synthetic.py --shape input6 --records $RECORDS --jobs ${GEN_JOBS:-16} --out $F || exit 1
s=$(date +%s%N)
timeout -k 10 600 /opt/conda/bin/mpiexec -np 1 ./final --timing --device=0 --input=$F \
  --batch-records=${BATCH:-16777216} --output=/dev/null 2> gpurun_out/final_1e10_timing.txt
rc=$?
e=$(date +%s%N)
echo "records=$RECORDS batch=${BATCH:-16777216} rc=$rc wall_ms=$(( (e - s) / 1000000 )) $(tail -1 gpurun_out/final_1e10_timing.txt)"
rm -f $F
exit $rc
