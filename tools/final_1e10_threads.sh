#!/bin/bash
# Host-phase scaling of BASELINE config 5 through the product: 1.0e10 input6-shaped letters (11.2 GB)
# streamed through ./final (--batch-records, csrc/apps/flow_stream.cpp) with THREADS OpenMP threads per
# rank at NPS ranks on the one GPU, rows to /dev/null. One line per run: ranks, threads, wall ms and the
# root's --timing JSON (count / fill / print / kernel phases). The input file is generated once.
#   THREADS="1 2 4 8 16"   NPS="1"   RECORDS=1176470589   BATCH=16777216
set -o pipefail
mkdir -p gpurun_out
F=/tmp/moc_1e10.txt
RECORDS=${RECORDS:-1176470589}
BATCH=${BATCH:-16777216}
if [ ! -s $F ]; then
  timeout -k 10 900 python3 tools/gen_synthetic.py --shape input6 --records $RECORDS --jobs ${GEN_JOBS:-16} --out $F || exit 1
fi
echo "# $(nproc) cpus visible, $(./final --help | tail -1), records=$RECORDS batch=$BATCH"
for np in ${NPS:-1}; do
  for t in ${THREADS:-1 2 4 8 16}; do
    s=$(date +%s%N)
    timeout -k 10 ${RUN_LIMIT:-240} /opt/conda/bin/mpiexec -np $np ./final --timing --device=0 --threads=$t --input=$F \
      --batch-records=$BATCH --output=/dev/null 2> gpurun_out/final_1e10_threads_timing.txt
    rc=$?
    e=$(date +%s%N)
    echo "np=$np threads=$t rc=$rc wall_ms=$(( (e - s) / 1000000 )) $(grep '^{' gpurun_out/final_1e10_threads_timing.txt | tail -1)"
    case $rc in 0) ;; *) tail -5 gpurun_out/final_1e10_threads_timing.txt; rm -f $F; exit $rc;; esac
  done
done
[ "${KEEP:-0}" = 1 ] || rm -f $F
