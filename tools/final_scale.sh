# End-to-end ./final at scale on one GPU (BASELINE.json "wall-clock" with 10^9 letters): generate an
# input6-shaped file, then time the whole job (read + parse + search + print to a file) and its phases.
# NP=2 runs two ranks on the one GPU (--device=0): each encodes, pins and streams its own slice.
set -e
mkdir -p gpurun_out
F=/tmp/moc_big6.txt
timeout -k 10 600 python3 tools/gen_synthetic.py --shape input6 --records ${RECORDS:-134217728} --jobs ${GEN_JOBS:-16} --out $F
# "--output": the root writes the file itself (parallel pwrite) instead of stdout, which mpiexec's proxy
# forwards through a pipe
# MODES: '|'-separated flag sets (each may hold several flags)
IFS='|' read -r -a MODE_LIST <<< "${MODES:- |--output=/tmp/moc_big6.out|--output=/tmp/moc_big6.out --gpu-prewarm-bytes=0|--batch-records=16777216}"
for np in ${NPS:-1}; do
for mode in "${MODE_LIST[@]}"; do
  rm -f /tmp/moc_big6.out  # untimed: dropping the previous 4.6 GB output
  so=/tmp/moc_big6.out
  case "$mode" in --output=*) so=/dev/null;; esac
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np $np ./final --timing --device=0 --input=$F $mode > $so \
    2> gpurun_out/final_scale_timing.txt
  e=$(date +%s%N)
  echo "np=$np mode='$mode' wall_ms=$(( (e - s) / 1000000 )) out_bytes=$(stat -c %s /tmp/moc_big6.out) $(tail -1 gpurun_out/final_scale_timing.txt)"
done
done
head -c 300 /tmp/moc_big6.out
rm -f $F /tmp/moc_big6.out
