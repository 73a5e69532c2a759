# End-to-end wall-clock of ./final on the reference inputs (the reference's sequential
# algorithm takes 0.016-14.4 s on them). One line per run: input, ranks, wall seconds, --timing JSON.
set -e
BACKEND=${BACKEND:-auto}
mkdir -p gpurun_out
for np in 1 2; do
  for i in 1 2 3 4 5 6; do
    s=$(date +%s%N)
    timeout -k 10 120 /opt/conda/bin/mpiexec -np $np ./final --backend=$BACKEND --timing --device=0 \
      --input=tests/data/input$i.txt > gpurun_out/final_out_$i.txt 2> gpurun_out/final_timing_$i.txt
    e=$(date +%s%N)
    cmp -s gpurun_out/final_out_$i.txt tests/data/expected/input$i.out && ok=ok || ok=MISMATCH
    echo "input$i backend=$BACKEND np=$np wall_ms=$(( (e - s) / 1000000 )) $ok $(tail -1 gpurun_out/final_timing_$i.txt)"
  done
done
