#!/bin/bash
# The reference's invocation (`mpiexec -np N ./final < inputX.txt`, default flags) after the lean MPI
# topology, next to --mpi-topology=full (MPI's own start-up) and a bare MPI hello-world, N = 1, 2, 4.
set -o pipefail
REPS=${REPS:-9}
MPIEXEC=${MPIEXEC:-/opt/conda/bin/mpiexec}
mkdir -p build gpurun_out
make -s build/mpilib/libmpi.so 2>/dev/null || make -s build
g++ -O2 tools/mpi_hello.cpp -I/opt/conda/include -Lbuild/mpilib -lmpi -Wl,-rpath-link,/opt/conda/lib \
  -Wl,-rpath,$PWD/build/mpilib -o build/mpi_hello || exit 1
stats() { sort -n | awk '{a[NR]=$1} END {printf "median_ms=%d best_ms=%d", a[int((NR+1)/2)], a[1]}'; }
run() {  # run <np> <label> <cmd...>  (stdin from $IN)
  local np=$1 label=$2; shift 2
  local t=() ok=ok
  for r in $(seq 1 $REPS); do
    s=$(date +%s%N)
    timeout -k 10 60 $MPIEXEC -np $np "$@" < $IN > gpurun_out/wt_out.txt 2> gpurun_out/wt_err.txt || ok=FAILED
    e=$(date +%s%N)
    t+=($(( (e - s) / 1000000 )))
  done
  [ -n "$EXPECT" ] && ! cmp -s gpurun_out/wt_out.txt $EXPECT && ok=MISMATCH
  echo "$label np=$np $(printf '%s\n' "${t[@]}" | stats) $ok"
}
echo "# host: $(nproc) cpus visible, OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset}, reps=$REPS, $(./final --help | tail -1)"
for np in ${NPS:-1 2 4}; do
  IN=tests/data/input6.txt EXPECT= run $np "mpi_hello              " build/mpi_hello
  IN=tests/data/input6.txt EXPECT=tests/data/expected/input6.out run $np "final input6 topo=full " ./final --mpi-topology=full
  for i in 1 2 3 4 5 6; do
    IN=tests/data/input$i.txt EXPECT=tests/data/expected/input$i.out run $np "final input$i           " ./final
  done
done
