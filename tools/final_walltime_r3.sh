#!/bin/bash
# The reference's own invocation, default flags: `mpiexec -np N ./final < inputX.txt` (makefile:10-11),
# X = 1..6, N = 1, 2 — median and best of REPS runs, output checked against the goldens — next to a bare
# MPI hello-world (tools/mpi_hello.cpp) under the same mpiexec: the part of the wall that is MPI's.
set -o pipefail
REPS=${REPS:-9}
MPIEXEC=${MPIEXEC:-/opt/conda/bin/mpiexec}
mkdir -p build gpurun_out
make -s build/mpilib/libmpi.so 2>/dev/null || make -s build
g++ -O2 tools/mpi_hello.cpp -I/opt/conda/include -Lbuild/mpilib -lmpi -Wl,-rpath-link,/opt/conda/lib \
  -Wl,-rpath,$PWD/build/mpilib -o build/mpi_hello || exit 1
stats() {  # "median best" of the ms values on stdin
  sort -n | awk '{a[NR]=$1} END {printf "median_ms=%d best_ms=%d", a[int((NR+1)/2)], a[1]}'
}
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
echo "# host: $(nproc) cpus visible, OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset}, reps=$REPS"
for np in 1 2; do
  IN=tests/data/input6.txt EXPECT= run $np "mpi_hello        " build/mpi_hello
  for i in 1 2 3 4 5 6; do
    IN=tests/data/input$i.txt EXPECT=tests/data/expected/input$i.out run $np "final input$i     " ./final
  done
done
