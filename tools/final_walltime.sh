#!/bin/bash
# Wall-clock of the reference's own invocation, `mpiexec -np N ./final [EXTRA] < inputX.txt`
# (/root/reference/makefile:10-11): median and best of REPS launches, output compared with the golden,
# next to a bare MPI hello-world (tools/mpi_hello.cpp) under the same mpiexec — the floor of any program
# that starts MPI — and a HIP hello-world (tools/hip_hello.hip: MPI + runtime + one queue + one empty
# kernel) — the floor of any program that starts MPI and runs a kernel.
#   NPS="1 2 4"      rank counts                 INPUTS="1 2 3 4 5 6"   reference inputs
#   EXTRA="--backend=hip"  flags for ./final      REPS=9                 launches per point
#   HELLO=1          also time the MPI hello-world (0: skip)
#   TIMING=1         keep the last launch's --timing JSON per point (adds --timing to EXTRA)
#   SPACING=0        seconds between launches: back-to-back GPU processes wait in the kernel driver for
#                    the previous one's teardown (profiles/hip_init_trace_b2b.log); 1-2 s gives the idle floor
set -o pipefail
REPS=${REPS:-9}
NPS=${NPS:-"1 2 4"}
INPUTS=${INPUTS:-"1 2 3 4 5 6"}
HELLO=${HELLO:-1}
MPIEXEC=${MPIEXEC:-/opt/conda/bin/mpiexec}
EXTRA=${EXTRA:-}
[ "${TIMING:-0}" = 1 ] && EXTRA="$EXTRA --timing"
mkdir -p build gpurun_out
if [ "$HELLO" = 1 ]; then
  make -s build/mpilib/libmpi.so 2>/dev/null || make -s build
  g++ -O2 tools/mpi_hello.cpp -I/opt/conda/include -Lbuild/mpilib -lmpi -Wl,-rpath-link,/opt/conda/lib \
    -Wl,-rpath,$PWD/build/mpilib -o build/mpi_hello || exit 1
  [ -x build/hip_hello ] || hipcc --offload-arch=gfx950 -O2 tools/hip_hello.hip -I/opt/conda/include -Lbuild/mpilib -lmpi \
    -Wl,-rpath-link,/opt/conda/lib -Wl,-rpath,$PWD/build/mpilib -o build/hip_hello || exit 1
fi
stats() { sort -n | awk '{a[NR]=$1} END {printf "median_ms=%d best_ms=%d", a[int((NR+1)/2)], a[1]}'; }
run() {  # run <np> <label> <cmd...>  (stdin from $IN)
  local np=$1 label=$2; shift 2
  local t=() ok=ok
  for r in $(seq 1 $REPS); do
    s=$(date +%s%N)
    timeout -k 10 60 $MPIEXEC -np $np "$@" < $IN > gpurun_out/wt_out.txt 2> gpurun_out/wt_err.txt || ok=FAILED
    e=$(date +%s%N)
    t+=($(( (e - s) / 1000000 )))
    [ "${SPACING:-0}" != 0 ] && sleep "$SPACING"
  done
  [ -n "$EXPECT" ] && ! cmp -s gpurun_out/wt_out.txt $EXPECT && ok=MISMATCH
  local extra=""
  [ "${TIMING:-0}" = 1 ] && extra=" $(grep -v '^{' gpurun_out/wt_err.txt | tr '\n' ' ' | cut -c1-600) $(grep '^{' gpurun_out/wt_err.txt | tail -1)"
  echo "$label np=$np $(printf '%s\n' "${t[@]}" | stats) $ok$extra"
}
echo "# host: $(nproc) cpus visible, OMP_NUM_THREADS=${OMP_NUM_THREADS:-unset}, reps=$REPS, extra='$EXTRA', $(./final --help | tail -1)"
for np in $NPS; do
  [ "$HELLO" = 1 ] && IN=tests/data/input6.txt EXPECT= run $np "mpi_hello    " build/mpi_hello
  [ "$HELLO" = 1 ] && IN=tests/data/input6.txt EXPECT= run $np "hip_hello    " build/hip_hello \
    && echo "  hip_hello last launch: $(grep '^{' gpurun_out/wt_err.txt | tail -1)"
  for i in $INPUTS; do
    IN=tests/data/input$i.txt EXPECT=tests/data/expected/input$i.out run $np "final input$i" ./final $EXTRA
  done
done
