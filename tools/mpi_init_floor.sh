#!/bin/bash
# How far below the lean topology (-x86,-linuxio) MPI_Init can go on the box: the linux component alone vs
# the no_os fallback, at 1/2/8 ranks (tools/mpi_startup_probe.cpp; rank 0's MPI_Init, median of REPS).
set -o pipefail
REPS=${REPS:-7}
MPIEXEC=${MPIEXEC:-/opt/conda/bin/mpiexec}
mkdir -p build gpurun_out
make -s build/mpilib/libmpi.so 2>/dev/null || make -s build
g++ -O2 tools/mpi_startup_probe.cpp -I/opt/conda/include -Lbuild/mpilib -lmpi -Wl,-rpath-link,/opt/conda/lib \
  -Wl,-rpath,$PWD/build/mpilib -o build/mpi_startup_probe || exit 1
variant() {  # variant <np> <label> <env assignments...>
  local np=$1 label=$2; shift 2
  local v=()
  for r in $(seq 1 $REPS); do
    x=$(env "$@" timeout -k 5 30 $MPIEXEC -np $np build/mpi_startup_probe | sed -n 's/^rank 0\/.*MPI_Init \([0-9.]*\) ms.*/\1/p')
    v+=(${x:-nan})
  done
  echo "np=$np $label: MPI_Init ms $(printf '%s\n' "${v[@]}" | sort -n | awk '{a[NR]=$1} END {printf "median %s best %s", a[int((NR+1)/2)], a[1]}')"
}
for np in 1 2 8; do
  variant $np "default                 " X=1
  variant $np "-x86,-linuxio (lean)    " HWLOC_COMPONENTS=-x86,-linuxio
  variant $np "-linux,-x86,-linuxio    " HWLOC_COMPONENTS=-linux,-x86,-linuxio
  variant $np "no_os,stop              " HWLOC_COMPONENTS=no_os,stop
done
