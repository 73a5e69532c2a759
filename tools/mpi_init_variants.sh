#!/bin/bash
# What MPI_Init spends ~200 ms on at one rank on the MI355X box (mpiexec itself: 5-9 ms): the MPICH
# (3.3.2, ch3:nemesis) start-up under environment variants — its embedded hwloc's discovery components,
# the tcp netmod's host lookup — MPI_Init median/best of REPS runs of tools/mpi_startup_probe.cpp.
set -o pipefail
REPS=${REPS:-7}
MPIEXEC=${MPIEXEC:-/opt/conda/bin/mpiexec}
mkdir -p build gpurun_out
make -s build/mpilib/libmpi.so 2>/dev/null || make -s build
g++ -O2 tools/mpi_startup_probe.cpp -I/opt/conda/include -Lbuild/mpilib -lmpi -Wl,-rpath-link,/opt/conda/lib \
  -Wl,-rpath,$PWD/build/mpilib -o build/mpi_startup_probe || exit 1
echo "# host: $(nproc) cpus visible; $(grep -c ^processor /proc/cpuinfo) in /proc/cpuinfo; $(ls -d /sys/devices/system/cpu/cpu[0-9]* | wc -l) in sysfs; $(ls /sys/bus/pci/devices | wc -l) PCI devices"
variant() {  # variant <label> <env assignments...>
  local label=$1; shift
  local v=()
  for r in $(seq 1 $REPS); do
    x=$(env "$@" timeout -k 5 30 $MPIEXEC -np 1 build/mpi_startup_probe | sed -n 's/.*MPI_Init \([0-9.]*\) ms.*/\1/p')
    v+=(${x:-nan})
  done
  echo "$label: MPI_Init ms $(printf '%s\n' "${v[@]}" | sort -n | awk '{a[NR]=$1} END {printf "median %s best %s", a[int((NR+1)/2)], a[1]}')"
}
variant "baseline                         " X=1
variant "HWLOC_COMPONENTS=-x86            " HWLOC_COMPONENTS=-x86
variant "HWLOC_COMPONENTS=-linuxio        " HWLOC_COMPONENTS=-linuxio
variant "HWLOC_COMPONENTS=-pci            " HWLOC_COMPONENTS=-pci
variant "HWLOC_COMPONENTS=-x86,-linuxio,-pci" HWLOC_COMPONENTS=-x86,-linuxio,-pci
variant "HWLOC_COMPONENTS=no_os           " HWLOC_COMPONENTS=no_os
variant "HWLOC_COMPONENTS=synthetic       " HWLOC_COMPONENTS=synthetic
variant "HWLOC_LINUX_USE_CPUINFO=1        " HWLOC_LINUX_USE_CPUINFO=1
variant "HWLOC_THISSYSTEM_ALLOWED_RESOURCES=0" HWLOC_THISSYSTEM_ALLOWED_RESOURCES=0
variant "INTERFACE_HOSTNAME=127.0.0.1     " MPIR_CVAR_INTERFACE_HOSTNAME=127.0.0.1
variant "NEMESIS_NETMOD=tcp               " MPIR_CVAR_NEMESIS_NETMOD=tcp
variant "HWLOC_COMPONENTS_VERBOSE=1 (once)" X=1
HWLOC_COMPONENTS_VERBOSE=1 timeout -k 5 30 $MPIEXEC -np 1 build/mpi_startup_probe 2>&1 | head -30
