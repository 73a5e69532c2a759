#!/bin/bash
# Tiny-job start-up on the box: the launcher alone (mpiexec of /bin/true), the in-process MPI phases
# (tools/mpi_startup_probe.cpp) under mpiexec and as a singleton, and ./final on input6 the same ways.
set -o pipefail
MPIEXEC=${MPIEXEC:-/opt/conda/bin/mpiexec}
mkdir -p build gpurun_out
make -s build/mpilib/libmpi.so 2>/dev/null || make -s build
g++ -O2 tools/mpi_startup_probe.cpp -I/opt/conda/include -Lbuild/mpilib -lmpi -Wl,-rpath-link,/opt/conda/lib \
  -Wl,-rpath,$PWD/build/mpilib -o build/mpi_startup_probe || exit 1
ms() { local s=$(date +%s%N); "$@" > /tmp/msp_out.txt 2>&1; local rc=$?; local e=$(date +%s%N); echo "$(( (e - s) / 1000000 )) ms rc=$rc"; }
echo "# host: $(nproc) cpus visible, hostname $(hostname)"
s=$(date +%s%N); getent hosts $(hostname); echo "getent hosts \$(hostname): rc=$? $(( ($(date +%s%N) - s) / 1000000 )) ms"
s=$(date +%s%N); getent ahosts $(hostname) > /dev/null; echo "getent ahosts: rc=$? $(( ($(date +%s%N) - s) / 1000000 )) ms"
cat /etc/resolv.conf 2>/dev/null | grep -v '^#' | head -5
for r in 1 2 3; do
  echo "mpiexec -np 1 /bin/true:        $(ms timeout -k 5 30 $MPIEXEC -np 1 /bin/true)"
  echo "mpiexec -np 2 /bin/true:        $(ms timeout -k 5 30 $MPIEXEC -np 2 /bin/true)"
  echo "probe singleton:                $(ms timeout -k 5 30 build/mpi_startup_probe)"; cat /tmp/msp_out.txt
  echo "mpiexec -np 1 probe:            $(ms timeout -k 5 30 $MPIEXEC -np 1 build/mpi_startup_probe)"; cat /tmp/msp_out.txt
  echo "mpiexec -np 1 probe multiple:   $(ms timeout -k 5 30 $MPIEXEC -np 1 build/mpi_startup_probe multiple)"; cat /tmp/msp_out.txt
  echo "mpiexec -np 2 probe:            $(ms timeout -k 5 30 $MPIEXEC -np 2 build/mpi_startup_probe)"; cat /tmp/msp_out.txt
  echo "mpiexec -np 1 probe iface=lo:   $(ms env MPIR_CVAR_CH3_INTERFACE_HOSTNAME=127.0.0.1 timeout -k 5 30 $MPIEXEC -np 1 build/mpi_startup_probe)"; cat /tmp/msp_out.txt
  echo "mpiexec -np 2 probe iface=lo:   $(ms env MPIR_CVAR_CH3_INTERFACE_HOSTNAME=127.0.0.1 timeout -k 5 30 $MPIEXEC -np 2 build/mpi_startup_probe)"; cat /tmp/msp_out.txt
  echo "mpiexec -np 1 probe nolocal=0 hostname=localhost: $(ms timeout -k 5 30 $MPIEXEC -hosts localhost -np 1 build/mpi_startup_probe)"; cat /tmp/msp_out.txt
  echo "./final singleton input6:       $(ms timeout -k 5 30 sh -c './final --timing < tests/data/input6.txt')"
  echo "mpiexec -np 1 ./final input6:   $(ms timeout -k 5 30 sh -c "$MPIEXEC -np 1 ./final < tests/data/input6.txt")"
done
