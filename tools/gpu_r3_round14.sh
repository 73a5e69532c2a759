#!/bin/bash
# GPU call: page-locking costs on the box (tools/pin_probe.cpp).
set -o pipefail
mkdir -p gpurun_out build
hipcc -O2 -std=c++17 -fopenmp -Icsrc/include --offload-arch=gfx950 tools/pin_probe.cpp -Lmpi_openmp_cuda_amd/lib -lmoc \
  -Wl,-rpath,$PWD/mpi_openmp_cuda_amd/lib -o build/pin_probe || exit 1
OMP_NUM_THREADS=16 timeout -k 5 120 build/pin_probe > gpurun_out/pin_probe_box.log 2>&1; rc=$?
cat gpurun_out/pin_probe_box.log
exit $rc
