#!/bin/bash
# GPU start-up of one rank on the box (what `final`'s setup / gpu_wait pays when a job runs on the GPU):
# tools/init_probe.cpp phase by phase, REPS runs per environment variant.
set -o pipefail
REPS=${REPS:-3}
mkdir -p build gpurun_out
/opt/rocm/bin/hipcc -O2 -std=c++17 -Icsrc/include tools/init_probe.cpp -Lmpi_openmp_cuda_amd/lib -lmoc \
  -Wl,-rpath,$PWD/mpi_openmp_cuda_amd/lib -o build/init_probe || exit 1
g++ -O2 -std=c++17 tools/plugin_load_probe.cpp -ldl -o build/plugin_load_probe || exit 1
for r in 1 2 3; do
  echo "== plugin load (run $r)"; timeout -k 5 60 build/plugin_load_probe 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== HIP runtime first, then the plugin (run $r)"; timeout -k 5 60 build/plugin_load_probe mpi_openmp_cuda_amd/lib/libmoc_final_gpu.so hip 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "# $(ls /sys/class/kfd/kfd/topology/nodes | wc -l) KFD topology nodes; $(ls /dev/dri | tr '\n' ' ')"
variant() {
  local label=$1; shift
  for r in $(seq 1 $REPS); do
    echo "== $label (run $r)"
    env "$@" timeout -k 5 60 build/init_probe 2>&1 | grep -v amdgpu.ids || return 1
  done
}
variant "default" X=1
variant "ROCR_VISIBLE_DEVICES=0" ROCR_VISIBLE_DEVICES=0
variant "HIP_ENABLE_DEFERRED_LOADING=0" HIP_ENABLE_DEFERRED_LOADING=0
variant "HSA_ENABLE_SDMA=0" HSA_ENABLE_SDMA=0
