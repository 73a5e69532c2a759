#!/bin/bash
# The GPU-box measurements behind profiles/, by name, in one gpurun call:
#   /usr/local/graft/bin/gpurun --timeout 1200 -- 'bash tools/gpu_checks.sh tier smoke bench wall-hip'
# Each check runs under its own time limit through tools/gpu_steps.sh (which stops at the first fault,
# abort or timeout) and writes gpurun_out/<check>.log (TAG=... adds a suffix: gpurun_out/<check>_<TAG>.log).
#
#   tier          the GPU test tier (pytest -m gpu)
#   smoke         __graft_entry__.smoke()
#   bench         python bench.py --steps 50 --warmup 5 (headline line with both wall-clock fields)
#   bench-trace   rocprofv3 kernel trace + stats of 20 headline steps -> gpurun_out/bench_trace/
#   wall          mpiexec -np 1/2/4 ./final < input1..6 (default engine) beside mpi_hello / hip_hello
#   wall-hip      the same forced onto the GPU (--backend=hip), launches 1 s apart, with --timing (np 1/2)
#   hip-trace     HIP API + kernel trace of one --backend=hip launch on input6 and input3
#                 -> gpurun_out/hip_wall_trace/ (summarise with tools/api_timeline.py)
#   copy-probe    the first host->device copy's cost by size, with and without SDMA (tools/copy_path_probe.hip)
#   kernels       device-resident kernel throughput (tools/kernel_bench.py)
#   swipe-ab      kernel_bench on input6 / input1 for the in-tree library and every build/variant_*/libmoc.so
#                 (make variant NAME=... VDEFS=...: A/B builds, e.g. -DMOC_T16_UNROLL=32)
#   isolate       --gpu-isolate=1 at np 1/2 (the rank's runtime shows its GPU only)
#   hello-env     tools/hip_hello.hip's runtime / first-queue times under runtime environment settings
#   dcheck        tools/dcheck.sh: the kernel tests on the device-bounds-checked library (make debug-kernels,
#                 then copy build/debug/libmoc.so to build/dbgk/), one COUNT line per distinct MOC_DCHECK report
# Longer studies have scripts of their own: step_variance.sh, pmc_ab.sh, rehearse_ranks.sh,
# final_1e10_threads.sh, rccl_init_rootcause.sh.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
sfx=${TAG:+_$TAG}
steps=()
for c in "$@"; do
  case $c in
    tier) steps+=("tier$sfx:900:python -u -m pytest -q --timeout 200 --timeout-method thread tests/ -m gpu") ;;
    smoke) steps+=("smoke$sfx:300:python -c 'import __graft_entry__ as g; g.smoke()'") ;;
    bench) steps+=("bench$sfx:300:python bench.py --steps 50 --warmup 5") ;;
    bench-trace) steps+=("bench_trace$sfx:300:timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/bench_trace -o b -- python3 bench.py --steps 20 --warmup 5 --final-wall 0") ;;
    wall) steps+=("wall$sfx:400:NPS='1 2 4' REPS=7 HELLO=1 bash tools/final_walltime.sh") ;;
    wall-hip) steps+=("wall_hip$sfx:400:NPS='1 2' INPUTS='6 1 3 4' REPS=7 SPACING=1 HELLO=1 TIMING=1 EXTRA='--backend=hip --log-level=debug' bash tools/final_walltime.sh") ;;
    hip-trace)
      mkdir -p gpurun_out/hip_wall_trace
      for i in 6 3; do
        steps+=("hip_trace_input$i$sfx:120:cd /tmp && timeout -k 10 100 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $R/gpurun_out/hip_wall_trace -o input$i -- $R/final --backend=hip --timing --quick-exit=0 < $R/tests/data/input$i.txt")
      done ;;
    copy-probe)
      steps+=("copy_probe$sfx:200:hipcc --offload-arch=gfx950 -O2 tools/copy_path_probe.hip -o build/copy_path_probe && for b in 4096 65536 131072 1048576 16777216; do timeout -k 10 30 build/copy_path_probe \$b && HSA_ENABLE_SDMA=0 timeout -k 10 30 build/copy_path_probe \$b || exit 1; done") ;;
    kernels) steps+=("kernels$sfx:400:python tools/kernel_bench.py") ;;
    swipe-ab)
      for lib in mpi_openmp_cuda_amd/lib/libmoc.so build/variant_*/libmoc.so; do
        [ -f "$lib" ] || continue
        n=$(basename "$(dirname "$lib")")
        steps+=("swipe_ab_$n$sfx:200:echo '# $lib' && MOC_LIB_PATH=$R/$lib python tools/kernel_bench.py input6 input1")
      done ;;
    hello-env)  # the runtime start and the first hardware queue (tools/hip_hello.hip) under runtime settings
      steps+=("hello_env$sfx:300:(cd build && [ -x hip_hello ] && [ hip_hello -nt ../tools/hip_hello.hip ] || { make -s -C .. build/mpilib/libmpi.so && hipcc --offload-arch=gfx950 -O2 ../tools/hip_hello.hip -I/opt/conda/include -Lmpilib -lmpi -Wl,-rpath-link,/opt/conda/lib -Wl,-rpath,\$PWD/mpilib -o hip_hello; }) && for e in NONE HELLO_NULL_STREAM=1 HSA_ENABLE_INTERRUPT=0 AMD_DIRECT_DISPATCH=0 ROC_AQL_QUEUE_SIZE=1024 HSA_ENABLE_SDMA=0 GPU_MAX_HW_QUEUES=1 HIP_FORCE_DEV_KERNARG=1; do for r in 1 2 3 4 5; do sleep 1; echo \"\$e \$(env \${e/NONE/X=1} timeout -k 10 30 build/hip_hello 2>&1 >/dev/null | tail -1)\" || exit 1; done; done") ;;
    isolate) steps+=("isolate$sfx:200:NPS='1 2' INPUTS='6' REPS=7 SPACING=1 HELLO=0 TIMING=1 EXTRA='--backend=hip --gpu-isolate=1 --log-level=info' bash tools/final_walltime.sh") ;;
    dcheck) steps+=("dcheck$sfx:900:bash tools/dcheck.sh") ;;
    *) echo "unknown check: $c (see the header of $0)"; exit 2 ;;
  esac
done
[ ${#steps[@]} -gt 0 ] || { echo "usage: $0 check ..."; exit 2; }
bash tools/gpu_steps.sh "${steps[@]}"
