#!/bin/bash
# GPU call: full GPU test tier; RCCL start-up variants; ./final streaming batch sizes and the rccl transport's
# distribute phase at 1.14 G letters (1 rank); bench at N=1 and the 2-rank gloo rehearsal (per-rank fields).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_r3_full.log 2>&1 || { tail -40 gpurun_out/gpu_tests_r3_full.log; exit 1; }
tail -2 gpurun_out/gpu_tests_r3_full.log
/opt/rocm/bin/hipcc -O2 -std=c++17 -fopenmp tools/rccl_init_probe.cpp -ldl -o build/rccl_init_probe || exit 1
timeout -k 10 600 bash tools/rccl_init_variants.sh > gpurun_out/rccl_init_variants.log 2>&1 || { tail -20 gpurun_out/rccl_init_variants.log; exit 1; }
grep -E "==|TOTAL|process wall|warm-up|InitRank|Destroy|Abort|exit" gpurun_out/rccl_init_variants.log
F=/tmp/moc_big6.txt
timeout -k 10 300 python3 tools/gen_synthetic.py --shape input6 --records 134217728 --jobs 16 --out $F || exit 1
for mode in "--batch-records=16777216" "--batch-records=67108864" "--transport=rccl" "--transport=rccl --batch-records=33554432"; do
  rm -f /tmp/moc_big6.out
  s=$(date +%s%N)
  timeout -k 10 300 /opt/conda/bin/mpiexec -np 1 ./final --timing --device=0 --input=$F --output=/tmp/moc_big6.out $mode \
    2> gpurun_out/r3_mode_timing.txt || { tail -5 gpurun_out/r3_mode_timing.txt; exit 1; }
  e=$(date +%s%N)
  echo "mode='$mode' wall_ms=$(( (e - s) / 1000000 )) out_bytes=$(stat -c %s /tmp/moc_big6.out) $(tail -1 gpurun_out/r3_mode_timing.txt)"
done > gpurun_out/final_modes_r3.log
cut -c1-700 gpurun_out/final_modes_r3.log
rm -f $F /tmp/moc_big6.out
timeout -k 10 300 python bench.py > gpurun_out/bench_r3_n1.log 2> gpurun_out/bench_r3_n1.err || { tail -5 gpurun_out/bench_r3_n1.err; exit 1; }
cat gpurun_out/bench_r3_n1.log
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --allow-shared-gpu --records-per-gpu 8388608 --steps 10 --warmup 2 > gpurun_out/bench_r3_gloo2.log 2> gpurun_out/bench_r3_gloo2.err || { tail -5 gpurun_out/bench_r3_gloo2.err; exit 1; }
cat gpurun_out/bench_r3_gloo2.log
