#!/bin/bash
# Multi-rank rehearsal on the one MI355X of a gpurun box (the paths the driver's N = 8 run takes):
#   1. mpiexec -np 8 ./final --backend=hip --gpu-isolate=1 on the goldens: the N = 8 bench's
#      final_input6_wall_hip field, 8 GPU ranks isolated onto the one device;
#   2. ./final --transport=rccl --timing at np 1 (the communicator, the new comm fields);
#   3. bench.py --gpus 4 --dist-backend gloo --allow-shared-gpu --final-wall 1: the bench's own N > 1 wall
#      fields (4 bench ranks + 4 ./final ranks on the GPU).
set -o pipefail
OUT=${OUT:-gpurun_out/rehearse}
mkdir -p $OUT
for i in 6 3 4 1; do
  timeout -k 10 120 /opt/conda/bin/mpiexec -np 8 ./final --backend=hip --gpu-isolate=1 --timing \
    < tests/data/input$i.txt > $OUT/np8_in$i.out 2> $OUT/np8_in$i.err || { tail -5 $OUT/np8_in$i.err; exit 1; }
  if cmp -s $OUT/np8_in$i.out tests/data/expected/input$i.out; then echo "np8 hip input$i: golden ok"; else echo "np8 input$i DIFFERS"; exit 1; fi
done
timeout -k 10 120 /opt/conda/bin/mpiexec -np 1 ./final --backend=hip --transport=rccl --timing \
  < tests/data/input3.txt > $OUT/rccl_np1.out 2> $OUT/rccl_np1.err || { tail -5 $OUT/rccl_np1.err; exit 1; }
cmp -s $OUT/rccl_np1.out tests/data/expected/input3.out && echo "rccl np1 input3: golden ok" || { echo "rccl np1 DIFFERS"; exit 1; }
grep '^{' $OUT/rccl_np1.err | tail -1 | cut -c1-600
timeout -k 10 900 python3 bench.py --gpus 4 --allow-shared-gpu --dist-backend gloo --steps 20 --warmup 3 --final-wall 1 \
  > $OUT/rehearse_bench_4.json 2> $OUT/rehearse_bench_4.err || { tail -20 $OUT/rehearse_bench_4.err; exit 1; }
cut -c1-300 $OUT/rehearse_bench_4.json
python3 -c "import json; d=json.loads(open('$OUT/rehearse_bench_4.json').read().splitlines()[-1]); print('wall', d['final_input6_wall'], d['final_input6_wall_hip'], 'verified', d['verified'])"
