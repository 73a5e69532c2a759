#!/bin/bash
# --backend=auto's GPU threshold (--gpu-min-cells): whole-job wall clock of ./final on the CPU engine vs the
# GPU for input6- and input3-shaped jobs of growing size, one rank, output to a file. The crossover is the
# job size where the GPU's start-up (HIP runtime + engine, 0.1-0.3 s) is paid back by its search speed.
set -e
mkdir -p gpurun_out
for shape in input6 input3; do
  for rec in ${RECORDS:-250000 1000000 4000000 16000000}; do
    n=$rec
    [ "$shape" = input3 ] && n=$((rec / 4000))
    [ "$n" -lt 1 ] && n=1
    F=/tmp/moc_cross_$shape.txt
    timeout -k 10 120 python3 tools/gen_synthetic.py --shape $shape --records $n --out $F > /dev/null
    for be in cpu hip; do
      s=$(date +%s%N)
      timeout -k 10 120 ./final --backend=$be --timing --input=$F --output=/tmp/moc_cross.out \
        --gpu-prewarm-bytes=1 2> gpurun_out/cross_timing.txt
      e=$(date +%s%N)
      cells=$(tail -1 gpurun_out/cross_timing.txt | python3 -c 'import sys,json; print(json.loads(sys.stdin.read())["cells"])')
      echo "shape=$shape records=$n backend=$be cells=$cells wall_ms=$(( (e - s) / 1000000 ))"
    done
    rm -f $F /tmp/moc_cross.out
  done
done
