set -e
mkdir -p gpurun_out
for t in 1024 512 256; do
  MOC_SWIPE_TILE=$t timeout -k 10 120 python tools/kernel_bench.py input6 > gpurun_out/abs_k$t.log 2>&1
  MOC_SWIPE_TILE=$t timeout -k 10 200 python bench.py --steps 30 > gpurun_out/abs_b$t.log 2>&1
done
