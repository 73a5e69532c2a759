# A/B of tile-kernel variants on the device-resident microbench (tools/kernel_bench.py):
# sub-tiles per wave tile (MOC_TILE_U) and tile-kernel waves per CU (MOC_TILE_WAVES_PER_CU).
set -e
mkdir -p gpurun_out
for cfg in "0 16" "0 8" "0 32" "4 32" "2 32"; do
  set -- $cfg
  MOC_TILE_U=$1 MOC_TILE_WAVES_PER_CU=$2 timeout -k 10 200 python tools/kernel_bench.py input4 input3 limits \
    > gpurun_out/ab_u$1_w$2.log 2>&1
done
