# round 5: GPU tier + device-resident kernel bench (lane-direct swipe vs block-tiled) + headline bench
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/gputest_b.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5/gputest_b.log; tail -3 gpurun_out/r5/gputest_b.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/kernel_bench.py input6 input1 > gpurun_out/r5/kb_direct_b.log 2>&1 || exit 1
MOC_SWIPE_DIRECT=0 timeout -k 10 240 python -u tools/kernel_bench.py input6 input1 > gpurun_out/r5/kb_tiled_b.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r5/bench_b.log 2> gpurun_out/r5/bench_b.err || exit 1
cut -c1-330 gpurun_out/r5/kb_direct_b.log gpurun_out/r5/kb_tiled_b.log; cut -c1-400 gpurun_out/r5/bench_b.log
