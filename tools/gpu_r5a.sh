set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5/gputest_a.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r5/gputest_a.log
tail -3 gpurun_out/r5/gputest_a.log
timeout -k 10 240 python -u tools/kernel_bench.py input6 input1 > gpurun_out/r5/kb_direct.log 2>&1 && \
MOC_SWIPE_DIRECT=0 timeout -k 10 240 python -u tools/kernel_bench.py input6 input1 > gpurun_out/r5/kb_tiled.log 2>&1
echo "kb rc=$?"
cut -c1-400 gpurun_out/r5/kb_direct.log gpurun_out/r5/kb_tiled.log
