# round 5: swipe b64-chunk layout — GPU tier (swipe + extremes + wire) then device-resident kernel bench
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "swipe or extreme or wire or golden or random or zero_copy or packed or group_coded or kernel_selection or small_brute" > gpurun_out/r5/gputest_c.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5/gputest_c.log; tail -3 gpurun_out/r5/gputest_c.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/kernel_bench.py input6 input1 mid > gpurun_out/r5/kb_c.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/kernel_bench.py --variants wire input6 input1 > gpurun_out/r5/kb_wire_c.log 2>&1 || exit 1
cut -c1-260 gpurun_out/r5/kb_c.log gpurun_out/r5/kb_wire_c.log
