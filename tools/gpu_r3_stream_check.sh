set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -v --timeout 120 --timeout-method thread -k "streaming or narrow_guess or final_cli or sliced" > gpurun_out/gpu_tests_stream.log 2>&1 || { tail -40 gpurun_out/gpu_tests_stream.log; exit 1; }
tail -3 gpurun_out/gpu_tests_stream.log
MODES="--output=/tmp/moc_big6.out|--output=/tmp/moc_big6.out --batch-records=16777216" NPS="1 2" timeout -k 10 600 bash tools/final_scale.sh > gpurun_out/final_scale_r3_stream.log 2>&1 || { tail -20 gpurun_out/final_scale_r3_stream.log; exit 1; }
cat gpurun_out/final_scale_r3_stream.log | cut -c1-1500
