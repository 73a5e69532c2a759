set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_steps.sh \
 "r4_stdin_test:300:python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu.py -k 'stdin_batches or streaming_slices'" \
 "final_walltime_hip_r4b_spaced:400:NPS='1 2' INPUTS='6 3' REPS=5 SPACING=2 HELLO=0 TIMING=1 EXTRA='--backend=hip --device=0 --log-level=debug' bash tools/final_walltime.sh"
