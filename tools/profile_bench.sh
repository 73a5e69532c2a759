# rocprofv3 captures of the headline bench (kernel trace + stats; then SQ counters in their own run) and
# a >1e9-element single-GPU run. Summaries are copied into profiles/ by hand after review.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench \
  -- python3 bench.py --steps 20 > gpurun_out/prof_bench.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
  SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_bench -o bench \
  -- python3 bench.py --steps 5 > gpurun_out/pmc_bench.log 2>&1
timeout -k 10 600 python3 bench.py --records-per-gpu 134217728 --steps 10 --warmup 2 > gpurun_out/bench_1g.log 2>&1
