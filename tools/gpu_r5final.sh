# round 5, end of session: the full GPU tier, smoke, the headline bench and its kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r5final
timeout -k 10 1500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/r5final/gpu_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r5final/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5final/smoke.log 2>&1 || { tail -5 gpurun_out/r5final/smoke.log; exit 1; }
tail -1 gpurun_out/r5final/smoke.log
timeout -k 10 600 python -u bench.py --steps 50 --warmup 5 > gpurun_out/r5final/bench.log 2>&1 || { tail -5 gpurun_out/r5final/bench.log; exit 1; }
tail -1 gpurun_out/r5final/bench.log | cut -c1-400
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5final/prof -o bench -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/r5final/bench_prof.log 2>&1 || { tail -5 gpurun_out/r5final/bench_prof.log; exit 1; }
find gpurun_out/r5final/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r5final/bench_kernel_stats.csv
head -5 gpurun_out/r5final/bench_kernel_stats.csv | cut -c1-200
