#!/bin/bash
# one GPU round: parity tests -> C2 bench -> rocprofv3 kernel trace of a short C2 run
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -q -m gpu -p no:cacheprovider -x > gpurun_out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ -n "$PROFILE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline-events ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 || { echo "PROF FAILED"; tail -30 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -20
fi
