#!/bin/bash
# one GPU round: parity tests -> smoke -> C2 bench (defaults) -> rocprofv3 kernel trace + PMC
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ -n "$PROFILE" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 10 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof.log 2>&1 || { echo "PROF FAILED"; tail -30 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -12
  tail -1 gpurun_out/prof.log | cut -c1-300
fi
if [ -n "$PMC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $c --kernel-include-regex 'k_sweep|k_stream' -d gpurun_out/pmc_$c -o pmc --output-format csv \
      -- python3 bench.py --steps 2 --warmup 10 --no-cpu-baseline --no-roofline-events ${BENCH_ARGS} > gpurun_out/pmc_$c.log 2>&1 \
      || { echo "PMC $c FAILED"; tail -20 gpurun_out/pmc_$c.log; exit 1; }
  done
  python3 scripts/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE
fi
