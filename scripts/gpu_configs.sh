#!/bin/bash
# bench every single-GPU config (c2 c3 c4) with the default options; one line each
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for c in ${CONFIGS:-c2 c3 c4}; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_$c.log 2>&1 || { echo "BENCH $c FAILED"; tail -30 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log | cut -c1-400
done
