#!/bin/bash
# block-size sweep of the C2 bench with solve phase timers
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for B in ${BLOCKS:-128 256 512}; do
  timeout -k 10 400 python bench.py --steps ${STEPS:-5} --warmup 2 --block-size $B --no-cpu-baseline --profile-solve ${BENCH_ARGS} > gpurun_out/bench_B$B.log 2>&1 || { echo "BENCH B=$B FAILED"; tail -30 gpurun_out/bench_B$B.log; exit 1; }
  tail -1 gpurun_out/bench_B$B.log
done
