#!/bin/bash
# GPU parity suite (incl. REFERENCE order over column shards), smoke, default bench
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/refshard_gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/refshard_gpu_tests.log; exit 1; }
tail -1 gpurun_out/refshard_gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/refshard_bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/refshard_bench.log; exit 1; }
tail -1 gpurun_out/refshard_bench.log | cut -c1-300
