#!/bin/bash
# column shards in two processes on the GPU (gloo exchange)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_multiprocess.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/mp_gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/mp_gpu_tests.log; exit 1; }
tail -6 gpurun_out/mp_gpu_tests.log
