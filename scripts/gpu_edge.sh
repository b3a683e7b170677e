#!/bin/bash
# edge-shape parity tests alone (tiny / ragged / degenerate shapes)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k edge_shapes -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/edge_gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/edge_gpu_tests.log; exit 1; }
tail -12 gpurun_out/edge_gpu_tests.log
