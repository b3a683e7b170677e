#!/bin/bash
# round 3: the list-prefetch parity test alone
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "prefetch" > gpurun_out/pf_test.log 2>&1
rc=$?
tail -12 gpurun_out/pf_test.log
exit $rc
