#!/bin/bash
# round 5: GPU test suite, then the A/B of scripts/r5_ab.sh (stops at the first failure)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TESTSEL:-} > gpurun_out/${TAG:-r5ab}_gpu_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/${TAG:-r5ab}_gpu_tests.log
  [ $rc = 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${TAG:-r5ab}_gpu_tests.log | head -20; exit $rc; }
fi
bash scripts/r5_ab.sh
