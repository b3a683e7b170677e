#!/bin/bash
# round 6: the whole GPU suite under an environment (SUITE_ENV, comma-separated K=V), then the A/B of
# scripts/r5_ab.sh.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r06d}
if [ "${TESTS:-1}" = 1 ]; then
  env $(echo "${SUITE_ENV:-}" | tr ',' ' ') timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -x -q \
    --timeout 150 --timeout-method thread ${TESTSEL:-} > gpurun_out/${TAG}_suite.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_suite.log
  [ $rc = 0 ] || { grep -E "^FAILED|Error" gpurun_out/${TAG}_suite.log | head -20; exit $rc; }
fi
TAG=$TAG bash scripts/r5_ab.sh
