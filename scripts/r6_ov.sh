#!/bin/bash
# round 6: the overlapped solver (BRR_OVS=1) -- GPU parity subset with it on, then a same-box A/B
# (scripts/r5_ab.sh) against the round-5 solver (BRR_OVS=0).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r06b}
if [ "${TESTS:-1}" = 1 ]; then
  BRR_OVS=1 timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest ${TESTFILES:-tests/test_gpu_parity.py tests/test_golden.py} -m gpu -x -q \
    --timeout 120 --timeout-method thread ${TESTSEL:-} > gpurun_out/${TAG}_ov_tests.log 2>&1
  rc=$?; tail -5 gpurun_out/${TAG}_ov_tests.log
  [ $rc = 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/${TAG}_ov_tests.log | head -30; exit $rc; }
fi
TAG=$TAG bash scripts/r5_ab.sh
