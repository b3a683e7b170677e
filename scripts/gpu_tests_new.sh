#!/bin/bash
# run a selection of GPU tests (-k expression in $SEL), one pytest process
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$SEL" > gpurun_out/tests_sel.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tests_sel.log | tail -40
exit $rc
