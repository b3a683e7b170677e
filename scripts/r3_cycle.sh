#!/bin/bash
# round 3 build -> measure cycle: GPU tests (TESTS, default the whole -m gpu suite), then the
# per-sweep burn-in trace of library variants (scripts/r3_variants.sh, VARIANTS)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
if [ "${TESTS:-all}" != "none" ]; then
  T=${TESTS:-tests}; [ "$T" = all ] && T=tests
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu $T > gpurun_out/r3_tests.log 2>&1; rc=$?
  tail -4 gpurun_out/r3_tests.log
  [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r3_tests.log | head -20; exit $rc; }
fi
[ -n "$VARIANTS" ] && bash scripts/r3_variants.sh
exit 0
