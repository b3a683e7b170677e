#!/bin/bash
# round 5 GPU runner: [GPU suite (any failure ends the run)], [smoke], then bench lines for the
# configs in RUNS (name:flags, flags comma-separated; --env K=V sets a variable for that run only),
# each under its own time limit.  Exit status: non-zero on any test failure or failed bench.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r05a}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_FILES} > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?
  tail -15 gpurun_out/${TAG}_gpu_tests.log
  [ $rc -eq 0 ] || { echo "GPU TESTS FAILED rc=$rc"; exit 1; }
fi
if [ "${SMOKE:-0}" = 1 ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
    || { echo "SMOKE FAILED"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -2 gpurun_out/${TAG}_smoke.log
fi
for cfg in $RUNS; do
  name=${cfg%%:*}; args=$(echo ${cfg#*:} | tr ',' ' ')
  envs=""; bargs=""
  set -- $args
  while [ $# -gt 0 ]; do if [ "$1" = "--env" ]; then envs="$envs $2"; shift 2; else bargs="$bargs $1"; shift; fi; done
  env $envs timeout -k 10 ${RUN_TIMEOUT:-240} python -u bench.py ${CPU_FLAG---no-cpu-baseline} $bargs > gpurun_out/${TAG}_$name.log 2>&1 \
    || { echo "$name FAILED"; tail -20 gpurun_out/${TAG}_$name.log; exit 1; }
  echo "== $name"; tail -1 gpurun_out/${TAG}_$name.log | cut -c1-${CUT:-700}
done
exit 0
