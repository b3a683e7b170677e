#!/bin/bash
# round 4 GPU runner: [GPU suite], then bench lines for the configs in RUNS (name:flags, flags comma-
# separated; --env K=V sets an environment variable for that run only), each under its own time limit
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04a}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 8 --timeout 150 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?
  tail -15 gpurun_out/${TAG}_gpu_tests.log
  [ $rc -eq 0 ] || { echo "GPU TESTS FAILED rc=$rc"; exit 1; }
fi
for cfg in $RUNS; do
  name=${cfg%%:*}; args=$(echo ${cfg#*:} | tr ',' ' ')
  envs=""; bargs=""
  set -- $args
  while [ $# -gt 0 ]; do if [ "$1" = "--env" ]; then envs="$envs $2"; shift 2; else bargs="$bargs $1"; shift; fi; done
  env $envs timeout -k 10 ${RUN_TIMEOUT:-240} python -u bench.py --no-cpu-baseline $bargs > gpurun_out/${TAG}_$name.log 2>&1 \
    || { echo "$name failed"; tail -20 gpurun_out/${TAG}_$name.log; exit 1; }
  echo "== $name"; tail -1 gpurun_out/${TAG}_$name.log | cut -c1-${CUT:-600}
done
exit 0
