#!/bin/bash
# round 3: new GPU tests, then the solver's phase breakdown during early (burn-in) sweeps
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu ${TESTS:-tests/test_gpu_exchange.py tests/test_gpu_configs.py tests/test_gpu_rowshard.py} > gpurun_out/r3_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r3_tests.log
[ $rc -eq 0 ] || exit $rc
for w in 4 8 20; do
  timeout -k 10 300 python bench.py --steps 1 --warmup $w --profile-solve --no-cpu-baseline --no-roofline-events $BENCH_ARGS > gpurun_out/r3_prof_w$w.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/r3_prof_w$w.log; exit 1; }
  echo "== warmup $w"
  python3 -c "import json;d=json.loads(open('gpurun_out/r3_prof_w$w.log').read().strip().splitlines()[-1]);dg=d['config']['diag'];[print(k, v) for k, v in dg.items() if k.startswith('solve') or k=='block_events_us']"
done
