#!/bin/bash
# round 4: GPU suite, then one C5 rank's real workload (N = 500,000 x P_local = 125,000, shard 0 of 8,
# f32) on one GPU at E = 1 / 4 / 8 / 16 exchanges per sweep (bench.py --rank-of 8: every exchange
# segment, the other ranks' deltas zero, no collective), then the default C2 bench line
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04a}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 480 python -u -m pytest tests -m gpu -q --maxfail 8 --timeout 150 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${TAG}_gpu_tests.log 2>&1
  rc=$?
  tail -15 gpurun_out/${TAG}_gpu_tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for E in ${ES:-1 4 8 16}; do
  timeout -k 10 300 python -u bench.py --config c5 --rank-of 8 --exchanges $E --steps ${STEPS:-20} --warmup 10 \
    --no-cpu-baseline ${C5ARGS} > gpurun_out/${TAG}_c5rank_E$E.log 2>&1 || { echo "c5 E=$E failed"; tail -20 gpurun_out/${TAG}_c5rank_E$E.log; exit 1; }
  echo "== E=$E"; tail -1 gpurun_out/${TAG}_c5rank_E$E.log | cut -c1-420
done
if [ "${C2:-1}" = 1 ]; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_c2.log 2>&1 || { echo "c2 failed"; tail -20 gpurun_out/${TAG}_c2.log; exit 1; }
  echo "== C2"; tail -1 gpurun_out/${TAG}_c2.log | cut -c1-420
fi
for cfg in ${EXTRA:-c2_2bit:--config,c2,--x-storage,2bit c2_2bit_nt512:--config,c2,--x-storage,2bit,--env,BRR_STREAM_NT=512 c4_cc_prof:--config,c4,--profile-solve,--env,BRR_F32_CODE_CACHE=1 c4_prof:--config,c4,--profile-solve}; do
  name=${cfg%%:*}; args=$(echo ${cfg#*:} | tr ',' ' ')
  envs=""; bargs=""
  set -- $args
  while [ $# -gt 0 ]; do if [ "$1" = "--env" ]; then envs="$envs $2"; shift 2; else bargs="$bargs $1"; shift; fi; done
  env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 10 --no-cpu-baseline $bargs > gpurun_out/${TAG}_$name.log 2>&1 || { echo "$name failed"; tail -20 gpurun_out/${TAG}_$name.log; exit 1; }
  echo "== $name"; tail -1 gpurun_out/${TAG}_$name.log | cut -c1-420
done
if [ "${ONESHOT:-1}" = 1 ]; then
  timeout -k 10 300 python -u bench.py --oneshot --no-cpu-baseline > gpurun_out/${TAG}_c1_oneshot.log 2>&1 || { echo "oneshot failed"; tail -20 gpurun_out/${TAG}_c1_oneshot.log; exit 1; }
  echo "== C1 one-shot"; tail -1 gpurun_out/${TAG}_c1_oneshot.log | cut -c1-3000
fi
exit 0
