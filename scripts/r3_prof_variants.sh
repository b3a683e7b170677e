#!/bin/bash
# round 3: solver phase breakdown (bench.py --profile-solve) of library variants at one warmup depth
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in ${VARIANTS:-default::}; do
  name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; envs=${rest#*:}
  if [ -n "$lib" ]; then export BRR_LIB=$lib; else unset BRR_LIB; fi
  env ${envs//,/ } timeout -k 10 300 python bench.py --steps 1 --warmup ${W:-4} --profile-solve --no-cpu-baseline --no-roofline-events $BENCH_ARGS > gpurun_out/r3_pv_$name.log 2>&1 || { echo "$name FAILED"; tail -20 gpurun_out/r3_pv_$name.log; exit 1; }
  echo "== $name"
  python3 -c "import json;d=json.loads(open('gpurun_out/r3_pv_$name.log').read().strip().splitlines()[-1]);dg=d['config']['diag'];[print(k, v) for k, v in dg.items() if k.startswith('solve')];b=dg.get('block_events_us',{});print({k: b[k] for k in ('period','solver_wait','solver_chain','solver_publish') if k in b})"
done
