#!/bin/bash
# round 3: per-sweep burn-in trace of library variants (VARIANTS="name:lib:env[:bench args] ...", comma-separated
# lists), C2 f32 by default
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in ${VARIANTS:-default::}; do
  name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; rest=${rest#*:}; envs=${rest%%:*}; bargs=""
  [ "$rest" != "$envs" ] && bargs=${rest#*:}
  if [ -n "$lib" ]; then export BRR_LIB=$lib; else unset BRR_LIB; fi
  env ${envs//,/ } timeout -k 10 300 python bench.py --steps 5 --warmup 25 --trace-sweeps 1 --no-cpu-baseline --no-roofline-events ${BENCH_ARGS} ${bargs//,/ } > gpurun_out/r3_var_$name.log 2>&1 || { echo "$name FAILED"; tail -20 gpurun_out/r3_var_$name.log; exit 1; }
  python3 - "$name" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r3_var_{sys.argv[1]}.log").read().strip().splitlines()[-1])
w = d['config']['diag']['sweep_trace_ms_changed']['warmup']
ms = [x[0] for x in w]
print(sys.argv[1], 'steady', d['value'], 'sweeps5-24 ms/step', round(sum(ms[5:25]) / 20, 2), 'first10', ms[:10])
PY
done
