#!/bin/bash
# round 3: the solver's phase breakdown at several warmup depths (burn-in diagnosis), C2 f32
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for w in ${WARMS:-4 6 8 20}; do
  timeout -k 10 200 python bench.py --steps 1 --warmup $w --profile-solve --no-cpu-baseline --no-roofline-events ${BENCH_ARGS} \
    > gpurun_out/r03diag_w$w.log 2>&1 || { tail -20 gpurun_out/r03diag_w$w.log; exit 1; }
  python3 - $w <<'PY'
import json, sys
w = sys.argv[1]
d = json.loads(open(f"gpurun_out/r03diag_w{w}.log").read().strip().splitlines()[-1])
dg = d["config"]["diag"]
print(w, d["ms_per_step"], {k: v for k, v in dg.items() if k.startswith("solve") and k != "solve_chain_clock_ghz"})
PY
done
