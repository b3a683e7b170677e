#!/bin/bash
# is the solver chain slow intrinsically or under load?  microbenchmark + C4/C3 at small N
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./scripts/mb_chain.bin > gpurun_out/mb_chain.log 2>&1 || { echo "MB FAILED"; cat gpurun_out/mb_chain.log; exit 1; }
cat gpurun_out/mb_chain.log
for n in 4096 100000; do
for c in c4 c3; do
  timeout -k 10 300 python bench.py --config $c --N $n --P 100000 --steps 5 --warmup 10 --no-cpu-baseline --profile-solve > gpurun_out/chain_${c}_$n.log 2>&1 || { echo "DIAG $c FAILED"; tail -30 gpurun_out/chain_${c}_$n.log; exit 1; }
  python3 - gpurun_out/chain_${c}_$n.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); g=d['config']['diag']
print(sys.argv[1], d['value'], d['roofline']['per_block_us'], g['solve_phase_us'], g['solve_chain_steps'], g.get('solve_wait_us'), {k:g['block_events_us'][k] for k in ('period','solver_wait','solver_chain')})
PY
done
done
