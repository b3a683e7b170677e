#!/bin/bash
# blocked Horseshoe chain: microbenchmark, then parity tests of the Horseshoe paths, then C4 diag
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./scripts/mb_chain2.bin > gpurun_out/mb_chain2.log 2>&1 || { echo "MB FAILED"; cat gpurun_out/mb_chain2.log; exit 1; }
cat gpurun_out/mb_chain2.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "horseshoe or c4_residual or lag_all_models" > gpurun_out/tests_hs.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/tests_hs.log; exit 1; }
tail -1 gpurun_out/tests_hs.log
for n in 4096 100000; do
  timeout -k 10 300 python bench.py --config c4 --N $n --steps 5 --warmup 10 --no-cpu-baseline --profile-solve > gpurun_out/chain2_c4_$n.log 2>&1 || { echo "DIAG FAILED"; tail -30 gpurun_out/chain2_c4_$n.log; exit 1; }
  python3 - gpurun_out/chain2_c4_$n.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); g=d['config']['diag']
print(sys.argv[1], d['value'], d['roofline']['per_block_us'], g['solve_phase_us'], g['solve_chain_loop_cycles_per_step'], {k:g['block_events_us'][k] for k in ('period','solver_wait','solver_chain','lat_apply_last','lat_items_last','lat_l2_last')})
PY
done
