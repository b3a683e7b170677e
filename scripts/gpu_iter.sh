#!/bin/bash
# iteration check: chain microbenchmark, full GPU test suite, then C2/C3/C4 benches with the
# solver phase breakdown (CONFIGS overrides)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
if [ -x scripts/mb_chain2.bin ]; then timeout -k 10 60 ./scripts/mb_chain2.bin > gpurun_out/mb_chain2.log 2>&1 && cat gpurun_out/mb_chain2.log; fi
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${TESTSEL:+-k "$TESTSEL"} > gpurun_out/tests_iter.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|error|assert" gpurun_out/tests_iter.log | head -20; tail -5 gpurun_out/tests_iter.log; exit 1; }
tail -1 gpurun_out/tests_iter.log
fi
for c in ${CONFIGS:-c2 c3 c4}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 10 --no-cpu-baseline --profile-solve ${BENCH_ARGS} > gpurun_out/iter_$c.log 2>&1 || { echo "BENCH $c FAILED"; tail -30 gpurun_out/iter_$c.log; exit 1; }
  python3 - gpurun_out/iter_$c.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); g=d['config']['diag']
be=g.get('block_events_us',{})
print(sys.argv[1], d['value'], 'frac', d['roofline']['frac'], 'blk', d['roofline']['per_block_us'], g.get('solve_phase_us'), 'cyc/step', g.get('solve_chain_loop_cycles_per_step'), 'steps', g.get('solve_chain_steps'), {k:be.get(k) for k in ('period','solver_wait','solver_chain','lat_apply_last','lat_items_last','lat_l2_last')}, 'wg_ms', be.get('wg_wait_ms_pct',[None]*3)[2], be.get('wg_apply_ms_pct',[None]*3)[2], be.get('wg_stream_ms_pct',[None]*3)[2])
PY
done
