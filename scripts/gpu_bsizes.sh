#!/bin/bash
# config x block-size grid: "c3:128 c3:256 c4:64" ...
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for cb in ${GRID}; do
  c=${cb%%:*}; b=${cb##*:}
  timeout -k 10 300 python bench.py --config $c --block-size $b --steps ${STEPS:-10} --warmup ${WARM:-10} --no-cpu-baseline --profile-solve ${BENCH_ARGS} > gpurun_out/bs_${c}_$b.log 2>&1 || { echo "RUN $cb FAILED"; tail -30 gpurun_out/bs_${c}_$b.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/bs_${c}_$b.log').read().strip().splitlines()[-1])
g=d['config']['diag']
print('$cb', d['value'], d['ms_per_step'], d['roofline']['per_block_us'], 'changed/sweep', round(g['changed_per_sweep']), 'phase', g.get('solve_phase_us'), 'wait', g.get('solve_wait_us'), 'steps', g.get('solve_chain_steps'), 'refr', g.get('solve_refreshes'), g.get('solve_refresh_us'), 'corr', g.get('solve_correct_us'), 'glob', g.get('solve_global_rows'))"
done
