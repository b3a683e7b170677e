#!/bin/bash
# variant sweep: config / storage / lag combinations (bench --profile-solve), one line each
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
run() {  # tag, env, args
  local tag=$1; shift; local envs=$1; shift
  env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 10 --no-cpu-baseline --profile-solve "$@" > gpurun_out/var_$tag.log 2>&1 || { echo "VAR $tag FAILED"; tail -5 gpurun_out/var_$tag.log; return 1; }
  python3 - gpurun_out/var_$tag.log $tag <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); g=d['config']['diag']; be=g.get('block_events_us',{})
print(sys.argv[2], d['value'], 'blk', d['roofline']['per_block_us'], 'lag', d['config']['pipeline_lag'], g.get('solve_phase_us'), g.get('solve_phaseA_us'), 'wait', g.get('solve_wait_us'), {k:be.get(k) for k in ('period','solver_wait','solver_chain','lat_apply_last','lat_items_last','lat_l2_last')}, 'wg', be.get('wg_wait_ms_pct',[None]*3)[2], be.get('wg_apply_ms_pct',[None]*3)[2], be.get('wg_stream_ms_pct',[None]*3)[2], 'apply list/products', be.get('wg_apply_list_ms_pct',[None]*3)[2], be.get('wg_apply_products_ms_pct',[None]*3)[2], be.get('wg_apply_partbar_ms_pct',[None]*3)[2], be.get('wg_apply_stage_ms_pct',[None]*3)[2])
PY
}
IFS=';' read -r -a specs <<< "${VARIANTS}"
for spec in "${specs[@]}"; do
  read -r tag envs args <<< "$spec"
  run $tag "$envs" $args || exit 1
done
