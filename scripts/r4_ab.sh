#!/bin/bash
# round 4: same-box A/B of library builds (VARIANTS="name:libpath ..."; empty path = the in-tree build)
# over the configs in CFGS ("name:bench flags, comma-separated"), REPS rounds interleaved
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CFGS:-c3:--config,c3 c2:--steps,20,--warmup,5}; do
    cname=${cfg%%:*}; cargs=$(echo ${cfg#*:} | tr ',' ' ')
    for v in ${VARIANTS:-head:}; do
      # name:library[:K=V] (empty library: the in-tree build; K=V: an environment variable for this variant)
      IFS=: read -r vname lib venv <<< "$v"
      if [ -n "$lib" ]; then export BRR_LIB=$lib; else unset BRR_LIB; fi
      env $(echo "$venv" | tr "," " ") timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-roofline-events $cargs > gpurun_out/r4ab_${cname}_${vname}_$rep.log 2>&1 \
        || { echo "$cname $vname FAILED"; tail -20 gpurun_out/r4ab_${cname}_${vname}_$rep.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$rep $cname $vname', d['value'], d['ms_per_step'])" gpurun_out/r4ab_${cname}_${vname}_$rep.log
    done
  done
done
unset BRR_LIB
if [ -n "$PROF" ]; then
  for cfg in $PROF; do
    cname=${cfg%%:*}; cargs=$(echo ${cfg#*:} | tr ',' ' ')
    timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-roofline-events --profile-solve --steps 2 $cargs > gpurun_out/r4prof_$cname.log 2>&1 || { echo "prof $cname FAILED"; exit 1; }
    python3 - gpurun_out/r4prof_$cname.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
dg = d['config']['diag']
be = dg.get('block_events_us', {})
print(sys.argv[1], {k: dg.get(k) for k in ('solve_phase_us', 'solve_wait_us', 'solve_phaseA_us', 'solve_chain_steps')})
print('   ', {k: be.get(k) for k in ('period', 'solver_wait', 'solver_chain', 'lat_apply_last', 'lat_items_last', 'lat_l2_last', 'lat_solver_sees', 'wg_wait_ms_pct', 'wg_apply_ms_pct', 'wg_stream_ms_pct', 'wg_apply_list_ms_pct', 'wg_apply_products_ms_pct', 'wg_apply_partbar_ms_pct')})
PY
  done
fi
exit 0
