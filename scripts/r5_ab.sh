#!/bin/bash
# round 5: same-box A/B of library builds (VARIANTS="name:libpath[:K=V,...]"; empty path = the in-tree build)
# over the configs in CFGS ("name:bench flags, comma-separated"), REPS rounds interleaved; prints value,
# ms/step and the state fingerprint (variants that must run the same chain print the same one).
# PROF="name:flags ..." adds --profile-solve runs of every variant.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r5ab}
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CFGS:-c3:--config,c3 c2:--steps,20,--warmup,5}; do
    cname=${cfg%%:*}; cargs=$(echo ${cfg#*:} | tr ',' ' ')
    for v in ${VARIANTS:-head:}; do
      IFS=: read -r vname lib venv <<< "$v"
      if [ -n "$lib" ]; then export BRR_LIB=$lib; else unset BRR_LIB; fi
      env $(echo "$venv" | tr "," " ") timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-roofline-events $cargs > gpurun_out/${TAG}_${cname}_${vname}_$rep.log 2>&1 \
        || { echo "$cname $vname FAILED"; tail -20 gpurun_out/${TAG}_${cname}_${vname}_$rep.log; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$rep $cname $vname', d['value'], d['ms_per_step'], d['config']['diag'].get('state_sha16'), 'census', d['config'].get('census_failures'))" gpurun_out/${TAG}_${cname}_${vname}_$rep.log
    done
  done
done
for cfg in $PROF; do
  cname=${cfg%%:*}; cargs=$(echo ${cfg#*:} | tr ',' ' ')
  for v in ${VARIANTS:-head:}; do
    IFS=: read -r vname lib venv <<< "$v"
    if [ -n "$lib" ]; then export BRR_LIB=$lib; else unset BRR_LIB; fi
    env $(echo "$venv" | tr "," " ") timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-roofline-events --profile-solve --steps 2 $cargs > gpurun_out/${TAG}_prof_${cname}_${vname}.log 2>&1 || { echo "prof $cname $vname FAILED"; exit 1; }
    python3 - gpurun_out/${TAG}_prof_${cname}_${vname}.log "$cname $vname" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
dg = d['config']['diag']
be = dg.get('block_events_us', {})
print(sys.argv[2], d['ms_per_step'], {k: dg.get(k) for k in ('solve_phase_us', 'solve_wait_us', 'solve_phaseA_us', 'solve_chain_steps', 'solve_correct_us', 'solve_ring_rows', 'solve_global_rows')})
print('   ', {k: be.get(k) for k in ('period', 'solver_wait', 'solver_chain', 'wg_wait_ms_pct', 'wg_apply_ms_pct', 'wg_stream_ms_pct')})
PY
  done
done
unset BRR_LIB
exit 0
