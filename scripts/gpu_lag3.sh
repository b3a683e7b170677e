#!/bin/bash
# A/B: pipeline lag 2 (default) vs 3 for C2 f32
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for lag in 2 3; do
    BRR_LAG=$lag timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/lag3_${lag}_$rep.log 2>&1 \
      || { echo "BENCH lag $lag FAILED"; tail -20 gpurun_out/lag3_${lag}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('lag', sys.argv[2], d['value'], d['ms_per_step'], d['config'].get('pipeline_lag'))" gpurun_out/lag3_${lag}_$rep.log $lag
  done
done
