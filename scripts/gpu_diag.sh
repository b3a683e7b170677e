#!/bin/bash
# solver phase breakdown + per-block event medians for each single-GPU config
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for c in ${CONFIGS:-c2 c3 c4}; do
  timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-5} --warmup ${WARM:-10} --no-cpu-baseline --profile-solve ${BENCH_ARGS} > gpurun_out/diag_$c.log 2>&1 || { echo "DIAG $c FAILED"; tail -30 gpurun_out/diag_$c.log; exit 1; }
  python3 -c "
import json
d=json.loads(open('gpurun_out/diag_$c.log').read().strip().splitlines()[-1])
print('$c', d['value'], d['ms_per_step'], d['roofline']['per_block_us'] if d['roofline'] else None)
print(json.dumps(d['config']['diag']))"
done
