#!/bin/bash
# bench CONFIGS x block sizes BS with BENCH_ARGS (e.g. --x-storage 2bit); one summary line each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in ${CONFIGS:-c2 c3 c4}; do
  for b in ${BS:-128 256}; do
    timeout -k 10 300 python bench.py --config $c --block-size $b --steps ${STEPS:-10} --warmup ${WARM:-10} --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bs_${c}_${b}.log 2>&1 || { echo "BENCH $c $b FAILED"; tail -5 gpurun_out/bs_${c}_${b}.log; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/bs_${c}_${b}.log').read().strip().splitlines()[-1]); c=d['config']
print('$c', $b, c.get('x_storage'), 'cache', c.get('code_cache'), d['value'], d['ms_per_step'], d['roofline']['per_block_us'])"
  done
done
