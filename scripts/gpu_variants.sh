#!/bin/bash
# A/B of kernel variants (variants/libbrr_*.so) on the C2 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in variants/libbrr_*.so; do
  name=$(basename $lib .so)
  BRR_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup ${WARM:-8} --block-size ${BS:-512} --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/var_$name.log 2>&1 || { echo "VARIANT $name FAILED"; tail -5 gpurun_out/var_$name.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/var_$name.log').read().strip().splitlines()[-1])
print('$name', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
