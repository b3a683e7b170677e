#!/bin/bash
# C3 / C4 f32 block size: 128 (automatic) vs 256
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for cfg in c3 c4; do
  for b in 128 256; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline --config $cfg --block-size $b > gpurun_out/bc34_${cfg}_$b.log 2>&1 \
      || { echo "BENCH $cfg B=$b FAILED"; tail -20 gpurun_out/bc34_${cfg}_$b.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'B', sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/bc34_${cfg}_$b.log $cfg $b
  done
done
