#!/bin/bash
# C2 2-bit: B = 512 (default) vs 256 (code cache in LDS) vs 384? (multiples of 128 only)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for b in 512 256; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline --x-storage 2bit --block-size $b > gpurun_out/b2bit_${b}_$rep.log 2>&1 \
      || { echo "BENCH B=$b FAILED"; tail -20 gpurun_out/b2bit_${b}_$rep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('B', sys.argv[2], d['value'], d['ms_per_step'], d['config'].get('code_cache'), d['config'].get('pipeline_lag'))" gpurun_out/b2bit_${b}_$rep.log $b
  done
done
