#!/bin/bash
# round 3: driver-equivalent bench + per-sweep burn-in trace (B = 512 lag 2, B = 128, lag 1)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3_bench_default.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/r3_bench_default.log; exit 1; }
tail -1 gpurun_out/r3_bench_default.log | cut -c1-400
for args in "" "--block-size 256" "--block-size 128"; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 25 --trace-sweeps 1 --no-cpu-baseline --no-roofline-events $args > gpurun_out/r3_trace.log 2>&1 || { echo TRACE FAILED; tail -20 gpurun_out/r3_trace.log; exit 1; }
  echo "== $args"
  python3 -c "import json;d=json.loads(open('gpurun_out/r3_trace.log').read().strip().splitlines()[-1]);print(d['value'], d['config']['diag']['sweep_trace_ms_changed']['warmup'])"
done
for lag in 1 3; do
  BRR_LAG=$lag timeout -k 10 300 python bench.py --steps 5 --warmup 25 --trace-sweeps 1 --no-cpu-baseline --no-roofline-events > gpurun_out/r3_trace.log 2>&1 || { echo TRACE FAILED; tail -20 gpurun_out/r3_trace.log; exit 1; }
  echo "== lag $lag"
  python3 -c "import json;d=json.loads(open('gpurun_out/r3_trace.log').read().strip().splitlines()[-1]);print(d['value'], d['config']['diag']['sweep_trace_ms_changed']['warmup'])"
done
