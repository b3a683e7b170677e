#!/bin/bash
# C2 bench under a list of environment settings (SCAN="VAR=val VAR2=val;VAR=val ..."), one line each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
IFS=';' read -ra SETS <<< "$SCAN"
i=0
for s in "${SETS[@]}"; do
  i=$((i+1))
  env $s timeout -k 10 300 python bench.py --steps ${STEPS:-5} --warmup ${WARM:-8} --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/scan_$i.log 2>&1 || { echo "SCAN [$s] FAILED"; tail -5 gpurun_out/scan_$i.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/scan_$i.log').read().strip().splitlines()[-1])
print('[$s]', d['value'], d['ms_per_step'], d['config']['fused_stream_wg'], d['roofline']['avg_launch_us'])"
done
