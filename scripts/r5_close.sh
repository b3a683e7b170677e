#!/bin/bash
# round 5 evidence run: rocprofv3 traces + FETCH/WRITE PMC passes of the timed paths (C2 f32, C3, C4:
# scripts/r5_evidence.sh), the default bench line with its CPU baseline, output off / on at C2 in the
# same call, and a kernel trace of the REFERENCE visit order.  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${RTAG:-r05}
if [ "${EVID:-1}" = 1 ]; then
  RTAG=$T CFGS=${CFGS:-"c2_f32:c2:512:f32:2.0e11 c4_f32:c4:128:f32:2.0e11 c3_f32:c3:128:f32:2.0e11"} bash scripts/r5_evidence.sh || exit 1
fi
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || { echo "default bench FAILED"; tail -20 gpurun_out/${T}_bench.log; exit 1; }
echo "== default bench"; tail -1 gpurun_out/${T}_bench.log | cut -c1-400
python3 -c "import json;d=json.loads(open('gpurun_out/${T}_bench.log').read().strip().splitlines()[-1]);print('cpu_baseline', json.dumps(d['cpu_baseline']))"
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 --warmup 10 > gpurun_out/${T}_c2_output_off_$rep.log 2>&1 || { echo "output-off FAILED"; exit 1; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 --warmup 10 --emit gpurun_out/${T}_c2_emit.csv --emit-thin 10 > gpurun_out/${T}_c2_output_on_$rep.log 2>&1 || { echo "output-on FAILED"; tail -20 gpurun_out/${T}_c2_output_on_$rep.log; exit 1; }
  for f in off on; do python3 -c "import json;d=json.loads(open('gpurun_out/${T}_c2_output_${f}_$rep.log').read().strip().splitlines()[-1]);print('output-$f $rep', d['value'], d['ms_per_step'], d['config'].get('output'))"; done
done
rm -f gpurun_out/${T}_c2_emit.csv
if [ "${REFTRACE:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_ref_trace -o run --output-format csv \
    -- python3 bench.py --order reference --steps 6 --warmup 2 --no-cpu-baseline --no-roofline-events > gpurun_out/${T}_ref_trace.log 2>&1 \
    || { echo "REF trace FAILED"; tail -20 gpurun_out/${T}_ref_trace.log; exit 1; }
  f=$(find gpurun_out/${T}_ref_trace -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/${T}_ref_kernel_stats.csv
  cut -c1-150 gpurun_out/${T}_ref_kernel_stats.csv | head -12
  tail -1 gpurun_out/${T}_ref_trace.log | cut -c1-300
fi
exit 0
