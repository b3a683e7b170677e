#!/bin/bash
# Round-2 evidence: rocprofv3 trace (steady-state k_sweep summary) + PMC for C2 / C3 / C4 f32,
# the C1 one-shot end to end beside the CPU oracle, and the C2 output-on run.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for c in ${PCONFIGS:-c2 c3 c4}; do
  B=512; [ "$c" != c2 ] && B=128
  TAG=r02_${c}_f32 CONFIG=$c XS=f32 B=$B ALG=200000000000 bash scripts/gpu_profile.sh || exit 1
done
if [ -z "$NO_SIDE" ]; then
timeout -k 10 600 python3 bench.py --oneshot --cpu-iters 100 > gpurun_out/r02_c1_oneshot.log 2>&1 || { echo C1 FAILED; tail -20 gpurun_out/r02_c1_oneshot.log; exit 1; }
tail -1 gpurun_out/r02_c1_oneshot.log | cut -c1-600
timeout -k 10 600 python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline --emit /tmp/brr_c2_emit.csv --emit-thin 10 > gpurun_out/r02_c2_emit.log 2>&1 || { echo EMIT FAILED; tail -20 gpurun_out/r02_c2_emit.log; exit 1; }
tail -1 gpurun_out/r02_c2_emit.log | cut -c1-300
fi
