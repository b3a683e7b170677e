#!/bin/bash
# round 3 closing run on the committed tree: r3_final.sh (suite, smoke, driver bench, configs, config
# tests) and the rocprofv3 kernel trace + PMC passes of the default C2 sweep (r3_profile.sh)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
TAG=r03f CONFIGS="c3:--config,c3 c4:--config,c4 c2_2bit:--config,c2,--x-storage,2bit c1:--config,c1" REPS=1 \
  bash scripts/r3_final.sh > gpurun_out/r03f_final.log 2>&1
rc=$?
cut -c1-250 gpurun_out/r03f_final.log
[ $rc -eq 0 ] || exit $rc
TAG=r03f_c2_f32 ALG=2.0e11 bash scripts/r3_profile.sh > gpurun_out/r03f_profile.log 2>&1
rc=$?
cut -c1-250 gpurun_out/r03f_profile.log
exit $rc
