#!/bin/bash
# round 3 closing evidence: GPU suite + smoke + driver bench + two configs, then the config tests
# (C1 at its stated shape, one C5 rank) twice more in their own processes
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03e} CONFIGS="${CONFIGS:-c3:--config,c3 c2_2bit:--config,c2,--x-storage,2bit}" bash scripts/r3_evidence.sh \
  > gpurun_out/${TAG:-r03e}_evidence.log 2>&1
rc=$?
cut -c1-300 gpurun_out/${TAG:-r03e}_evidence.log
[ $rc -eq 0 ] || exit $rc
for i in ${REPS:-1 2}; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_configs.py -m gpu -q --timeout 150 --timeout-method thread \
    > gpurun_out/${TAG:-r03e}_configs_$i.log 2>&1
  r=$?
  echo "configs rep $i rc=$r"; tail -1 gpurun_out/${TAG:-r03e}_configs_$i.log
  [ $r -eq 0 ] || [ $r -eq 1 ] || exit $r
done
