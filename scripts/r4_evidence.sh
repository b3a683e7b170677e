#!/bin/bash
# round 4 evidence: rocprofv3 kernel trace + FETCH/WRITE PMC passes (scripts/r4_profile.sh) for the
# configs in CFGS (tag:config:block:storage:alg_bytes[:extra bench flags, comma-separated])
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for c in ${CFGS:-c2_f32:c2:512:f32:2.0e11 c3_f32:c3:128:f32:2.0e11 c4_f32:c4:128:f32:2.0e11 c2_2bit:c2:512:2bit:1.2508e10:--x-storage,2bit}; do
  IFS=: read -r tag cfg b xs alg extra <<< "$c"
  extra=$(echo "$extra" | tr ',' ' ')
  TAG=r04_$tag CONFIG=$cfg B=$b XS=$xs ALG=$alg BENCH_ARGS="--config $cfg $extra" SKIP=${SKIP:-20} \
    bash scripts/r4_profile.sh > gpurun_out/r04_${tag}_profile.log 2>&1
  rc=$?
  echo "== $tag rc=$rc"; tail -4 gpurun_out/r04_${tag}_profile.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
exit 0
