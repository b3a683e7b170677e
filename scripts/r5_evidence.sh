#!/bin/bash
# round 5 evidence: rocprofv3 kernel trace + FETCH/WRITE PMC passes (scripts/r5_profile.sh) for the
# configs in CFGS (tag:config:block:storage:alg_bytes[:extra bench flags, comma-separated]).  The PMC
# passes run the one-kernel k_sweep, which instantiates the timed form's streaming variant (C2 f32:
# the list prefetch, C4: the class-code cache k_sweep<true,128,2>).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for c in ${CFGS:-c2_f32:c2:512:f32:2.0e11 c4_f32:c4:128:f32:2.0e11}; do
  IFS=: read -r tag cfg b xs alg extra <<< "$c"
  extra=$(echo "$extra" | tr ',' ' ')
  TAG=${RTAG:-r05}_$tag CONFIG=$cfg B=$b XS=$xs ALG=$alg BENCH_ARGS="--config $cfg $extra" SKIP=${SKIP:-20} \
    bash scripts/r5_profile.sh > gpurun_out/${RTAG:-r05}_${tag}_profile.log 2>&1
  rc=$?
  echo "== $tag rc=$rc"; tail -4 gpurun_out/${RTAG:-r05}_${tag}_profile.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
exit 0
