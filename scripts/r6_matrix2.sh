#!/bin/bash
# round 6: one pytest selection under several environment variants (VARIANTS="name:ENV=1,ENV2=0 ..."),
# each its own process and log; reports every variant (does not stop at the first failure).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r06x}
for v in $VARIANTS; do
  name=${v%%:*}; envs=${v#*:}
  ( IFS=','; for e in $envs; do [ -n "$e" ] && export "$e"; done
    timeout -k 10 ${TEST_TIMEOUT:-300} python -u -m pytest $SEL ${KSEL:+-k "$KSEL"} -m gpu -q --timeout 120 --timeout-method thread \
      > gpurun_out/${TAG}_$name.log 2>&1 )
  rc=$?
  echo "== $name rc=$rc: $(tail -1 gpurun_out/${TAG}_$name.log)"
  grep -E "AssertionError" gpurun_out/${TAG}_$name.log | head -4
  [ $rc = 124 ] || [ $rc = 137 ] || [ $rc -ge 128 ] && exit $rc
done
exit 0
