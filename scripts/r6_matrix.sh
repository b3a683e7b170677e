#!/bin/bash
# round 6: run pytest selections under library builds / environment variants, one after another.
# RUNS="name|env assignments (comma-separated)|pytest args (comma-separated)" ...; a failing selection
# (assertions) does not stop the next one, a timeout / crash does.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r06m}
for r in $RUNS; do
  IFS='|' read -r name envs args <<< "$r"
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 ${T:-400} python -u -m pytest -m gpu -q --timeout 150 --timeout-method thread \
    $(echo "$args" | tr ',' ' ') > gpurun_out/${TAG}_$name.log 2>&1
  rc=$?
  echo "== $name rc=$rc: $(tail -1 gpurun_out/${TAG}_$name.log)"
  grep -E "^FAILED|Error:" gpurun_out/${TAG}_$name.log | head -8
  case $rc in 0|1) ;; *) echo "STOP rc=$rc"; exit $rc;; esac
done
exit 0
