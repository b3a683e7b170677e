#!/bin/bash
# Submit one gpurun command; if no box / slot was free (nothing ran, nothing charged: exit 3 or a
# "transient" status with 0 s run), wait and submit it again -- at most TRIES times, WAIT s apart.
# A command that ran (whatever its result) is never resubmitted.
cmd="$1"
out=${OUT:-/tmp/gpurun_last.txt}
for i in $(seq 1 ${TRIES:-8}); do
  timeout ${OUTER:-2000} /usr/local/graft/bin/gpurun --timeout ${LIMIT:-1200} -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "run 0.0s of limit\|run Nones of limit" "$out"; then
    echo "attempt $i: no box (rc=$rc); waiting" >> "$out.attempts"
    sleep ${WAIT:-330}
    continue
  fi
  echo "attempt $i: ran (rc=$rc)" >> "$out.attempts"
  exit $rc
done
exit 3
