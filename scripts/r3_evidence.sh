#!/bin/bash
# round 3 evidence on the committed tree: the -m gpu suite, smoke(), the driver's default bench,
# then one bench line per single-GPU config (CONFIGS, "name:args" pairs)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03}
if [ "${TESTS:-all}" != "none" ]; then
  T=${TESTS:-tests}; [ "$T" = all ] && T=tests
  timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu $T > gpurun_out/${TAG}_gpu_tests.log 2>&1; rc=$?
  tail -3 gpurun_out/${TAG}_gpu_tests.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/${TAG}_gpu_tests.log | head -20; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -1 gpurun_out/${TAG}_smoke.log
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log | cut -c1-600
for c in ${CONFIGS:-c2_2bit:--config,c2,--x-storage,2bit c3:--config,c3 c4:--config,c4 c4_2bit:--config,c4,--x-storage,2bit}; do
  name=${c%%:*}; args=${c#*:}
  timeout -k 10 400 python bench.py --no-cpu-baseline ${args//,/ } > gpurun_out/${TAG}_$name.log 2>&1 || { echo "BENCH $name FAILED"; tail -20 gpurun_out/${TAG}_$name.log; exit 1; }
  echo "== $name"; tail -1 gpurun_out/${TAG}_$name.log | cut -c1-300
done
exit 0
