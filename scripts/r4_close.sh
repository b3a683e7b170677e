#!/bin/bash
# round 4 closing run on the committed tree: GPU suite, smoke(), the driver's default bench line,
# then one bench line per BASELINE config (and the one-shot, REFERENCE order, one C5 rank)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04z}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail 8 --timeout 150 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -eq 0 ] || { echo "GPU TESTS FAILED rc=$rc"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
  || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
echo "== default bench"; tail -1 gpurun_out/${TAG}_bench.log | cut -c1-700
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_driver_window.log 2>&1 \
  || { echo "driver-window bench failed"; exit 1; }
echo "== driver window"; tail -1 gpurun_out/${TAG}_bench_driver_window.log | cut -c1-300
RUNS=${RUNS:-"c3:--config,c3 c4:--config,c4 c2_2bit:--x-storage,2bit c1:--config,c1 oneshot:--oneshot ref:--order,reference c5rank:--config,c5"} \
  TESTS=0 TAG=$TAG RUN_TIMEOUT=300 bash scripts/r4_run.sh
