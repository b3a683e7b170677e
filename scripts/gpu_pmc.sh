#!/bin/bash
# HBM traffic of k_stream from PMC counters (separate passes: FETCH_SIZE and WRITE_SIZE do not
# fit one TCC pass on gfx950), on a short C2 run.  Summaries land in gpurun_out/pmc_*.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $c --kernel-include-regex 'k_stream|k_solve' -d gpurun_out/pmc_$c -o pmc --output-format csv \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-roofline-events ${BENCH_ARGS} > gpurun_out/pmc_$c.log 2>&1 \
    || { echo "PMC $c FAILED"; tail -20 gpurun_out/pmc_$c.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc_FETCH_SIZE gpurun_out/pmc_WRITE_SIZE > gpurun_out/pmc_summary.txt && cat gpurun_out/pmc_summary.txt
