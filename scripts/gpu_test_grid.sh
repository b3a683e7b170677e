#!/bin/bash
# GPU parity tests, then a config x block-size grid (scripts/gpu_bsizes.sh)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -q -m gpu -p no:cacheprovider -x --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
bash scripts/gpu_bsizes.sh
