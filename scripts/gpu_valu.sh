#!/bin/bash
# VALU / LDS activity of the steady-state k_sweep (one PMC pass per storage): is the 2-bit sweep
# bound by the streamers' decode-dot instructions?
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp BRR_PLAIN_LAUNCH=1
for xs in 2bit f32; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc VALUBusy SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
    --kernel-include-regex 'k_sweep' -d gpurun_out/valu_$xs -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 10 --no-roofline-events --no-cpu-baseline --config c2 --x-storage $xs \
    > gpurun_out/valu_$xs.log 2>&1 || { echo "PMC $xs FAILED"; tail -20 gpurun_out/valu_$xs.log; exit 1; }
  find gpurun_out/valu_$xs -name "*counter_collection.csv" | head -1
done
