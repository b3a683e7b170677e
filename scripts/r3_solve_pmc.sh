#!/bin/bash
# round 3: what the per-block k_solve spends its cycles on in burn-in sweeps (C2 f32, B = 512)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
export BRR_PER_BLOCK=1
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/r3_avail.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3_solve_trace -o run --output-format csv -- python3 bench.py --steps 1 --warmup 4 --no-cpu-baseline --no-roofline-events > gpurun_out/r3_solve_trace.log 2>&1 || { echo TRACE FAILED; tail -5 gpurun_out/r3_solve_trace.log; }
for w in 4 20; do
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM --kernel-include-regex 'k_solve' -d gpurun_out/r3_solve_pmc_w$w -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup $w --no-cpu-baseline --no-roofline-events > gpurun_out/r3_solve_pmc_w$w.log 2>&1 || { echo "PMC w$w FAILED"; tail -5 gpurun_out/r3_solve_pmc_w$w.log; }
done
ls -R gpurun_out/r3_solve_pmc_w4 | head
