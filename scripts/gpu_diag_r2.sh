#!/bin/bash
# round-2 diagnostics: solver phase breakdown for C3/C4, one C5 rank (P_local = 125k) on 1 GPU,
# C5 whole (P = 1M) at 2-bit storage on 1 GPU
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
for c in c3 c4; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 10 --no-cpu-baseline --profile-solve > gpurun_out/diag_$c.log 2>&1 || { echo "DIAG $c FAILED"; tail -30 gpurun_out/diag_$c.log; exit 1; }
  tail -1 gpurun_out/diag_$c.log | cut -c1-300
done
timeout -k 10 400 python bench.py --config c5 --P 125000 --steps 10 --warmup 10 --no-cpu-baseline > gpurun_out/c5rank.log 2>&1 || { echo "C5 rank FAILED"; tail -30 gpurun_out/c5rank.log; exit 1; }
tail -1 gpurun_out/c5rank.log | cut -c1-400
timeout -k 10 400 python bench.py --config c5 --x-storage 2bit --steps 10 --warmup 10 --no-cpu-baseline > gpurun_out/c5_2bit.log 2>&1 || { echo "C5 2bit FAILED"; tail -30 gpurun_out/c5_2bit.log; exit 1; }
tail -1 gpurun_out/c5_2bit.log | cut -c1-400
