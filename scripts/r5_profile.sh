#!/bin/bash
# round 5 rocprofv3 evidence for the default (two-kernel) sweep:
#   1. kernel trace + stats of the driver's bench command (BENCH_ARGS extra flags), per-sweep spans
#      of k_sweep_solve + k_sweep_stream (scripts/steady_stats.py, SKIP dispatches dropped)
#   2. FETCH_SIZE and WRITE_SIZE in separate PMC passes (scripts/pmc_json.py, ALG bytes per sweep)
#   3. (SOLVE=1) the solver's phase breakdown at a few warmup depths (burn-in diagnosis)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r05_c2_f32}
ARGS="--no-cpu-baseline ${BENCH_ARGS}"
[ "${TRACE:-1}" = 1 ] && { timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o run --output-format csv \
  -- python3 bench.py --steps ${STEPS:-20} --warmup ${WARM:-5} $ARGS > gpurun_out/${TAG}_trace.log 2>&1 \
  || { echo "TRACE FAILED"; tail -30 gpurun_out/${TAG}_trace.log; exit 1; }
f=$(find gpurun_out/${TAG}_trace -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${TAG}_kernel_stats.csv
cut -c1-160 gpurun_out/${TAG}_kernel_stats.csv | head -6
python3 scripts/steady_stats.py gpurun_out/${TAG}_trace ${SKIP:-20} gpurun_out/${TAG}_ksweep || exit 1
tail -1 gpurun_out/${TAG}_trace.log | cut -c1-300; }
if [ -n "$ALG" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    # counter collection serialises dispatches: the two side-by-side kernels of the default sweep
    # cannot be co-resident under it, so the PMC passes count the one-kernel form of the same roles
    # (BRR_FUSED_SINGLE=1), which since round 5 instantiates the timed form's streaming variant: the
    # f32 list prefetch (C2) and the class-code cache (C4: k_sweep<true, 128, 2>)
    BRR_FUSED_SINGLE=1 timeout -k 10 -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex 'k_sweep' -d gpurun_out/${TAG}_pmc_$c -o pmc \
      --output-format csv -- python3 bench.py --steps 2 --warmup 10 --no-roofline-events $ARGS \
      > gpurun_out/${TAG}_pmc_$c.log 2>&1 || { echo "PMC $c FAILED"; tail -20 gpurun_out/${TAG}_pmc_$c.log; exit 1; }
  done
  python3 scripts/pmc_json.py gpurun_out/${TAG}_pmc_FETCH_SIZE gpurun_out/${TAG}_pmc_WRITE_SIZE ${CONFIG:-c2} ${B:-512} \
    ${XS:-f32} ${ALG} gpurun_out/${TAG}_pmc.json || exit 1
fi
if [ "${SOLVE:-0}" = 1 ]; then
  for w in ${SOLVE_W:-4 8 20}; do
    timeout -k 10 300 python bench.py --steps 1 --warmup $w --profile-solve --no-cpu-baseline --no-roofline-events $BENCH_ARGS > gpurun_out/${TAG}_solve_w$w.log 2>&1 || { echo PROF FAILED; tail -20 gpurun_out/${TAG}_solve_w$w.log; exit 1; }
    echo "== warmup $w"
    python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_solve_w$w.log').read().strip().splitlines()[-1]);dg=d['config']['diag'];[print(k, v) for k, v in dg.items() if k.startswith('solve') or k=='block_events_us']"
  done
fi
if [ "${REF:-0}" = 1 ]; then
  # where a REFERENCE-order sweep's time goes (Gram blocks recomputed every sweep)
  for rb in ${REF_B:-512 128}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_ref$rb -o run --output-format csv \
      -- python3 bench.py --order reference --block-size $rb --steps 2 --warmup 1 --no-roofline-events $ARGS > gpurun_out/${TAG}_ref$rb.log 2>&1 \
      || { echo "REF FAILED"; tail -30 gpurun_out/${TAG}_ref$rb.log; exit 1; }
    echo "== reference order B = $rb"
    cut -c1-160 $(find gpurun_out/${TAG}_ref$rb -name "*kernel_stats.csv" | head -1) | head -8
    tail -1 gpurun_out/${TAG}_ref$rb.log | cut -c1-300
  done
fi
exit 0
