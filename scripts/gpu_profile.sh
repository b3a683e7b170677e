#!/bin/bash
# rocprofv3 evidence for one bench configuration:
#   kernel trace + stats of `bench.py --steps 5`, then FETCH_SIZE and WRITE_SIZE in separate PMC
#   passes, summarised by scripts/pmc_json.py into gpurun_out/<TAG>_pmc.json.
# env: TAG (file prefix), CONFIG (c2|c3|c4), XS (f32|2bit), B (block size), ALG (algorithmic bytes
#      per k_sweep launch), BENCH_ARGS (extra bench flags)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
# rocprofv3 + cooperative launch: segfault at process exit (tool teardown); profile the plain
# launch of the same kernel
export BRR_PLAIN_LAUNCH=1
TAG=${TAG:-prof}
ARGS="--config ${CONFIG:-c2} --x-storage ${XS:-f32} --no-cpu-baseline ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_trace -o run --output-format csv \
  -- python3 bench.py --steps 5 --warmup 10 $ARGS > gpurun_out/${TAG}_trace.log 2>&1 \
  || { echo "TRACE FAILED"; tail -30 gpurun_out/${TAG}_trace.log; exit 1; }
f=$(find gpurun_out/${TAG}_trace -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${TAG}_kernel_stats.csv
cut -c1-200 gpurun_out/${TAG}_kernel_stats.csv | head -8
python3 scripts/steady_stats.py gpurun_out/${TAG}_trace 10 gpurun_out/${TAG}_ksweep || exit 1
tail -1 gpurun_out/${TAG}_trace.log | cut -c1-400
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex 'k_sweep' -d gpurun_out/${TAG}_pmc_$c -o pmc \
    --output-format csv -- python3 bench.py --steps 2 --warmup 10 --no-roofline-events $ARGS \
    > gpurun_out/${TAG}_pmc_$c.log 2>&1 || { echo "PMC $c FAILED"; tail -20 gpurun_out/${TAG}_pmc_$c.log; exit 1; }
done
python3 scripts/pmc_json.py gpurun_out/${TAG}_pmc_FETCH_SIZE gpurun_out/${TAG}_pmc_WRITE_SIZE ${CONFIG:-c2} ${B:-512} \
  ${XS:-f32} ${ALG} gpurun_out/${TAG}_pmc.json
