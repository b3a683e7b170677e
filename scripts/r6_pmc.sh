#!/bin/bash
# round 6: FETCH_SIZE / WRITE_SIZE of the TIMED two-kernel sweep.  Only k_sweep_stream is profiled
# (--kernel-include-regex): the solver kernel is not, so it runs beside it as in the timed bench (the
# census in the bench line says whether they were co-resident), and the device's TCC counters over
# the streaming kernel's dispatch cover both.  One configuration per call of this script:
#   TAG, BENCH_ARGS, CONFIG, B, XS, ALG (algorithmic bytes per sweep)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r06_c2_2bit}
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex 'k_sweep_stream' -d gpurun_out/${TAG}_pmc_$c -o pmc \
    --output-format csv -- python3 bench.py --steps 2 --warmup 10 --no-roofline-events --no-cpu-baseline ${BENCH_ARGS} \
    > gpurun_out/${TAG}_pmc_$c.log 2>&1 || { echo "PMC $c FAILED"; tail -20 gpurun_out/${TAG}_pmc_$c.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$c pass: census_failures', d['config'].get('census_failures'), 'value', d['value'])" gpurun_out/${TAG}_pmc_$c.log
done
python3 scripts/pmc_json.py gpurun_out/${TAG}_pmc_FETCH_SIZE gpurun_out/${TAG}_pmc_WRITE_SIZE ${CONFIG:-c2} ${B:-512} \
  ${XS:-2bit} ${ALG} gpurun_out/${TAG}_pmc.json || exit 1
