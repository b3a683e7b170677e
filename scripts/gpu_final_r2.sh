#!/bin/bash
# Round-2 closing run: full GPU suite, smoke(), the default bench line, and the other configs'
# bench lines (logs under gpurun_out/final_*)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/final_gpu_tests.log 2>&1 || { echo "TESTS FAILED"; tail -20 gpurun_out/final_gpu_tests.log; exit 1; }
tail -1 gpurun_out/final_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 \
  || { echo "SMOKE FAILED"; tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -2 gpurun_out/final_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final_bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/final_bench.log; exit 1; }
tail -1 gpurun_out/final_bench.log | cut -c1-600
for spec in "c2_2bit --x-storage 2bit" "c4_f32 --config c4" "c4_2bit --config c4 --x-storage 2bit" "c3_f32 --config c3"; do
  read -r tag args <<< "$spec"
  timeout -k 10 300 python bench.py --steps 20 --warmup 10 --no-cpu-baseline $args > gpurun_out/final_$tag.log 2>&1 \
    || { echo "BENCH $tag FAILED"; tail -20 gpurun_out/final_$tag.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/final_$tag.log $tag
done
