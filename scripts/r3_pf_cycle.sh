#!/bin/bash
# round 3: GPU suite + same-box A/B of the streamers' list prefetch (C2 f32, driver's 5 + 20 window)
# against the library built from the previous commit (ablib/libbrr_base.so)
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3pf_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r3pf_tests.log
# 0 = green, 1 = a failing test (no fault): the A/B still says something; anything else: stop
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
VARIANTS="${PF_VARIANTS:-base:ablib/libbrr_base.so: new:: nopf::BRR_LIST_PREFETCH=0 base2:ablib/libbrr_base.so: new2::}" \
  bash scripts/r3_variants.sh || exit 1
timeout -k 10 200 python bench.py --steps 3 --warmup 20 --profile-solve --no-cpu-baseline > gpurun_out/r3pf_prof.log 2>&1 || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r3pf_prof.log").read().strip().splitlines()[-1])
dg = d["config"]["diag"]
be = dg.get("block_events_us", {})
print("prefetch frac", dg.get("list_prefetch_frac"), "apply", be.get("wg_apply_ms_pct"), "wait", be.get("wg_wait_ms_pct"),
      "stream", be.get("wg_stream_ms_pct"), "list", be.get("wg_apply_list_ms_pct"), "products", be.get("wg_apply_products_ms_pct"),
      "partbar", be.get("wg_apply_partbar_ms_pct"))
PY
