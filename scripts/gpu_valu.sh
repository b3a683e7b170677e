#!/bin/bash
# VALU / LDS activity of the steady-state k_sweep (one PMC pass per storage): is the 2-bit sweep
# bound by the streamers' decode-dot instructions?
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
# (counter collection serialises dispatches: the one-kernel form of the sweep's roles, plain launch)
export TMPDIR=/tmp BRR_FUSED_SINGLE=1
for xs in ${XS_LIST:-2bit f32}; do
  timeout -k 10 -s KILL 240 rocprofv3 --pmc VALUBusy SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
    --kernel-include-regex 'k_sweep' -d gpurun_out/${TAG:-valu}_$xs -o pmc --output-format csv \
    -- python3 bench.py --steps 2 --warmup 10 --no-roofline-events --no-cpu-baseline --config c2 --x-storage $xs \
    > gpurun_out/${TAG:-valu}_$xs.log 2>&1 || { echo "PMC $xs FAILED"; tail -20 gpurun_out/${TAG:-valu}_$xs.log; exit 1; }
  find gpurun_out/${TAG:-valu}_$xs -name "*counter_collection.csv" | head -1
done
python3 - "${TAG:-valu}" <<'PY'
import csv, glob, json, sys
from collections import defaultdict
tag = sys.argv[1]
out = {}
for xs in ("2bit", "f32"):
    files = glob.glob(f"gpurun_out/{tag}_{xs}/**/*counter_collection.csv", recursive=True)
    acc = defaultdict(list)
    kern = None
    for f in files:
        for row in csv.DictReader(open(f)):
            if "k_sweep<" in row.get("Kernel_Name", ""):
                kern = row["Kernel_Name"]
                acc[row["Counter_Name"]].append(float(row["Counter_Value"] or 0))
    if acc:
        # the last two dispatches: the steady sweeps after the burn-in
        out[xs] = {"kernel": kern, "per_dispatch": {k: v[-2:] for k, v in sorted(acc.items())}}
json.dump(out, open(f"gpurun_out/{tag}_pmc.json", "w"), indent=1)
print(json.dumps({xs: d["per_dispatch"].get("VALUBusy") for xs, d in out.items()}))
PY
