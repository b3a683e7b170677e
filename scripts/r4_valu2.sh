#!/bin/bash
# round 4: VALU / LDS counters of the 2-bit streaming kernel as the bench runs it (two kernels side by
# side, k_sweep_stream<1, 1024>): counters collected for the streaming kernel only; the bench line
# reports census failures if counter collection kept the two kernels from being co-resident
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04_valu2}
timeout -k 10 -s KILL 150 rocprofv3 --pmc VALUBusy SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-include-regex 'k_sweep_stream' -d gpurun_out/${TAG} -o pmc --output-format csv \
  -- python3 bench.py --steps 2 --warmup 10 --no-roofline-events --no-cpu-baseline --config c2 --x-storage 2bit \
  > gpurun_out/${TAG}.log 2>&1 || { echo "PMC FAILED"; tail -20 gpurun_out/${TAG}.log; exit 1; }
tail -1 gpurun_out/${TAG}.log | cut -c1-400
python3 - "$TAG" <<'PY'
import csv, glob, json, sys
from collections import defaultdict
tag = sys.argv[1]
acc = defaultdict(list)
kern = None
for f in glob.glob(f"gpurun_out/{tag}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "k_sweep_stream" in row.get("Kernel_Name", ""):
            kern = row["Kernel_Name"]
            acc[row["Counter_Name"]].append(float(row["Counter_Value"] or 0))
out = {"kernel": kern, "per_dispatch": {k: v[-2:] for k, v in sorted(acc.items())}}
json.dump(out, open(f"gpurun_out/{tag}_pmc.json", "w"), indent=1)
print(json.dumps(out)[:600])
PY
