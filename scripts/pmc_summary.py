"""Average per-dispatch PMC values per kernel from rocprofv3 counter_collection.csv files."""
import csv
import glob
import os
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    acc = defaultdict(lambda: [0.0, 0])
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = (row.get("Kernel_Name", "?")[:60], row.get("Counter_Name", "?"))
                acc[k][0] += float(row.get("Counter_Value", 0) or 0)
                acc[k][1] += 1
    for (kern, ctr), (tot, n) in sorted(acc.items()):
        print(f"{d}\t{kern}\t{ctr}\tdispatches={n}\tavg={tot / max(1, n):.6g}")
