"""Steady-state per-dispatch summary of the fused sweep kernel from a rocprofv3 kernel trace.

usage: steady_stats.py TRACE_DIR SKIP OUT_PREFIX

rocprofv3's kernel_stats.csv averages over every dispatch, including the burn-in sweeps of a
fresh chain (the first sweeps from beta = 0 change ~25 % of the markers and are several times
slower).  This keeps the k_sweep dispatches after the first SKIP (bench.py's --warmup) and writes
OUT_PREFIX_dispatches.csv (one row per dispatch: index, duration us) and OUT_PREFIX_steady.json
(calls, mean / min / max us over the steady-state dispatches) -- the figure bench.py's roofline
'avg_launch_us' is compared with.
"""
import csv
import glob
import json
import os
import sys


def main():
    tdir, skip, prefix = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    rows = []
    for f in glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "k_sweep<" in r.get("Kernel_Name", ""):
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if not rows:
        sys.exit("no k_sweep dispatches in the trace")
    dur = [(e - s) / 1e3 for s, e, _ in rows]
    with open(prefix + "_dispatches.csv", "w") as fh:
        fh.write("dispatch,duration_us,steady_state\n")
        for i, d in enumerate(dur):
            fh.write(f"{i},{d:.3f},{int(i >= skip)}\n")
    ss = dur[skip:]
    out = {"kernel": rows[0][2][:80], "dispatches": len(dur), "skipped_burn_in": skip, "calls": len(ss),
           "mean_us": sum(ss) / len(ss), "min_us": min(ss), "max_us": max(ss),
           "all_dispatch_mean_us": sum(dur) / len(dur)}
    with open(prefix + "_steady.json", "w") as fh:
        json.dump(out, fh, indent=1)
    print(prefix, json.dumps(out))


if __name__ == "__main__":
    main()
