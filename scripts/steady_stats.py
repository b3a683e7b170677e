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
    rows, solve, stream, split = [], [], [], None
    for f in glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                kn = r.get("Kernel_Name", "")
                if "k_sweep<" in kn:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kn))
                elif "k_sweep_solve<" in kn:
                    solve.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kn))
                elif "k_sweep_stream<" in kn:
                    stream.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kn))
    if not rows and solve and len(solve) == len(stream):
        # the two-kernel sweep (k_sweep_solve beside k_sweep_stream, launched together): one sweep
        # = the span from the first start to the last end of the pair
        solve.sort()
        stream.sort()
        rows = [(min(a[0], b[0]), max(a[1], b[1]), "k_sweep_solve + " + b[2]) for a, b in zip(solve, stream)]
        split = {"solve_us": [(e - s) / 1e3 for s, e, _ in solve], "stream_us": [(e - s) / 1e3 for s, e, _ in stream]}
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
    if split:
        for k, v in split.items():
            out["steady_" + k.replace("_us", "_mean_us")] = sum(v[skip:]) / len(v[skip:])
    with open(prefix + "_steady.json", "w") as fh:
        json.dump(out, fh, indent=1)
    print(prefix, json.dumps(out))


if __name__ == "__main__":
    main()
