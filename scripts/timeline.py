"""Per-block timeline of k_stream / k_solve from a rocprofv3 kernel trace (csv)."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ks = [r for r in rows if "k_stream" in r["Kernel_Name"] or "k_solve" in r["Kernel_Name"]]
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
st = [r for r in ks if "k_stream" in r["Kernel_Name"]]
sv = [r for r in ks if "k_solve" in r["Kernel_Name"]]
n = min(len(st), len(sv))
skip = int(sys.argv[2]) if len(sys.argv) > 2 else n // 2
def t(r, k): return int(r[k]) / 1000.0
print("blocks", n, "analysing", skip, "..", min(n, skip + 12))
t0 = t(st[skip], "Start_Timestamp")
for b in range(skip, min(n, skip + 12)):
    a, c = st[b], sv[b]
    print(f"b={b}: stream {t(a,'Start_Timestamp')-t0:8.1f} .. {t(a,'End_Timestamp')-t0:8.1f} ({t(a,'End_Timestamp')-t(a,'Start_Timestamp'):6.1f})"
          f"   solve {t(c,'Start_Timestamp')-t0:8.1f} .. {t(c,'End_Timestamp')-t0:8.1f} ({t(c,'End_Timestamp')-t(c,'Start_Timestamp'):6.1f})")
import statistics as S
d_st = [t(r, "End_Timestamp") - t(r, "Start_Timestamp") for r in st[skip:]]
d_sv = [t(r, "End_Timestamp") - t(r, "Start_Timestamp") for r in sv[skip:]]
per = (t(st[-1], "Start_Timestamp") - t(st[skip], "Start_Timestamp")) / max(1, len(st) - 1 - skip)
print(f"median stream {S.median(d_st):.1f} us, median solve {S.median(d_sv):.1f} us, period {per:.1f} us")
