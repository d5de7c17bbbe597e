"""Kernel timeline of one tick from a rocprofv3 kernel trace: python tools/tick_timeline.py <dir> <anchor kernel substring> [k]
Prints every kernel between the k-th-from-last and the (k-1)-th-from-last anchor (start offsets in us)."""
import csv
import glob
import sys

d, anchor = sys.argv[1], sys.argv[2]
k = int(sys.argv[3]) if len(sys.argv) > 3 else 3
f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
a, b = idx[-k], idx[-k + 1]
t0 = int(rows[a]["End_Timestamp"])
busy = 0
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:100]}")
print(f"span {(int(rows[b]['End_Timestamp']) - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")
