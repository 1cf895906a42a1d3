"""Print the durations (us) of the last `n` dispatches of kernels whose name
contains `pat`, in launch order, from a rocprofv3 kernel-trace csv, with the
idle gap before each (from the previous dispatch's end)."""
import csv
import sys

path, pat, n = sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 8
rows = [r for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
prev = None
for r in rows[-n:]:
    blocks = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (st - prev) / 1e3 if prev is not None else 0.0
    prev = en
    print(f"  {r['Kernel_Name'].split('(')[0][-60:]:60s} blocks {blocks:6d} {(en - st) / 1e3:9.1f} us  gap {gap:7.1f}")
