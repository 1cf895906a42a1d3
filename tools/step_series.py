"""Per-batch completion intervals over a bench run from a rocprofv3 kernel
trace (each batch ends with one finalize launch): shows how the step time
settles after the start.   python tools/step_series.py <kernel_trace.csv> [group]"""
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3, r["Kernel_Name"])
              for r in csv.DictReader(open(sys.argv[1])))
ends = sorted(b for a, b, n in rows if "finalize" in n)
g = int(sys.argv[2]) if len(sys.argv) > 2 else 6
t0 = ends[0]
for i in range(g, len(ends), g):
    print(f"batches {i - g:3d}-{i:3d}: t={ends[i] - t0:8.0f} us  {(ends[i] - ends[i - g]) / g:6.1f} us/batch")
