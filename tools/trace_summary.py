"""Summarise a rocprofv3 kernel trace (csv) per kernel and grid size.

Per kernel: launches, median / min / mean duration, and the wall time during
which at least one launch of it was running (union of [start, end]) divided
by the launch count -- the figure bench.py reports as
roofline.effective_ms_per_launch when launches overlap across streams.
"""
import csv
import sys
from collections import defaultdict


def union_us(iv):
    total, a0, b0 = 0.0, None, None
    for a, b in sorted(iv):
        if b0 is None or a > b0:
            if b0 is not None:
                total += b0 - a0
            a0, b0 = a, b
        else:
            b0 = max(b0, b)
    if b0 is not None:
        total += b0 - a0
    return total


def main(path, title=""):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        if "catears" not in name:
            continue
        name = name.split("(")[0].replace("catears::", "").replace("void ", "")
        blocks = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        d[(name, blocks)].append((int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3))
    by_name = defaultdict(list)
    for (name, _), iv in d.items():
        by_name[name] += iv
    if title:
        print(title)
    print(f"{'kernel':88s} {'blocks':>7s} {'n':>5s} {'median_us':>10s} {'min_us':>8s} {'mean_us':>8s}")
    for k, iv in sorted(d.items(), key=lambda kv: -sum(b - a for a, b in kv[1])):
        v = sorted(b - a for a, b in iv)
        print(f"{k[0][:88]:88s} {k[1]:7d} {len(v):5d} {v[len(v)//2]:10.1f} {v[0]:8.1f} {sum(v)/len(v):8.1f}")
    print()
    print(f"{'kernel (all grids)':88s} {'n':>5s} {'mean_us':>8s} {'union_us/launch':>16s}")
    for k, iv in sorted(by_name.items(), key=lambda kv: -sum(b - a for a, b in kv[1])):
        n = len(iv)
        print(f"{k[:88]:88s} {n:5d} {sum(b - a for a, b in iv)/n:8.1f} {union_us(iv)/n:16.1f}")
    # one kernel template, every instantiation (e.g. a GEMM's hidden-layer
    # and last-layer forms): bench.py's roofline unions over all of them
    by_tmpl = defaultdict(list)
    for name, iv in by_name.items():
        by_tmpl[name.split("<")[0]] += iv
    print()
    print(f"{'kernel template (all instantiations)':88s} {'n':>5s} {'mean_us':>8s} {'union_us/launch':>16s}")
    for k, iv in sorted(by_tmpl.items(), key=lambda kv: -sum(b - a for a, b in kv[1])):
        n = len(iv)
        print(f"{k[:88]:88s} {n:5d} {sum(b - a for a, b in iv)/n:8.1f} {union_us(iv)/n:16.1f}")


if __name__ == "__main__":
    main(sys.argv[1], " ".join(sys.argv[2:]))
