"""Summarise a rocprofv3 kernel trace (csv) per kernel and grid size."""
import csv
import sys
from collections import defaultdict


def main(path, title=""):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        if "catears" not in name:
            continue
        name = name.split("(")[0].replace("catears::", "").replace("void ", "")
        blocks = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        d[(name, blocks)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if title:
        print(title)
    print(f"{'kernel':88s} {'blocks':>7s} {'n':>4s} {'median_us':>10s} {'min_us':>8s} {'mean_us':>8s}")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        v = sorted(v)
        print(f"{k[0][:88]:88s} {k[1]:7d} {len(v):4d} {v[len(v)//2]:10.1f} {v[0]:8.1f} {sum(v)/len(v):8.1f}")


if __name__ == "__main__":
    main(sys.argv[1], " ".join(sys.argv[2:]))
