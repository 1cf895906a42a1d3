#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

usage: pmc_traffic.py <fetch_dir> <write_dir> <out.json> [--layers N]

--layers N: also the GEMM launches per position in a step of N GEMM layers
(every gemm_* dispatch in dispatch order, position = index mod N; the
serial bench runs the layers of each batch in order), for the per-layer
traffic bench.py reports beside the algorithmic bytes.

Per kernel instance: mean FETCH_SIZE and WRITE_SIZE per dispatch (rocprofv3
reports KB = 1024 B) and the corrected HBM bytes per launch,
2 * FETCH + WRITE: on gfx950 FETCH_SIZE counts half the bytes of wide
coalesced streaming reads (MI355X_MICROARCH.md, HBM section), WRITE_SIZE is
exact for 16-B-per-lane stores.
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict


def per_kernel(d, counter):
    acc = defaultdict(list)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            name = re.sub(r"\(anonymous namespace\)::", "", row["Kernel_Name"])
            name = name.split("(")[0] if not name.startswith("void ") else name[5:].split("(")[0]
            acc[name].append(float(row["Counter_Value"]))
    return acc


def gemm_sequence(d, counter):
    """[(kernel, value)] of the gemm_* dispatches in dispatch order."""
    rows = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter or "gemm_" not in row["Kernel_Name"]:
                continue
            name = re.sub(r"\(anonymous namespace\)::", "", row["Kernel_Name"])
            name = name.split("(")[0] if not name.startswith("void ") else name[5:].split("(")[0]
            rows.append((int(row["Dispatch_Id"]), name, float(row["Counter_Value"])))
    return [(n, v) for _, n, v in sorted(rows)]


def per_layer(fetch, write, n_layers):
    fs, ws = gemm_sequence(fetch, "FETCH_SIZE"), gemm_sequence(write, "WRITE_SIZE")
    # each pass is its own run (the time-based pre-warm gives them different
    # step counts): positions are counted within each pass
    if not fs or not ws or len(fs) % n_layers or len(ws) % n_layers:
        return None
    out = []
    for pos in range(n_layers):
        f = [v for i, (_, v) in enumerate(fs) if i % n_layers == pos]
        w = [v for i, (_, v) in enumerate(ws) if i % n_layers == pos]
        out.append({"layer": pos + 1, "kernel": fs[pos][0], "dispatches": len(f),
                    "hbm_bytes_per_launch": round((2 * sum(f) / len(f) + sum(w) / len(w)) * 1024)})
    return out


def main():
    fetch, write, out = sys.argv[1:4]
    n_layers = int(sys.argv[sys.argv.index("--layers") + 1]) if "--layers" in sys.argv else 0
    fk, wk = per_kernel(fetch, "FETCH_SIZE"), per_kernel(write, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fk) | set(wk)):
        f = sum(fk.get(k, [0])) / max(len(fk.get(k, [])), 1)
        w = sum(wk.get(k, [0])) / max(len(wk.get(k, [])), 1)
        res[k] = {"dispatches": len(fk.get(k, [])), "fetch_kb_mean": round(f, 1), "write_kb_mean": round(w, 1),
                  "hbm_bytes_per_launch": round((2 * f + w) * 1024)}
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py --serial",
           "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving)",
           "kernels": res}
    if n_layers:
        layers = per_layer(fetch, write, n_layers)
        if layers:
            doc["gemm_layers"] = layers
            for L in layers:
                print(f"  layer {L['layer']}: {L['hbm_bytes_per_launch'] / 1e6:8.2f} MB/launch  {L['kernel']}")
    json.dump(doc, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{v['hbm_bytes_per_launch'] / 1e6:10.2f} MB/launch  {v['dispatches']:5d}  {k}")


if __name__ == "__main__":
    main()
