#!/usr/bin/env python3
"""MFMA utilisation per GEMM launch from a rocprofv3 --pmc pass with
SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (bench.py --serial, so each
dispatch runs alone).

usage: pmc_mfma.py <pmc_dir> <out.json>

SQ_VALU_MFMA_BUSY_CYCLES is summed over every SIMD of the chip and counts
the matrix pipe's busy cycles (16 per v_mfma_f32_16x16x32_bf16, 32 per
v_mfma_i32_32x32x32_i8); GRBM_GUI_ACTIVE is summed over the 8 XCDs, so
GUI / 8 is the dispatch's length in cycles (MI355X_MICROARCH.md, DVFS
give-back note).  Per kernel:
  chip   = MFMA busy / (cycles x 1024 SIMDs)        -- the whole chip
  active = MFMA busy / (cycles x 4 x CUs with a block) -- the CUs the grid
           occupies (these kernels run one block per CU), idle tail waves
           included
both weighted over the kernel's dispatches by cycles.
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

SIMDS, CUS = 1024, 256


def main():
    src, out = sys.argv[1:3]
    disp = defaultdict(dict)
    for f in glob.glob(f"{src}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            name = re.sub(r"\(anonymous namespace\)::", "", row["Kernel_Name"])
            name = name.split("(")[0] if not name.startswith("void ") else name[5:].split("(")[0]
            d = disp[(f, row["Dispatch_Id"])]
            d["name"] = name
            d["blocks"] = int(row["Grid_Size"]) // max(1, int(row["Workgroup_Size"]))
            d[row["Counter_Name"]] = float(row["Counter_Value"])
    acc = defaultdict(lambda: {"busy": 0.0, "chip": 0.0, "active": 0.0, "n": 0})
    for d in disp.values():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in d or "GRBM_GUI_ACTIVE" not in d:
            continue
        cyc = d["GRBM_GUI_ACTIVE"] / 8
        a = acc[d["name"]]
        a["busy"] += d["SQ_VALU_MFMA_BUSY_CYCLES"]
        a["chip"] += cyc * SIMDS
        a["active"] += cyc * 4 * min(d["blocks"], CUS)
        a["n"] += 1
    res = {k: {"dispatches": v["n"], "mfma_util_chip": round(v["busy"] / v["chip"], 4),
               "mfma_util_active_cus": round(v["busy"] / v["active"], 4)}
           for k, v in sorted(acc.items()) if v["n"]}
    json.dump({"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE, bench.py --serial",
               "definition": "MFMA busy cycles / (GRBM_GUI_ACTIVE/8 cycles x SIMDs): chip = 1024 SIMDs, "
                             "active_cus = 4 SIMDs x min(blocks, 256)", "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"  mfma util chip {v['mfma_util_chip']:.3f} active {v['mfma_util_active_cus']:.3f}  {v['dispatches']:4d}  {k}")


if __name__ == "__main__":
    main()
