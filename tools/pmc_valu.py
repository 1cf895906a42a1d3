#!/usr/bin/env python3
"""Measured VALU occupancy of a kernel from one rocprofv3 --pmc pass with
  SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY
  SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE
(7 SQ + 1 GRBM counters: one pass; bench.py --workload c2, tools/round_gpu.sh).

usage: pmc_valu.py <out.json> <pmc_dir>...

Units (counter_defs.yaml, MI355X_MICROARCH.md): SQ_ACTIVE_INST_*, SQ_WAIT_*,
SQ_WAVE_CYCLES and SQ_BUSY_CU_CYCLES count quad-cycles (4 shader cycles),
summed over waves / CUs; GRBM_GUI_ACTIVE counts cycles summed over the 8
XCDs.  Per kernel, over its dispatches:

  valu_active_per_simd = SQ_ACTIVE_INST_VALU / SQ_BUSY_CU_CYCLES
      the cycles in which a wave of the SIMD was executing VALU work, per
      busy cycle of the SIMD (the VERDICT r5 ratio).  SQ_BUSY_CU_CYCLES is
      summed over a CU's 4 SIMDs in quad-cycles, i.e. it counts the CU's busy
      cycles (cu_busy below reads 0.92 on the C2 launch, not 3.7).  Above 1
      means the VALU work of several waves of one SIMD overlaps in time: it is
      per-wave occupancy, not the pipe's
  valu_busy_amd = SQ_ACTIVE_INST_VALU / (CUs x GRBM_GUI_ACTIVE / 8)
      AMD's own derived `VALUBusy` (counter_defs.yaml), the same quotient
      over the dispatch's cycles instead of the CUs' busy cycles
  valu_issue_2cyc = SQ_INSTS_VALU x 2 / (SIMDs x GRBM_GUI_ACTIVE / 8)
      the instructions against the VALU pipe's rate with two or more waves
      per SIMD: one wave64 v_fma_f32 per 2 cycles (MI355X_MICROARCH.md,
      per-instruction constants; one wave alone: 4) -- the pipe's occupancy
      if every instruction were a 2-cycle one (f64 and transcendental ones
      take longer, so this is a lower bound)
  wave state: SQ_ACTIVE_INST_ANY, SQ_WAIT_INST_ANY (issue stalls: dependency
      or pipe busy), SQ_WAIT_ANY (parked at s_waitcnt / barrier) as fractions
      of SQ_WAVE_CYCLES (the three are disjoint, MI355X_MICROARCH.md PMC
      slots); the remainder is the wave waiting for its turn to issue.
"""
import csv
import glob
import json
import re
import sys
from collections import defaultdict

SIMDS, CUS = 1024, 256
NEED = ("SQ_ACTIVE_INST_VALU", "SQ_BUSY_CU_CYCLES", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY",
        "SQ_WAIT_INST_ANY", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE")


def main():
    out, srcs = sys.argv[1], sys.argv[2:]
    disp = defaultdict(dict)
    for f in [f for src in srcs for f in glob.glob(f"{src}/**/*counter_collection.csv", recursive=True)]:
        for row in csv.DictReader(open(f)):
            name = re.sub(r"\(anonymous namespace\)::", "", row["Kernel_Name"])
            name = name.split("(")[0] if not name.startswith("void ") else name[5:].split("(")[0]
            d = disp[(f, row["Dispatch_Id"])]
            d["name"] = name
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    acc = defaultdict(lambda: defaultdict(float))
    for d in disp.values():
        if not all(k in d for k in NEED):
            continue
        a = acc[d["name"]]
        for k in NEED:
            a[k] += d[k]
        a["n"] += 1
    res = {}
    for k, a in sorted(acc.items()):
        cyc = a["GRBM_GUI_ACTIVE"] / 8
        wc = a["SQ_WAVE_CYCLES"]
        res[k] = {
            "dispatches": int(a["n"]),
            "valu_active_per_simd": round(a["SQ_ACTIVE_INST_VALU"] / a["SQ_BUSY_CU_CYCLES"], 4),
            "valu_busy_amd": round(a["SQ_ACTIVE_INST_VALU"] / (CUS * cyc), 4),
            "valu_issue_2cyc": round(a["SQ_INSTS_VALU"] * 2 / (SIMDS * cyc), 4),
            "cu_busy": round(a["SQ_BUSY_CU_CYCLES"] / (CUS * cyc), 4),
            "wave_active": round(a["SQ_ACTIVE_INST_ANY"] / wc, 4),
            "wave_issue_stall": round(a["SQ_WAIT_INST_ANY"] / wc, 4),
            "wave_parked": round(a["SQ_WAIT_ANY"] / wc, 4),
            "valu_insts_per_dispatch": round(a["SQ_INSTS_VALU"] / a["n"]),
            "cycles_per_dispatch": round(cyc / a["n"]),
        }
    json.dump({"source": "rocprofv3 --pmc " + " ".join(NEED), "definition": __doc__.split("usage")[0].strip()
               + " -- see tools/pmc_valu.py", "kernels": res}, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"  {k}: " + ", ".join(f"{kk} {vv}" for kk, vv in v.items()))


if __name__ == "__main__":
    main()
