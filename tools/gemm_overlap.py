"""How fully a pipelined bench run keeps the chip in GEMMs, from a rocprofv3
kernel trace (tools/trace_short.sh).  Over the busiest GPU work segment
(timeline.py's rule), sweeps the GEMM launches' start / end events and
reports the share of the time with 0, 1 or >= 2 GEMM launches running and
the time-averaged CU demand min(1, sum of running GEMM workgroups / 256)
(each bf16x6 block holds a whole CU's LDS, so one block per CU).
    python tools/gemm_overlap.py <kernel_trace.csv>"""
import collections
import csv
import sys

from timeline import GAP, short  # same segment rule and kernel names

CUS = 256


def main(path):
    rows = []
    for r in csv.DictReader(open(path)):
        a, b = int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        rows.append((a, b, short(r["Kernel_Name"]), wg))
    rows.sort()
    segs, cur, end = [], [], None
    for row in rows:
        if end is not None and row[0] - end > GAP:
            segs.append(cur)
            cur = []
        cur.append(row)
        end = row[1] if end is None else max(end, row[1])
    segs.append(cur)
    seg = max(segs, key=lambda s: sum(1 for r in s if r[2].startswith("gemm")))
    t0, t1 = seg[0][0], max(r[1] for r in seg)
    ev = []
    for a, b, name, wg in seg:
        if name.startswith("gemm"):
            ev.append((a, 1, wg))
            ev.append((b, -1, wg))
    ev.sort()
    state = collections.Counter()
    n, wgs, last, demand = 0, 0, t0, 0.0
    for t, d, wg in ev:
        dt = t - last
        state[min(n, 2)] += dt
        if n == 1:
            state["1_full" if wgs >= CUS else "1_part"] += dt
        demand += dt * min(1.0, wgs / CUS)
        n += d
        wgs += d * wg
        last = t
    state[0] += t1 - last
    span = t1 - t0
    by = collections.defaultdict(list)
    for a, b, name, wg in seg:
        if name.startswith("gemm"):
            by[wg].append(b - a)
    print(f"segment {span:.1f} us, {sum(1 for r in seg if r[2].startswith('gemm'))} GEMM launches")
    print(f"time share: no GEMM {state[0] / span:.3f}, one GEMM {state[1] / span:.3f} "
          f"(< {CUS} blocks {state['1_part'] / span:.3f}), two or more {state[2] / span:.3f}")
    print(f"time-averaged GEMM CU demand {demand / span:.3f}")
    for wg in sorted(by):
        v = sorted(by[wg])
        print(f"  {wg:5d} blocks: {len(v):5d} launches, median {v[len(v) // 2]:7.1f} us, "
              f"min {v[0]:7.1f}, sum {sum(v):9.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
