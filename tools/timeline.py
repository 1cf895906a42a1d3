"""Coarse timeline of the timed region of a bench run from a rocprofv3
kernel trace: the GPU work segment (between idle gaps > GAP us) holding the
most GEMM launches.  Prints per-bin concurrency (GEMM launches running,
their workgroups) and the per-stream kernel sequence at the start and end.
    python tools/timeline.py <kernel_trace.csv> [bin_us]"""
import csv
import sys

GAP = 40.0


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("catears::", "")
    for k in ("gemm_bf16x6", "gemm_f32", "gemm_f16x3", "fbank", "cmvn", "finalize", "splice", "gemm_i8"):
        if k in n:
            return k
    return n.split("(")[0][:24]


def main(path, bin_us=50.0):
    rows = []
    for r in csv.DictReader(open(path)):
        a, b = int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        rows.append((a, b, short(r["Kernel_Name"]), int(r.get("Queue_Id", 0)), wg))
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
    t0 = seg[0][0]
    t1 = max(r[1] for r in seg)
    print(f"segment: {len(seg)} kernels, {t1 - t0:.1f} us, "
          f"{sum(1 for r in seg if r[2] == 'fbank')} fbank launches")
    nb = int((t1 - t0) / bin_us) + 1
    for i in range(nb):
        lo, hi = t0 + i * bin_us, t0 + (i + 1) * bin_us
        act = [r for r in seg if r[0] < hi and r[1] > lo]
        g = [r for r in act if r[2].startswith("gemm")]
        busy = sum(min(r[1], hi) - max(r[0], lo) for r in g) / bin_us
        wgs = sum(r[4] for r in g)
        other = sorted(set(r[2] for r in act if not r[2].startswith("gemm")))
        print(f"{i * bin_us:7.0f} gemm x{busy:4.2f} wg {wgs:4d}  {' '.join(other)}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 50.0)
