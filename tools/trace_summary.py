"""Summarise a rocprofv3 kernel trace (csv) per kernel and grid size.

Per kernel: launches, median / min / mean duration, and the wall time during
which at least one launch of it was running (union of [start, end]) divided
by the launch count -- the figure bench.py reports as
roofline.effective_ms_per_launch when launches overlap across streams.

--window: keep only the launches between bench.py's two window markers
(catears::trace_mark_kernel, 1 workgroup before the timed steps, 2 after
them; ce_gpu_trace_mark), so the summary covers exactly the steps the bench
line timed -- not the pre-warm and warm-up steps before them.

--check BENCH_JSON: recompute the line's roofline from this trace -- the
dominant kernel template's algorithmic work per launch (the line's
flops_per_launch / ops_per_launch) over its union time per launch -- and
compare it with the line's `frac` (and the GEMM time per step with the
line's ms_per_step).

Usage: trace_summary.py TRACE_CSV [--window] [--check BENCH_JSON] [title ...]
"""
import argparse
import csv
import json
from collections import defaultdict

MARK = "trace_mark_kernel"


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


def read_trace(path):
    """[(name, blocks, start_us, end_us)] for the catears kernels."""
    out = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        if "catears" not in name:
            continue
        name = name.split("(")[0].replace("catears::", "").replace("void ", "")
        blocks = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
        out.append((name, blocks, int(r["Start_Timestamp"]) / 1e3, int(r["End_Timestamp"]) / 1e3))
    return out


def window(rows):
    """The launches after the last tag-1 marker and before the tag-2 marker
    that follows it; (rows, window_us)."""
    marks = sorted((a, blocks) for name, blocks, a, _ in rows if name.startswith(MARK))
    starts = [a for a, tag in marks if tag == 1]
    if not starts:
        raise SystemExit("--window: no trace_mark_kernel launch with 1 workgroup in the trace")
    w0 = starts[-1]
    ends = [a for a, tag in marks if tag == 2 and a > w0]
    if not ends:
        raise SystemExit("--window: no closing trace_mark_kernel (2 workgroups) after the opening one")
    w1 = ends[0]
    keep = [r for r in rows if not r[0].startswith(MARK) and r[2] >= w0 and r[3] <= w1]
    return keep, w1 - w0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("title", nargs="*")
    ap.add_argument("--window", action="store_true")
    ap.add_argument("--check")
    args = ap.parse_intermixed_args()
    rows = [r for r in read_trace(args.trace)]
    win_us = None
    if args.window:
        rows, win_us = window(rows)
    else:
        rows = [r for r in rows if not r[0].startswith(MARK)]
    d = defaultdict(list)
    for name, blocks, a, b in rows:
        d[(name, blocks)].append((a, b))
    by_name = defaultdict(list)
    for (name, _), iv in d.items():
        by_name[name] += iv
    if args.title:
        print(" ".join(args.title))
    if win_us is not None:
        print(f"window: the launches between bench.py's trace markers (the timed steps only): "
              f"{win_us / 1e3:.4f} ms, {len(rows)} launches")
        print()
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
    if args.check:
        check(args.check, by_tmpl, win_us)


def check(path, by_tmpl, win_us):
    """The bench line's roofline, recomputed from this trace."""
    line = None
    for s in open(path):
        if s.startswith("{"):
            line = json.loads(s)
    if line is None or not line.get("roofline"):
        raise SystemExit(f"--check: no bench line with a roofline in {path}")
    rf = line["roofline"]
    tmpl = rf["kernel"].split("<")[0].split(" ")[0]
    if tmpl.endswith("*"):  # every template with this prefix (e.g. gemm_bf16x6*: the d and w kernels)
        iv = [x for k, v in by_tmpl.items() if k.startswith(tmpl[:-1]) for x in v]
    else:
        iv = by_tmpl.get(tmpl)
    print()
    print(f"check against {path}:")
    if not iv:
        print(f"  no launches of {tmpl} in the trace")
        return
    n = len(iv)
    u = union_us(iv)
    steps = line["steps"]
    work = rf.get("flops_per_launch") or rf.get("ops_per_launch")
    if work is None and rf.get("algorithmic_bytes_per_launch") and rf.get("unit") == "GB/s":
        work = rf["algorithmic_bytes_per_launch"]
    print(f"  kernel template {tmpl}: {n} launches in the window = {n / steps:g} per step over {steps} steps")
    print(f"  union time {u / 1e3:.4f} ms = {u / n:.2f} us per launch; per step {u / 1e3 / steps:.4f} ms "
          f"vs the line's ms_per_step {line['ms_per_step']:.4f} ({'<=' if u / 1e3 / steps <= line['ms_per_step'] else 'EXCEEDS'})")
    if win_us is not None:
        print(f"  trace window {win_us / 1e3:.4f} ms = {win_us / 1e3 / steps:.4f} ms per step "
              f"(the line's timed region, by the host clock: {line['ms_per_step'] * steps:.4f} ms)")
    if work:
        scale = 1e9 if rf.get("unit") == "GB/s" else 1e12
        achieved = work / (u / n * 1e-6) / scale
        frac = achieved / rf["peak"]
        print(f"  achieved from the trace: {achieved:.2f} {rf['unit']} = frac {frac:.4f} of {rf['peak']} "
              f"(line: achieved {rf['achieved']}, frac {rf['frac']}; ratio {frac / rf['frac']:.4f})")


if __name__ == "__main__":
    main()
