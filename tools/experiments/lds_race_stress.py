"""Stress for the intra-wave LDS hand-off.

One front stream runs the fbank kernel over the C3 batch (4 x 10 s) again and
again while `--gemm-streams` streams run TDNN-S forwards of a fixed batch
beside it -- the bench pipeline's co-residency, with far more fbank launches
per second.  Every fbank output is compared bit for bit with the output of the
same launch made alone before the stress (on the front stream, no host sync):
per iteration the number of differing rows, and per (row, band) how often it
differed.  Prints one JSON line: iterations, differing iterations and rows,
the rows' residues (row % 4 = the 16-lane group of fbank_fast_kernel, row % 8
= the 8-lane group of fbank_kernel) and the first differing rows with their
bands and values.

  CATEARS_HIP_LIB=<lib> python tools/experiments/lds_race_stress.py --fbank fast --seconds 20
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from catears_amd import gpu, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fbank", default="fast", choices=["fast", "exact"])
    ap.add_argument("--pcm", default="f32", choices=["f32", "s16"])
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--utts", type=int, default=4)
    ap.add_argument("--gemm-streams", type=int, default=3)
    ap.add_argument("--fbank-per-gemm", type=int, default=8, help="fbank launches per enqueued forward")
    a = ap.parse_args()

    mdir = os.path.join(tempfile.gettempdir(), f"catears_bench_{os.getuid()}")
    conf = synth.write_model(mdir, "tdnn-s")
    backs = [torch.cuda.Stream() for _ in range(a.gemm_streams)]
    front = torch.cuda.Stream()
    ctxs = [gpu.Context(0, s) for s in backs]
    cf = gpu.Context(0, front)
    cf.set_fbank(a.fbank)
    model = gpu.Model(ctxs[0], conf)
    n = 160000
    plan = gpu.Plan(cf, [n] * a.utts, model)
    T = plan.total_frames
    pcm_np = np.stack([synth.pcm(i, n) for i in range(a.utts)]).reshape(-1)
    pcm = torch.from_numpy(pcm_np.astype(np.int16) if a.pcm == "s16" else pcm_np).cuda()
    gstats = torch.from_numpy(synth.cmvn_stats_synthetic()).cuda()

    gold = torch.empty((T, 40), dtype=torch.float32, device="cuda")
    gpu.fbank(cf, plan, pcm, gold)
    norm = torch.empty_like(gold)
    gpu.cmvn(cf, plan, gstats, gold, norm)
    torch.cuda.synchronize()
    gi = gold.view(torch.int32)
    RING = 256
    outs = [torch.empty_like(gold) for _ in range(RING)]
    captured = []  # (iteration, host copy) of the first differing outputs
    gouts = [torch.empty((T, model.num_pdfs), dtype=torch.float32, device="cuda") for _ in backs]
    hits = torch.zeros((T, 40), dtype=torch.int32, device="cuda")
    nbad = []  # per iteration: differing rows (device scalars)
    t0 = time.perf_counter()
    it = 0
    k = 0
    while time.perf_counter() - t0 < a.seconds:
        b = k % len(backs)
        gpu.am_forward(ctxs[b], model, plan, norm, gouts[b])
        k += 1
        with torch.cuda.stream(front):
            for _ in range(a.fbank_per_gemm):
                o = outs[it % len(outs)]
                gpu.fbank(cf, plan, pcm, o)
                d = o.view(torch.int32) != gi
                hits += d.int()
                nbad.append(d.any(1).sum())
                it += 1
        if k % 32 == 0:
            torch.cuda.synchronize()  # bounds the queue (32 x fbank-per-gemm <= RING launches)
            if len(captured) < 3:
                lo = max(0, it - min(RING, 32 * a.fbank_per_gemm))
                win = torch.stack(nbad[lo:it]).cpu().numpy()
                for q in np.nonzero(win)[0][:3 - len(captured)]:
                    captured.append((lo + int(q), outs[(lo + int(q)) % RING].cpu().numpy()))
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    nb = torch.stack(nbad).cpu().numpy()
    h = hits.cpu().numpy()
    rows = np.nonzero(h.any(1))[0]
    res = {
        "lib": os.environ.get("CATEARS_HIP_LIB", "default"),
        "fbank": a.fbank, "pcm": a.pcm, "frames_per_launch": T, "gemm_streams": a.gemm_streams,
        "iterations": int(it), "gemm_launches": int(k), "seconds": round(elapsed, 2),
        "differing_iterations": int((nb > 0).sum()), "differing_rows_total": int(nb.sum()),
        "rows_ever_differing": int(rows.size),
        "row_mod4": np.bincount(rows % 4, minlength=4).tolist() if rows.size else [0] * 4,
        "row_mod8": np.bincount(rows % 8, minlength=8).tolist() if rows.size else [0] * 8,
        "first_rows": [{"row": int(r), "block16": int(r // 16), "hits": int(h[r].max()),
                        "bands": np.nonzero(h[r])[0].tolist()} for r in rows[:12]],
    }
    g = gold.cpu().numpy()
    cap = []
    for itn, o in captured:
        bad = np.nonzero((o.view(np.int32) != g.view(np.int32)).any(1))[0]
        rows_info = []
        for r in bad[:6]:
            d = np.abs(o[r].astype(np.float64) - g[r])
            same = np.nonzero((g.view(np.int32) == o[r].view(np.int32)[None, :]).all(1))[0]
            rows_info.append({"row": int(r), "max_abs": float(d.max()), "mean_abs": float(d.mean()),
                              "bands": int((d > 0).sum()), "equals_gold_row": same[:4].tolist(),
                              "finite": bool(np.isfinite(o[r]).all()),
                              "out": [round(float(x), 4) for x in o[r][:6]],
                              "gold": [round(float(x), 4) for x in g[r][:6]]})
        cap.append({"iteration": itn, "rows": int(bad.size), "row_mod4": np.bincount(bad % 4, minlength=4).tolist(),
                    "first": rows_info})
    res["captured"] = cap
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
