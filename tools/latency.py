"""Per-call latency of ce_gpu_nnet_propagate on TDNN-S (one stream, calls back
to back, HIP events), default (throughput) mode vs latency mode
(ce_gpu_ctx_set_latency): the streaming AcousticModel chunk (chunk_size 50 +
20 context rows), a 250-frame chunk, one 10 s utterance (1018 rows) and the
bench's 4072-row batch.   python tools/latency.py [calls]
(LAT_MODES=latency LAT_ROWS=70 restrict the modes and row counts)"""
import hashlib
import json
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from catears_amd import gpu, synth  # noqa: E402


def main(calls=200):
    mdir = os.path.join(tempfile.gettempdir(), f"catears_bench_{os.getuid()}")
    conf = synth.write_model(mdir, "tdnn-s")
    res = {}
    modes = os.environ.get("LAT_MODES", "throughput,latency").split(",")
    sizes = [int(v) for v in os.environ.get("LAT_ROWS", "70,270,1018,4072").split(",")]
    for mode in modes:
        ctx = gpu.Context(0)
        ctx.set_latency(mode == "latency")
        model = gpu.Model(ctx, conf)
        for rows in sizes:
            x = torch.from_numpy(np.random.default_rng(rows).normal(0, 3, size=(rows, 40)).astype(np.float32)).cuda()
            out = gpu.nnet_propagate(ctx, model, x)
            for _ in range(20):
                gpu.nnet_propagate(ctx, model, x, out=out)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(calls):
                gpu.nnet_propagate(ctx, model, x, out=out)
            b.record()
            torch.cuda.synchronize()
            us = a.elapsed_time(b) * 1e3 / calls
            frames = rows - model.left - model.right
            digest = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
            res[f"{mode}/{rows}"] = {"us_per_call": round(us, 1), "frames_per_s": round(frames / us * 1e6),
                                     "sha1": digest}
            print(f"{mode:10s} rows {rows:5d}: {us:8.1f} us/call  {frames / us * 1e6 / 1e6:7.3f} M frames/s"
                  f"  out {digest}", flush=True)
    if os.environ.get("LAT_GRAPH"):
        # the same calls captured once in a HIP graph (fixed input / output
        # buffers) and replayed: the launch cost of a serving loop that stages
        # each chunk into the captured input
        for mode in modes:
            s = torch.cuda.Stream()
            ctx = gpu.Context(0, s)
            ctx.set_latency(mode == "latency")
            model = gpu.Model(ctx, conf)
            for rows in sizes:
                x = torch.from_numpy(np.random.default_rng(rows).normal(0, 3, size=(rows, 40))
                                     .astype(np.float32)).cuda()
                with torch.cuda.stream(s):
                    out = gpu.nnet_propagate(ctx, model, x)
                    for _ in range(3):
                        gpu.nnet_propagate(ctx, model, x, out=out)
                s.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    gpu.nnet_propagate(ctx, model, x, out=out)
                for _ in range(20):
                    g.replay()
                torch.cuda.synchronize()
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(calls):
                    g.replay()
                b.record()
                torch.cuda.synchronize()
                us = a.elapsed_time(b) * 1e3 / calls
                frames = rows - model.left - model.right
                digest = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
                res[f"graph-{mode}/{rows}"] = {"us_per_call": round(us, 1), "frames_per_s": round(frames / us * 1e6),
                                               "sha1": digest}
                print(f"graph {mode:10s} rows {rows:5d}: {us:8.1f} us/call  {frames / us * 1e6 / 1e6:7.3f} M frames/s"
                      f"  out {digest}", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200)
