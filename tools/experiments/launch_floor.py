"""Kernel-boundary floor on this GPU: back-to-back launches of tiny torch
kernels on one stream, timed with HIP events (run under rocprofv3
--kernel-trace for per-kernel durations).  python launch_floor.py"""
import torch

x = torch.zeros(16, device="cuda")
y = torch.zeros(1 << 20, device="cuda")
for name, t in (("tiny", x), ("1M", y)):
    for _ in range(50):
        t.add_(1.0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(1000):
        t.add_(1.0)
    b.record()
    torch.cuda.synchronize()
    print(f"{name}: {a.elapsed_time(b):.3f} us per launch (1000 launches, ms total = us each)", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(100):
        x.add_(1.0)
g.replay()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    g.replay()
b.record()
torch.cuda.synchronize()
print(f"graph tiny: {a.elapsed_time(b):.3f} us per launch (10 x 100 in graphs)", flush=True)
