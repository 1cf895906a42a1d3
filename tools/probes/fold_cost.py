"""Cost of rank 0's per-batch fold (RowGather: the float64 sum of a received
4072 x 3456 fp32 log-likelihood batch) on one MI355X: torch.sum with a
float64 accumulator as RowGather had it, other float64 forms, an fp32 sum and
a copy of the same bytes.   python tools/probes/fold_cost.py"""
import torch

x = torch.randn(4072, 3456, device="cuda")
acc = torch.zeros((), dtype=torch.float64, device="cuda")


def timed(fn, reps=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


y = torch.empty_like(x)
ref = torch.sum(x, dtype=torch.float64).item()
import sys, os  # noqa: E401
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from catears_amd import gpu  # noqa: E402
part = torch.empty(gpu.SUM_PARTS, dtype=torch.float64, device="cuda")
acc2 = torch.zeros((), dtype=torch.float64, device="cuda")


def fold_ce():
    acc2.zero_()
    return gpu.sum_f64(x, acc2, part)


forms = [
    ("ce_gpu_sum_f64 (RowGather fold since round 5)", fold_ce),
    ("torch.sum f64 (RowGather fold before)", lambda: torch.sum(x, dtype=torch.float64)),
    ("rows f64 then sum", lambda: x.sum(dim=1, dtype=torch.float64).sum()),
    ("1024-chunks f64 then sum", lambda: x.view(-1, 1024).sum(dim=1, dtype=torch.float64).sum()),
    ("256 slabs f64 then sum", lambda: x.view(256, -1).sum(dim=1, dtype=torch.float64).sum()),
    ("double() then sum", lambda: x.double().sum()),
    ("sum f32", lambda: torch.sum(x)),
    ("copy (read + write)", lambda: y.copy_(x)),
]
for name, fn in forms:
    us = timed(fn)
    v = fn()
    rel = abs(v.item() - ref) / abs(ref) if v.dtype == torch.float64 else float("nan")
    print(f"{name}: {us:.1f} us, {x.numel() * 4 / us / 1e6:.2f} TB/s read, rel vs fold {rel:.2e}", flush=True)
