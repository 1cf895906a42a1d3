"""Calibration: hipBLASLt (torch.matmul) bf16 / fp32 on the TDNN-S hidden-layer
shape, to place the bf16x6 kernel's per-CU efficiency against the vendor GEMM.
    python tools/probes/blas_calib.py"""
import torch

M, K, N = 4072, 3072, 1024
for dt in (torch.bfloat16, torch.float32):
    a = torch.randn(M, K, device="cuda", dtype=dt)
    b = torch.randn(K, N, device="cuda", dtype=dt)
    for _ in range(20):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 200
    e0.record()
    for _ in range(reps):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tf = 2 * M * K * N / ms / 1e9
    print(f"{dt}: {ms * 1e3:.1f} us per GEMM, {tf:.0f} TFLOP/s", flush=True)
