"""Calibration: the vendor int8 GEMM (torch._int_mm -> hipBLASLt on ROCm) on
the C5 hidden-layer shape (8192 x 3072 x 1024, int8 in, int32 out), and a
bf16 / fp8 GEMM of the same shape where torch offers one, to place the int8
kernel's per-CU efficiency.   python tools/probes/i8_blas_calib.py"""
import torch

M, K, N = 8192, 3072, 1024


def timed(fn, reps=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


a8 = torch.randint(-128, 127, (M, K), device="cuda", dtype=torch.int8)
b8 = torch.randint(-128, 127, (N, K), device="cuda", dtype=torch.int8)
for name, fn in [("int8 _int_mm (A x B^T view)", lambda: torch._int_mm(a8, b8.t())),
                 ("int8 _int_mm (A x B)", lambda: torch._int_mm(a8, b8.t().contiguous()))]:
    try:
        ms = timed(fn)
        print(f"{name}: {ms * 1e3:.1f} us, {2 * M * K * N / ms / 1e9:.0f} TOP/s", flush=True)
    except Exception as e:  # not every layout is supported
        print(f"{name}: unavailable ({type(e).__name__}: {str(e)[:120]})", flush=True)
ab = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
bb = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
ms = timed(lambda: ab @ bb)
print(f"bf16 matmul: {ms * 1e3:.1f} us, {2 * M * K * N / ms / 1e9:.0f} TFLOP/s", flush=True)
try:
    af = ab.to(torch.float8_e4m3fn)
    bf = bb.t().contiguous().to(torch.float8_e4m3fn).t()
    one = torch.ones((), device="cuda")
    ms = timed(lambda: torch._scaled_mm(af, bf, scale_a=one, scale_b=one, out_dtype=torch.bfloat16))
    print(f"fp8 _scaled_mm: {ms * 1e3:.1f} us, {2 * M * K * N / ms / 1e9:.0f} TFLOP/s", flush=True)
except Exception as e:
    print(f"fp8 _scaled_mm: unavailable ({type(e).__name__}: {str(e)[:120]})", flush=True)
