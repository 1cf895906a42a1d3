"""The C-ABI library (no GPU needed): it loads, exports exactly the entry
points include/catears_gpu.h declares, and its host-only functions behave."""
import ctypes
import os
import re

from conftest import ROOT


def header_symbols():
    text = open(os.path.join(ROOT, "include", "catears_gpu.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ce_gpu_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from catears_amd import gpu
    lib = gpu.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(gpu.ABI) == syms


def test_frame_count_matches_reference_rule(oracle):
    from catears_amd import gpu
    for n in [0, 1, 399, 400, 401, 559, 560, 7802, 160000, 1600000]:
        assert gpu.num_frames(n) == oracle.Fbank.num_frames(n)


def test_version_and_error_string():
    from catears_amd import gpu
    assert b"gfx950" in gpu.lib().ce_gpu_version()
    assert gpu.lib().ce_gpu_last_error() is not None


def test_only_gfx950_code_objects():
    # the library carries gfx950 code only (no CUDA/other-arch fallbacks)
    data = open(os.path.join(ROOT, "catears_amd", "lib", "libcatears_hip.so"), "rb").read()
    assert b"gfx950" in data
    for other in (b"gfx942", b"gfx90a", b"sm_80", b"sm_90"):
        assert other not in data


def test_product_library_has_no_ablation_kernels():
    """The DIAG ablation builds of the bf16x6 GEMM (wrong results, timing
    only) are compiled only into `make EXPERIMENTS=1`'s separate library: no
    gemm_bf16x6f_kernel instantiation in the product library has a non-zero
    DIAG template argument (the third one), and the experiment-only tilings
    are absent too."""
    data = open(os.path.join(ROOT, "catears_amd", "lib", "libcatears_hip.so"), "rb").read()
    inst = re.findall(rb"gemm_bf16x6f_kernelINS0_5X6CfgI(?:Li\d+E)+EELi(\d+)ELi(\d+)E", data)
    assert inst, "no bf16x6 kernel found"
    assert all(diag == b"0" for _, diag in inst), sorted(set(inst))
    # SCHED 6 (variant 55) and the 128 x 256 warp-specialised forms are experiments
    assert not any(sched == b"6" for sched, _ in inst)
    assert b"gemm_bf16x6ws_kernelINS0_5X6CfgILi128ELi256E" not in data
    # the int8 GEMM's and the latency GEMM's ablation builds (last template
    # argument DIAG) likewise
    i8 = re.findall(rb"gemm_i8_glds_kernelILi\d+ELi\d+ELi\d+ELi\d+ELi\d+ELi\d+ELi(\d+)E", data)
    assert i8, "no int8 LDS-DMA GEMM found"
    assert set(i8) == {b"0"}, sorted(set(i8))
    lat = re.findall(rb"lat_gemm_kernelILi\d+ELi\d+ELb[01]ELi(\d+)E", data)
    assert lat, "no latency GEMM found"
    assert set(lat) == {b"0"}, sorted(set(lat))


def test_dropin_library_defines_no_test_hook():
    """The drop-in's failure injection is test-only: libcatears_pk.so holds an
    undefined weak reference to catears_test_inject_failure (null in every
    product binary) and no definition; only the test driver defines it."""
    import subprocess
    pk = os.path.join(ROOT, "catears_amd", "lib", "libcatears_pk.so")
    out = subprocess.run(["nm", "-D", pk], capture_output=True, text=True, check=True).stdout
    hook = [ln.split() for ln in out.splitlines() if ln.endswith(" catears_test_inject_failure")]
    assert hook and all(f[-2] == "w" for f in hook), hook
    assert "InjectDeviceFailures" not in out
