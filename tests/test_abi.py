"""The C-ABI library (no GPU needed): it loads, exports exactly the entry
points include/catears_gpu.h declares, and its host-only functions behave."""
import ctypes
import os
import re

import pytest

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
    # the int8 GEMM's ablation builds (last template argument DIAG) likewise,
    # and the register-direct bf16x6 schedule (measured slower) is an
    # experiment too
    i8 = re.findall(rb"gemm_i8_glds_kernelILi\d+ELi\d+ELi\d+ELi\d+ELi\d+ELi\d+ELi(\d+)E", data)
    assert i8, "no int8 LDS-DMA GEMM found"
    assert set(i8) == {b"0"}, sorted(set(i8))
    assert b"gemm_i8_pipe_kernel" in data and b"lat_gemm_kernel" in data
    assert b"gemm_bf16x6r_kernel" not in data


def test_product_library_reads_no_environment_switch():
    """The tuning switches of the measurement tools (CE_KNOB, internal.h) are
    read from the environment only by the experiments library; the product
    library compiles their defaults in, so no CATEARS_* name
    -- and no getenv call -- is in it.  Mode choices go through the C-ABI
    (ce_gpu_model_set_gemm, ce_gpu_ctx_set_*).  The drop-in layer's
    CATEARS_DEVICE / CATEARS_LANES / CATEARS_FBANK (host/src/runtime.cc,
    libcatears_pk.so) are its documented configuration, not switches here."""
    data = open(os.path.join(ROOT, "catears_amd", "lib", "libcatears_hip.so"), "rb").read()
    assert re.findall(rb"CATEARS_[A-Z0-9_]+", data) == []
    assert b"getenv" not in data


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


def _code_objects(path):
    """Every gfx950 code object in a HIP shared library: the .hip_fatbin
    section holds one clang offload bundle per translation unit."""
    import struct
    data = open(path, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    objs, at = [], data.find(magic)
    while at >= 0:
        n = struct.unpack_from("<Q", data, at + 24)[0]
        p = at + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "gfx950" in triple:
                objs.append(data[at + off:at + off + size])
        at = data.find(magic, p)
    return objs


def kernel_private_segments(path):
    """{kernel symbol: .private_segment_fixed_size} from the code objects'
    AMDGPU metadata notes (llvm-readelf --notes)."""
    import subprocess
    import tempfile
    readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not os.path.exists(readelf):
        pytest.skip("llvm-readelf not in this image")
    out = {}
    for co in _code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.check_output([readelf, "--notes", f.name], text=True)
        name = None
        for ln in notes.splitlines():
            m = re.match(r"\s+\.name:\s+(\S+)", ln)
            if m:
                name = m.group(1)
            m = re.match(r"\s+\.private_segment_fixed_size:\s+(\d+)", ln)
            if m and name:
                out[name] = int(m.group(1))
    return out


def test_product_kernels_use_no_scratch():
    """No kernel of the product library has a private (scratch) segment.
    The exact fbank kernel once spilled 3 VGPRs to scratch under a forced
    5-waves-per-SIMD budget and, only in the multi-stream pipeline, gave a
    different value for one frame in some runs; every kernel
    on the path now keeps its state in registers and LDS."""
    segs = kernel_private_segments(os.path.join(ROOT, "catears_amd", "lib", "libcatears_hip.so"))
    assert len(segs) >= 20, sorted(segs)
    assert any("fbank_kernel" in k for k in segs)
    scratch = {k: v for k, v in segs.items() if v}
    assert not scratch, scratch


def kernel_instruction_counts(path, pattern):
    """{kernel symbol: count of instructions whose mnemonic matches pattern}
    from llvm-objdump of the library's gfx950 code objects."""
    import collections
    import subprocess
    import tempfile
    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    if not os.path.exists(objdump):
        pytest.skip("llvm-objdump not in this image")
    rx = re.compile(pattern)
    out = collections.Counter()
    n_kernels = 0
    for co in _code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            asm = subprocess.check_output([objdump, "-d", "--mcpu=gfx950", f.name], text=True)
        name = None
        for ln in asm.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:", ln)
            if m:
                name = m.group(1)
                n_kernels += 1
                continue
            m = re.match(r"^\s+([a-z_0-9]+)", ln)
            if m and name and rx.fullmatch(m.group(1)):
                out[name] += 1
    return out, n_kernels


def test_product_kernels_use_no_packed_fp32_valu():
    """No kernel of the product library issues packed-FP32 VALU instructions
    (v_pk_add_f32, v_pk_mul_f32, v_pk_fma_f32, v_pk_mov_b32).  With them, the
    fast fbank kernel's lanes 48-63 computed wrong values in about 2 % of its
    launches while bf16 MFMA GEMMs ran beside it on other streams (round 4's
    GPUTEST failure; tools/experiments/lds_race_stress.py: 2 x 126 k launches
    without a difference once they were gone).  The Makefile
    builds every kernel with the packed-fp32-ops target feature off."""
    counts, n = kernel_instruction_counts(os.path.join(ROOT, "catears_amd", "lib", "libcatears_hip.so"),
                                          r"v_pk_(add|mul|fma)_f32|v_pk_mov_b32")
    assert n >= 20
    assert not counts, dict(counts)
