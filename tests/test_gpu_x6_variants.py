"""The alternative bf16x6 GEMM schedules give the default's bits.  They are
selected by the experiments library's CATEARS_* switches (read once per
process: one child process each, on libcatears_hip_exp.so -- the product
library compiles the defaults in and reads no environment).  Every variant accumulates each output element over the same
K-tiles in the same order with the same six products per tile,
so the tile shape (128 x 128, variant 40; 256 x 128, the rounds 3-5 default
300; the product's 512 x 128 of 8 waves), the warp-specialised producer /
MFMA-wave split (200) and the one-wave-per-SIMD forms (500-507) must not
change any bit of TDNN-S's output.  A value
the product build does not carry (measurement variants, the DIAG ablations)
fails loudly with CE_GPU_EINVAL instead of running something else.  The
product library's own choices (wide tiles) run in-process on it."""
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

CHILD = r"""
import sys, numpy as np, torch
from catears_amd import gpu
ctx = gpu.Context(0)
if len(sys.argv) > 3 and sys.argv[3] == "wide":
    ctx.set_wide_tiles(True)
model = gpu.Model(ctx, sys.argv[1])
assert model.gemm == "bf16x6", model.gemm
x = np.random.default_rng(750).normal(9.0, 3.0, size=(3000, 40)).astype(np.float32)
out = gpu.nnet_propagate(ctx, model, torch.from_numpy(x).to("cuda:0")).cpu().numpy()
np.save(sys.argv[2], out)
"""


def _child(variant, cfg, path, *args, lib=None, **extra_env):
    env = dict(os.environ, CATEARS_X6_VARIANT=str(variant), PYTHONPATH=ROOT, **extra_env)
    env.pop("CATEARS_HIP_LIB", None)
    if lib:
        env["CATEARS_HIP_LIB"] = lib
    return subprocess.run([sys.executable, "-c", CHILD, cfg, str(path), *args], env=env, capture_output=True,
                          text=True, timeout=300, cwd=ROOT)


def _run(variant, cfg, path, *args, lib=None, **extra_env):
    r = _child(variant, cfg, path, *args, lib=lib, **extra_env)
    assert r.returncode == 0, r.stderr[-3000:]
    return np.load(path).view(np.uint32)


def test_x6_variants_bit_identical(tmp_path, s_config, exp_lib):
    base = _run(0, s_config, tmp_path / "v0.npy")  # the product library
    assert np.array_equal(_run(0, s_config, tmp_path / "e0.npy", lib=exp_lib), base), \
        "the experiments library's default differs from the product library"
    assert base.ndim == 2 and base.shape[0] > 0
    # 300: the rounds 3-5 default (256 x 128 tiles of gemm_bf16x6d_kernel);
    # 500-507: the one-wave-per-SIMD forms of gemm_bf16x6w_kernel
    for v in (40, 200, 300, 500, 501, 502, 503, 505, 507):
        got = _run(v, s_config, tmp_path / f"v{v}.npy", lib=exp_lib)
        assert np.array_equal(got, base), f"variant {v} differs from the default"
    # the first layer's splice + row gather in the default kernel's loader
    # against the round-3 splice_pad launch before it (CATEARS_X6_FIRST=0)
    padded = _run(0, s_config, tmp_path / "pad.npy", CATEARS_X6_FIRST="0", lib=exp_lib)
    assert np.array_equal(padded, base), "the gathered first layer differs from splice_pad"
    # the gathered first layer on the hidden layers' 256 x 128 tiles
    wide = _run(0, s_config, tmp_path / "t256.npy", CATEARS_X6_FIRST_TILE="256", lib=exp_lib)
    assert np.array_equal(wide, base), "the first layer's 256-unit tiles differ"
    # two K-tiles per LDS stage against one (the default)
    ks2 = _run(0, s_config, tmp_path / "ks2.npy", CATEARS_X6_KS="2", lib=exp_lib)
    assert np.array_equal(ks2, base), "two K-tiles per LDS stage differ from one"
    # the plane chain: every layer's output split once, in its epilogue, and
    # read as planes by the next (CATEARS_X6_CHAIN=1), on both first-layer
    # tile widths
    chain = _run(0, s_config, tmp_path / "chain.npy", CATEARS_X6_CHAIN="1", lib=exp_lib)
    assert np.array_equal(chain, base), "the plane chain differs from the fp32 chain"
    chain256 = _run(0, s_config, tmp_path / "chain256.npy", CATEARS_X6_CHAIN="1", CATEARS_X6_FIRST_TILE="256", lib=exp_lib)
    assert np.array_equal(chain256, base), "the plane chain on 256-unit first-layer tiles differs"
    # planes into the output layer only (CATEARS_X6_CHAIN=2)
    last = _run(0, s_config, tmp_path / "chain2.npy", CATEARS_X6_CHAIN="2", lib=exp_lib)
    assert np.array_equal(last, base), "planes into the output layer only differ"
    # every layer on 128 x 128 tiles (ce_gpu_ctx_set_wide_tiles)
    wide = _run(0, s_config, tmp_path / "wide.npy", "wide")
    assert np.array_equal(wide, base), "128 x 128 tiles (wide) differ from the default tiles"


def test_x6_plane_chain_xs(tmp_path, xs_config, exp_lib):
    """The plane chain on TDNN-XS (256-wide hidden layers, 512 pdfs: one
    unit tile per layer, a partial last tile of the output layer)."""
    base = _run(0, xs_config, tmp_path / "v0.npy")
    chain = _run(0, xs_config, tmp_path / "chain.npy", CATEARS_X6_CHAIN="1", lib=exp_lib)
    assert np.array_equal(chain, base), "the plane chain differs from the fp32 chain on TDNN-XS"


def test_unknown_variant_fails_loudly(tmp_path, s_config, exp_lib):
    for v in (7, 12345):
        r = _child(v, s_config, tmp_path / f"bad{v}.npy", lib=exp_lib)
        assert r.returncode != 0
        assert "EINVAL" in r.stderr and f"schedule {v}" in r.stderr, r.stderr[-2000:]


def test_product_library_ignores_the_switches(tmp_path, s_config):
    """The product library reads no CATEARS_* switch: a schedule number that
    the experiments library would reject runs the default here."""
    base = _run(0, s_config, tmp_path / "v0.npy")
    assert np.array_equal(_run(12345, s_config, tmp_path / "v12345.npy", CATEARS_X6_CHAIN="1"), base)
