"""Latency mode (ce_gpu_ctx_set_latency, kernels/gemm_bf16x6_lat.hip): small
row blocks -- the streaming AcousticModel::Process chunk (src/am.cc:115-142)
or one utterance -- spread over the chip by splitting each layer's K over
64-unit x 80-row blocks (a split chosen from the layer's shape only); the
blocks' partials are summed in split order by a reduce launch, or, for the
last layer, inside the finalize.  Same bars as the default mode:
log-likelihoods within 1e-4 of the oracle, bit-identical across row
segmentations, row groupings and batchings, and deterministic run to run (no
atomics, no inter-block hand-off)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from test_gpu_parity import LOGLIK_TOL, bits, dev

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


@pytest.fixture(scope="module")
def G():
    from catears_amd import gpu
    gpu.lib()
    return gpu


@pytest.fixture(scope="module")
def lctx(torch, G):
    c = G.Context(0)
    c.set_latency(True)
    return c


def test_latency_s_vs_oracle(torch, G, lctx, oracle, s_config):
    from catears_amd import formats, synth
    am = formats.read_am(s_config)
    model = G.Model(lctx, s_config)
    assert model.gemm == "bf16x6"
    fb = oracle.Fbank()
    feats = [fb.compute(synth.pcm(700 + i, n)) for i, n in enumerate([48000, 9000])]
    plan = G.Plan(lctx, [48000, 9000], model)
    out = G.am_forward(lctx, model, plan, dev(torch, np.concatenate(feats))).cpu().numpy()
    off = plan.frame_offsets
    for u, x in enumerate(feats):
        ref = oracle.am_whole(am, x, gemm=lambda a, w: a @ w)
        assert np.abs(out[off[u]:off[u + 1]] - ref).max() <= LOGLIK_TOL
    # the default (throughput) mode differs only by fp32 summation order
    tctx = G.Context(0)
    tmodel = G.Model(tctx, s_config)
    tout = G.am_forward(tctx, tmodel, G.Plan(tctx, [48000, 9000], tmodel), dev(torch, np.concatenate(feats))).cpu().numpy()
    assert np.abs(out - tout).max() <= LOGLIK_TOL / 2


def test_latency_segmentation_and_blocks_exact(torch, G, lctx, oracle, xs_config):
    """Row segmentation (max_rows) and batching of independent blocks
    (propagate_blocks, the multi-stream AcousticModel batcher) change no bit."""
    from catears_amd import synth
    model = G.Model(lctx, xs_config)
    fb = oracle.Fbank()
    feats = [fb.compute(synth.pcm(720 + i, n)) for i, n in enumerate([48000, 16000, 30000])]
    ns = [(len(x) - 1) * 160 + 400 for x in feats]
    x = dev(torch, np.concatenate(feats))
    outs = [G.am_forward(lctx, model, G.Plan(lctx, ns, model, max_rows=r), x).cpu().numpy()
            for r in (4096, 333, 64)]
    assert np.array_equal(bits(outs[0]), bits(outs[1]))
    assert np.array_equal(bits(outs[0]), bits(outs[2]))
    rng = np.random.default_rng(721)
    ctxr = model.left + model.right
    rows = [70, 123, 70, 501]
    blocks = [rng.normal(9.0, 3.0, size=(r, 40)).astype(np.float32) for r in rows]
    together = G.nnet_propagate_blocks(lctx, model, dev(torch, np.concatenate(blocks)), rows).cpu().numpy()
    alone = np.concatenate([G.nnet_propagate(lctx, model, dev(torch, b)).cpu().numpy() for b in blocks])
    assert together.shape == (sum(rows) - len(rows) * ctxr, 512)
    assert np.array_equal(bits(together), bits(alone))


def test_latency_streaming_chunks_deterministic(torch, G, lctx, oracle, s_config):
    """The streaming shape -- 50-frame chunks plus 20 context rows through
    TDNN-S, one call each, 40 calls -- gives identical bits every time (the
    no state carries between calls) and matches the oracle."""
    from catears_amd import formats
    am = formats.read_am(s_config)
    model = G.Model(lctx, s_config)
    rng = np.random.default_rng(730)
    chunk = rng.normal(0.0, 3.0, size=(70, 40)).astype(np.float32)
    d = dev(torch, chunk)
    first = G.nnet_propagate(lctx, model, d).cpu().numpy()
    for _ in range(40):
        again = G.nnet_propagate(lctx, model, d)
    assert np.array_equal(bits(first), bits(again.cpu().numpy()))
    want = oracle.nnet_propagate(am["layers"], chunk, gemm=lambda a, w: a @ w)
    assert np.abs(first - want).max() <= LOGLIK_TOL


def test_latency_long_block_windows(torch, G, lctx, oracle, xs_config):
    """A 5000-row block (thousands of row tiles): the same bits as scoring two
    overlapping halves separately, and the oracle's values in the middle."""
    from catears_amd import formats
    am = formats.read_am(xs_config)
    model = G.Model(lctx, xs_config)
    ctx_rows = model.left + model.right
    rows = 5000
    x = np.random.default_rng(740).normal(9.0, 3.0, size=(rows, 40)).astype(np.float32)
    dx = dev(torch, x)
    got = G.nnet_propagate(lctx, model, dx).cpu().numpy()
    cut = 3000
    a = G.nnet_propagate(lctx, model, dx[:cut + ctx_rows]).cpu().numpy()
    b = G.nnet_propagate(lctx, model, dx[cut:]).cpu().numpy()
    assert np.array_equal(bits(got), bits(np.concatenate([a, b])))
    lo, hi = 2048 - 30, 2048 + 30
    want = oracle.nnet_propagate(am["layers"], x[lo:hi + ctx_rows])
    assert np.abs(got[lo:hi] - want).max() <= LOGLIK_TOL


FUSED_CHILD = r"""
import sys, numpy as np, torch
from catears_amd import gpu
ctx = gpu.Context(0)
ctx.set_latency(True)
model = gpu.Model(ctx, sys.argv[1])
outs = []
for rows, seed in ((70, 760), (1018, 761)):
    x = np.random.default_rng(seed).normal(0.0, 3.0, size=(rows, 40)).astype(np.float32)
    outs.append(gpu.nnet_propagate(ctx, model, torch.from_numpy(x).to("cuda:0"), subtract_prior=True).cpu().numpy())
np.save(sys.argv[2], np.concatenate(outs))
"""


def test_latency_fused_final_reduce_exact(tmp_path, s_config, exp_lib):
    """The last layer's split-K reduce run inside the finalize (the default)
    gives the bits of its own reduce launch followed by the finalize
    (CATEARS_LAT_FUSED_FINAL=0, a switch of the experiments library)."""
    from conftest import ROOT
    got = {}
    for flag in ("1", "0"):
        env = dict(os.environ, CATEARS_LAT_FUSED_FINAL=flag, PYTHONPATH=ROOT, CATEARS_HIP_LIB=exp_lib)
        path = tmp_path / f"f{flag}.npy"
        r = subprocess.run([sys.executable, "-c", FUSED_CHILD, s_config, str(path)], env=env, capture_output=True,
                           text=True, timeout=300, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        got[flag] = np.load(path).view(np.uint32)
    assert got["1"].size > 0
    assert np.array_equal(got["1"], got["0"])


def test_latency_fixup_reduce_exact(tmp_path, s_config, exp_lib):
    """The split-K fix-up (the tile's last slice block does the reduce,
    CATEARS_LAT_FIXUP=1, an experiments-library variant measured slower:
    profiles/r06o_lat_fixup.txt) gives the bits of the reduce launch."""
    from conftest import ROOT
    got = {}
    for flag in ("1", "0"):
        env = dict(os.environ, CATEARS_LAT_FIXUP=flag, PYTHONPATH=ROOT, CATEARS_HIP_LIB=exp_lib)
        path = tmp_path / f"x{flag}.npy"
        r = subprocess.run([sys.executable, "-c", FUSED_CHILD, s_config, str(path)], env=env, capture_output=True,
                           text=True, timeout=300, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        got[flag] = np.load(path).view(np.uint32)
    assert got["1"].size > 0
    assert np.array_equal(got["1"], got["0"])


def test_first_layer_reads_stay_inside_the_input(torch, G, lctx, xs_config):
    """The first layer reads the caller's 40-wide rows directly; its K
    padding (5 x 40 = 200 of 224 / 256) loads column 0 of a valid row, never
    past the row.  The input here ends exactly at the end of a
    2 MiB allocation; both modes give the bits of the same rows scored from
    an ordinary tensor."""
    model = G.Model(lctx, xs_config)
    tctx = G.Context(0)
    tmodel = G.Model(tctx, xs_config)
    rows = 70
    n = 2 * 1024 * 1024 // 4
    buf = torch.empty(n, dtype=torch.float32, device="cuda")
    x = buf[n - rows * 40:].view(rows, 40)
    host = np.random.default_rng(770).normal(0.0, 3.0, size=(rows, 40)).astype(np.float32)
    x.copy_(torch.from_numpy(host))
    for c, m in ((lctx, model), (tctx, tmodel)):
        got = G.nnet_propagate(c, m, x).cpu().numpy()
        want = G.nnet_propagate(c, m, dev(torch, host)).cpu().numpy()
        assert np.array_equal(bits(got), bits(want))


def test_unspliced_first_linear_reads_stay_inside_the_input(torch, G, lctx, oracle):
    """A model whose first component is a Linear on the raw 40-wide rows (no
    Splice): din 40 is not a whole K-tile, so both the throughput and the
    latency kernels must gather it (the throughput kernel picked
    the plain loader for nseg == 1 and read 24 floats past the caller's
    last row).  Input at the very end of a 2 MiB allocation; same bits as
    from an ordinary tensor in both modes, and the oracle's values."""
    from catears_amd import formats, synth
    layers, left, right, prior = synth.tdnn_layers(256, 512, seed=29)
    rng = np.random.default_rng(31)
    first = [{"kind": "linear", "W": (rng.uniform(-1, 1, (40, 40)) * np.sqrt(3.0 / 40)).astype(np.float32),
              "b": (0.1 * rng.uniform(-1, 1, 40)).astype(np.float32)}, {"kind": "relu"}]
    layers = first + layers
    image = formats.nnet_bytes(layers, left, right)
    tctx = G.Context(0)
    rows = 70
    n = 2 * 1024 * 1024 // 4
    buf = torch.empty(n, dtype=torch.float32, device="cuda")
    x = buf[n - rows * 40:].view(rows, 40)
    host = np.random.default_rng(771).normal(0.0, 3.0, size=(rows, 40)).astype(np.float32)
    x.copy_(torch.from_numpy(host))
    ref = oracle.nnet_propagate(layers, host)
    for c in (lctx, tctx):
        m = G.Model(c, image=image, prior=prior)
        got = G.nnet_propagate(c, m, x).cpu().numpy()
        want = G.nnet_propagate(c, m, dev(torch, host)).cpu().numpy()
        assert np.array_equal(bits(got), bits(want))
        assert np.isfinite(got).all()
        assert np.abs(got - ref).max() <= LOGLIK_TOL


POST_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[2])
from test_gpu_latency import post_model_layers
from catears_amd import gpu, formats
layers, left, right, prior = post_model_layers()
ctx = gpu.Context(0)
ctx.set_latency(True)
model = gpu.Model(ctx, image=formats.nnet_bytes(layers, left, right), prior=prior)
x = np.random.default_rng(763).normal(0.0, 3.0, size=(70, 40)).astype(np.float32)
np.save(sys.argv[1], gpu.nnet_propagate(ctx, model, torch.from_numpy(x).to("cuda:0")).cpu().numpy())
"""


def post_model_layers():
    """TDNN-XS with ReLU + BatchNorm after its last Linear (legal NN02): the
    last GEMM carries post ops, so the fused finalize applies them."""
    from catears_amd import synth
    layers, left, right, prior = synth.tdnn_layers(256, 512, seed=21)
    last = layers.pop()
    rng = np.random.default_rng(5)
    layers += [{"kind": "relu"},
               {"kind": "batchnorm", "scale": (1.0 + 0.1 * rng.uniform(-1, 1, 512)).astype(np.float32),
                "offset": (0.1 * rng.uniform(-1, 1, 512)).astype(np.float32)},
               last]
    return layers, left, right, prior


def test_latency_fused_final_with_post_ops(tmp_path, oracle, exp_lib):
    """A last Linear followed by ReLU + BatchNorm: the fused finalize (the
    default) gives the bits of its own reduce launch and the finalize, and
    the oracle's values (experiments library, CATEARS_LAT_FUSED_FINAL)."""
    from conftest import ROOT
    got = {}
    for flag in ("1", "0"):
        env = dict(os.environ, CATEARS_LAT_FUSED_FINAL=flag, PYTHONPATH=ROOT, CATEARS_HIP_LIB=exp_lib)
        path = tmp_path / f"p{flag}.npy"
        r = subprocess.run([sys.executable, "-c", POST_CHILD, str(path), os.path.join(ROOT, "tests")], env=env,
                           capture_output=True, text=True, timeout=300, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        got[flag] = np.load(path)
    assert np.array_equal(bits(got["1"]), bits(got["0"]))
    layers, _, _, _ = post_model_layers()
    x = np.random.default_rng(763).normal(0.0, 3.0, size=(70, 40)).astype(np.float32)
    want = oracle.nnet_propagate(layers, x, gemm=lambda a, w: a @ w)
    assert np.abs(got["1"] - want).max() <= LOGLIK_TOL
