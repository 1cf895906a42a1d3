"""The int8 nnet path (BASELINE config C5, ce_gpu_model_quantize) against the
oracle's restatement of LinearLayer-as-Quantize+MatMat_U8U8F32
(oracle/pyoracle.py nnet_propagate_int8).

Every int8 layer is exact arithmetic -- per-tensor parameters from an exact
min/max, elementwise quantization, an int32 accumulation that is exact modulo
2^32, then float(acc) * (sA*sW) + b and ReLU / BatchNorm in the reference's
rounding order -- so a network without a final LogSoftmax must match bit for
bit.  With the LogSoftmax (a float sum whose order differs) the bar is the
north star's 1e-4.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LOGLIK_TOL = 1e-4


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
def ctx(torch, G):
    return G.Context(0)


def dev(torch, x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def _tdnn(hidden, pdfs, final_logsm=True, seed=3):
    from catears_amd import synth
    layers, left, right, prior = synth.tdnn_layers(hidden, pdfs, seed=seed)
    if not final_logsm:
        layers = [L for L in layers if L["kind"] != "log_softmax"]
    return layers, left, right, prior


@pytest.mark.parametrize("rows", [21, 137, 1100])
def test_int8_block_bit_exact(torch, G, ctx, oracle, rows):
    from catears_amd import formats
    layers, left, right, _ = _tdnn(64, 96, final_logsm=False)
    model = G.Model(ctx, image=formats.nnet_bytes(layers, left, right)).quantize(ctx)
    x = np.random.default_rng(rows).normal(9.0, 3.0, size=(rows, 40)).astype(np.float32)
    got = G.nnet_propagate(ctx, model, dev(torch, x))
    torch.cuda.synchronize()
    want = oracle.nnet_propagate_int8(layers, x)
    got = got.cpu().numpy()
    assert got.shape == want.shape
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def test_int8_blocks_are_independent(torch, G, ctx, oracle):
    """ce_gpu_nnet_propagate_blocks on an int8 model: every block's rows equal
    the block scored alone (per-block quantization parameters), and match the
    oracle bit for bit -- the batcher's contract holds for int8 too."""
    from catears_amd import formats
    layers, left, right, _ = _tdnn(64, 96, final_logsm=False)
    model = G.Model(ctx, image=formats.nnet_bytes(layers, left, right)).quantize(ctx)
    rng = np.random.default_rng(77)
    sizes = [70, 33, 151]
    blocks = [rng.normal(9.0 + 4 * i, 1.0 + 2 * i, size=(n, 40)).astype(np.float32) for i, n in enumerate(sizes)]
    got = G.nnet_propagate_blocks(ctx, model, dev(torch, np.concatenate(blocks)), sizes).cpu().numpy()
    at = 0
    for b in blocks:
        alone = G.nnet_propagate(ctx, model, dev(torch, b)).cpu().numpy()
        want = oracle.nnet_propagate_int8(layers, b)
        part = got[at:at + len(alone)]
        assert np.array_equal(part.view(np.uint32), alone.view(np.uint32))
        assert np.array_equal(part.view(np.uint32), want.view(np.uint32))
        at += len(alone)
    assert at == len(got)


def test_int8_am_forward_matches_oracle(torch, G, ctx, oracle, xs_config):
    from catears_amd import formats, synth
    am = formats.read_am(xs_config)
    model = G.Model(ctx, xs_config).quantize(ctx)
    wave = synth.pcm(41, 16000 * 4 + 77)
    feats = oracle.Fbank().compute(wave)
    plan = G.Plan(ctx, [len(wave)], model)  # one utterance, one chunk
    out = G.am_forward(ctx, model, plan, dev(torch, feats))
    torch.cuda.synchronize()
    L, R = am["left"], am["right"]
    block = np.concatenate([np.repeat(feats[:1], L, 0), feats, np.repeat(feats[-1:], R, 0)], 0)
    want = oracle.nnet_propagate_int8(am["layers"], block) - am["log_prior"][None, :]
    assert np.max(np.abs(out.cpu().numpy() - want)) <= LOGLIK_TOL


def test_int8_tracks_fp32(torch, G, ctx, oracle, xs_config):
    """Not parity (int8 is an approximation): the C5 question of how far the
    int8 posteriors move from fp32 -- argmax agreement and a loose bound."""
    from catears_amd import synth
    m32 = G.Model(ctx, xs_config)
    m8 = G.Model(ctx, xs_config).quantize(ctx)
    waves = [synth.pcm(50 + i, 16000 * 3) for i in range(3)]
    plan = G.Plan(ctx, [len(w) for w in waves], m32)
    pcm = dev(torch, np.concatenate(waves))
    a = G.score(ctx, m32, plan, pcm).cpu().numpy()
    b = G.score(ctx, m8, plan, pcm).cpu().numpy()
    agree = float(np.mean(a.argmax(1) == b.argmax(1)))
    assert agree > 0.5, agree
    assert np.isfinite(b).all()


def test_int8_c5_full_batch(torch, G, ctx, oracle):
    """BASELINE config C5 at its size: TDNN-S int8, one 8192-row block
    (ce_gpu_nnet_propagate), against the oracle's int8 restatement over the
    whole block (its u8 GEMMs through the exact float64 form, so every row of
    every layer -- and hence every per-tensor quantization parameter -- is
    the reference's).  Without the final LogSoftmax every output bit must
    match; with it (a float sum in another order) 1e-4."""
    from catears_amd import formats, synth
    layers, left, right, _ = synth.tdnn_layers(1024, 3456, seed=7)
    body = [L for L in layers if L["kind"] != "log_softmax"]
    x = np.random.default_rng(8192).normal(9.0, 3.0, size=(8192, 40)).astype(np.float32)
    want = oracle.nnet_propagate_int8(body, x, exact_f64=True)
    m_body = G.Model(ctx, image=formats.nnet_bytes(body, left, right)).quantize(ctx)
    got = G.nnet_propagate(ctx, m_body, dev(torch, x)).cpu().numpy()
    assert got.shape == want.shape == (8192 - left - right, 3456)
    diff = np.flatnonzero(got.view(np.uint32) != want.view(np.uint32))
    assert diff.size == 0, f"{diff.size} elements differ, first at {np.unravel_index(diff[0], got.shape)}"
    m_full = G.Model(ctx, image=formats.nnet_bytes(layers, left, right)).quantize(ctx)
    got_ls = G.nnet_propagate(ctx, m_full, dev(torch, x)).cpu().numpy()
    want_ls = oracle.layer_forward({"kind": "log_softmax"}, want)
    assert np.max(np.abs(got_ls - want_ls)) <= LOGLIK_TOL


@pytest.mark.parametrize("case", ["dead_layer", "wide_range"])
def test_int8_quantize_edge_ranges(torch, G, ctx, oracle, case):
    """Hidden-layer Quantize passes (quantize_fast_kernel) at the edges of the
    parameter math.  dead_layer: a Linear whose ReLU output is all zero, so
    the next layer's range is [0, FLT_MIN] (max starts at FLT_MIN,
    matrix.cc:332) and its scale FLT_MIN / 255 is a denormal: the corrected
    reciprocal overflows and every element takes the division fallback.
    wide_range: a Linear scaled by 2^90, outputs near 1e27.  Bit for bit
    against the oracle either way."""
    from catears_amd import formats
    layers, left, right, _ = _tdnn(64, 96, final_logsm=False)
    lin = [i for i, L in enumerate(layers) if L["kind"] == "linear"]
    i = lin[1]
    if case == "dead_layer":
        layers[i] = dict(layers[i], W=np.zeros_like(layers[i]["W"]), b=np.full_like(layers[i]["b"], -1.0))
        bn = next(j for j in range(i, len(layers)) if layers[j]["kind"] == "batchnorm")
        layers[bn] = dict(layers[bn], offset=np.zeros_like(layers[bn]["offset"]))
    else:
        layers[i] = dict(layers[i], W=(layers[i]["W"] * np.float32(2.0 ** 90)).astype(np.float32))
    model = G.Model(ctx, image=formats.nnet_bytes(layers, left, right)).quantize(ctx)
    x = np.random.default_rng(5).normal(9.0, 3.0, size=(700, 40)).astype(np.float32)
    got = G.nnet_propagate(ctx, model, dev(torch, x)).cpu().numpy()
    want = oracle.nnet_propagate_int8(layers, x)
    assert got.shape == want.shape
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
