"""Parity of the HIP path (through the C-ABI) with the oracle, on an MI355X.

Bars: bit-exact where the reference is exact IEEE arithmetic -- pre-log mel
energies, CMVN, Quantize, the int32 u8 GEMM accumulator -- and for fp32 GEMM
work the north-star tolerance, |loglik - oracle| <= 1e-4 absolute.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

LOGLIK_TOL = 1e-4   # BASELINE.json north star: log-likelihoods within 1e-4
FEAT_TOL = 1e-5     # log-mel: only the final logf may differ (<= 1-2 ulp)


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


@pytest.fixture(scope="module")
def G():
    from catears_amd import gpu
    gpu.lib()  # fail loudly if the HIP library is missing
    return gpu


@pytest.fixture(scope="module")
def ctx(torch, G):
    return G.Context(0)


def dev(torch, x):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def gpu_fbank(torch, G, ctx, waves, with_mel=True):
    plan = G.Plan(ctx, [len(w) for w in waves])
    pcm = dev(torch, np.concatenate(waves) if waves else np.zeros(1, np.float32))
    feats = torch.empty((max(plan.total_frames, 1), 40), dtype=torch.float32, device="cuda")
    mel = torch.empty_like(feats) if with_mel else None
    G.fbank(ctx, plan, pcm, feats, mel)
    torch.cuda.synchronize()
    off = plan.frame_offsets
    f = feats.cpu().numpy()[:plan.total_frames]
    m = mel.cpu().numpy()[:plan.total_frames] if with_mel else None
    return plan, off, f, m


# ------------------------------------------------------------------ fbank --

def test_fbank_goldens(torch, G, ctx, oracle):
    waves = [oracle.read_wav(os.path.join(GOLDEN, n)) for n in ("en-us-hello.wav", "en-us-cat.wav")]
    plan, off, f, m = gpu_fbank(torch, G, ctx, waves)
    fb = oracle.Fbank()
    for u, w in enumerate(waves):
        of, om = fb.compute(w, with_mel=True)
        assert np.array_equal(bits(m[off[u]:off[u + 1]]), bits(om)), "pre-log mel not bit-exact"
        assert np.abs(f[off[u]:off[u + 1]] - of).max() <= FEAT_TOL
    k = np.loadtxt(os.path.join(GOLDEN, "fbankmat_en-us-hello.wav.txt")).reshape(-1, 40)
    assert np.abs(f[:47] - k).max() < 1e-4  # test/fbank_test.cc:56


def test_fbank_ragged_batch_edges(torch, G, ctx, oracle):
    from catears_amd import synth
    lengths = [0, 399, 400, 559, 560, 16000, 160000, 1, 1600000]
    waves = [synth.pcm(100 + i, n) for i, n in enumerate(lengths)]
    waves.append(np.zeros(16000, np.float32))                 # log-floor path
    waves.append(np.full(16000, 32767.0, np.float32))         # DC only
    plan, off, f, m = gpu_fbank(torch, G, ctx, waves)
    fb = oracle.Fbank()
    for u, w in enumerate(waves):
        of, om = fb.compute(w, with_mel=True)
        assert off[u + 1] - off[u] == len(of)
        if len(of):
            assert np.array_equal(bits(m[off[u]:off[u + 1]]), bits(om)), f"utt {u}"
            assert np.abs(f[off[u]:off[u + 1]] - of).max() <= FEAT_TOL


def test_fbank_full_c2_scale(torch, G, ctx, oracle):
    """BASELINE config C2 at full size -- 1000 x 10 s utterances, 998 000
    frames in one launch -- every pre-log mel energy bit-exact against the
    oracle, plus the size-independent property that an utterance's frames do
    not depend on its neighbours (the batch reversed gives the same rows)."""
    from catears_amd import synth
    n = 160000
    base = [synth.pcm(5000 + i, n) for i in range(40)]
    waves = [base[i % 40] * (1.0 if (i // 40) % 2 == 0 else -1.0) for i in range(1000)]  # 80 distinct
    plan, off, f, m = gpu_fbank(torch, G, ctx, waves)
    assert plan.total_frames == 998000
    fb = oracle.Fbank()
    ref = {}
    for i in range(80):
        ref[i] = fb.compute(waves[i], with_mel=True)
    for u in range(1000):
        of, om = ref[u % 80]
        assert np.array_equal(bits(m[off[u]:off[u + 1]]), bits(om)), f"utt {u}"
        assert np.abs(f[off[u]:off[u + 1]] - of).max() <= FEAT_TOL
    plan_r, off_r, f_r, m_r = gpu_fbank(torch, G, ctx, waves[::-1])
    for u in range(0, 1000, 37):
        v = 999 - u
        assert np.array_equal(bits(m[off[u]:off[u + 1]]), bits(m_r[off_r[v]:off_r[v + 1]]))


# ------------------------------------------------------------------- cmvn --

def test_cmvn_bitexact(torch, G, ctx, oracle, global_stats):
    from catears_amd import synth
    waves = [synth.pcm(200 + i, n) for i, n in enumerate([16000, 400, 0, 160000, 250000])]
    plan, off, f, _ = gpu_fbank(torch, G, ctx, waves, with_mel=False)
    feats = dev(torch, f)
    out = G.cmvn(ctx, plan, dev(torch, global_stats), feats)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    for u in range(len(waves)):
        ref = oracle.cmvn(global_stats, f[off[u]:off[u + 1]])
        assert np.array_equal(bits(o[off[u]:off[u + 1]]), bits(ref)), f"utt {u}"
    k = np.loadtxt(os.path.join(GOLDEN, "fbankcmvnmat_en-us-hello.wav.txt")).reshape(-1, 40)
    w = oracle.read_wav(os.path.join(GOLDEN, "en-us-hello.wav"))
    p2, _, f2, _ = gpu_fbank(torch, G, ctx, [w], with_mel=False)
    c2 = G.cmvn(ctx, p2, dev(torch, global_stats), dev(torch, f2)).cpu().numpy()
    assert np.abs(c2 - k).max() < 1e-4  # test/cmvn_test.cc:76, two-sided


def test_cmvn_rejects_aliasing(torch, G, ctx, global_stats):
    plan = G.Plan(ctx, [16000])
    x = torch.zeros((plan.total_frames, 40), dtype=torch.float32, device="cuda")
    with pytest.raises(G.CatearsError):
        G.cmvn(ctx, plan, dev(torch, global_stats), x, x)


# --------------------------------------------------------------------- am --

def am_oracle(oracle, am, feats, gemm=None):
    return oracle.am_stream(am, feats, chunk_size=am["chunk"], gemm=gemm)


@pytest.mark.parametrize("gemm", ["fp32", "bf16x6", "bf16x6p", "f16x3"])
def test_am_xs_vs_oracle(torch, G, ctx, oracle, xs_config, gemm):
    from catears_amd import formats, synth
    am = formats.read_am(xs_config)
    model = G.Model(ctx, xs_config).set_gemm(gemm)
    assert (model.left, model.right, model.input_dim, model.num_pdfs) == (10, 10, 40, 512)
    assert np.array_equal(model.tid2pdf(), am["tid2pdf"])
    fb = oracle.Fbank()
    feats = [fb.compute(synth.pcm(300 + i, n)) for i, n in enumerate([16000, 560, 400, 48000, 3000])]
    feats.insert(2, np.zeros((0, 40), np.float32))
    plan = G.Plan(ctx, [(len(x) - 1) * 160 + 400 if len(x) else 0 for x in feats], model)
    assert plan.total_frames == sum(len(x) for x in feats)
    out = G.am_forward(ctx, model, plan, dev(torch, np.concatenate(feats)))
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    off = plan.frame_offsets
    for u, x in enumerate(feats):
        ref = am_oracle(oracle, am, x)
        assert ref.shape == (off[u + 1] - off[u], 512)
        if len(x):
            assert np.abs(o[off[u]:off[u + 1]] - ref).max() <= LOGLIK_TOL, f"utt {u}"


def test_long_propagate_runs_in_exact_windows(torch, G, ctx, oracle, xs_config):
    """ce_gpu_nnet_propagate on a block longer than its 65536-row window:
    the windowed pass gives the same bits as scoring two overlapping halves
    separately, and the rows around the window seam match the oracle."""
    from catears_amd import formats
    am = formats.read_am(xs_config)
    model = G.Model(ctx, xs_config)
    ctx_rows = model.left + model.right
    rows = (1 << 16) + 3001
    x = np.random.default_rng(65).normal(9.0, 3.0, size=(rows, 40)).astype(np.float32)
    dx = dev(torch, x)
    got = G.nnet_propagate(ctx, model, dx).cpu().numpy()
    assert got.shape == (rows - ctx_rows, 512)
    cut = 40000
    a = G.nnet_propagate(ctx, model, dx[:cut + ctx_rows]).cpu().numpy()
    b = G.nnet_propagate(ctx, model, dx[cut:]).cpu().numpy()
    assert np.array_equal(bits(got), bits(np.concatenate([a, b])))
    seam = (1 << 16) - ctx_rows
    lo, hi = seam - 40, seam + 40
    want = oracle.nnet_propagate(am["layers"], x[lo:hi + ctx_rows])
    assert np.abs(got[lo:hi] - want).max() <= LOGLIK_TOL


@pytest.mark.parametrize("gemm", ["fp32", "bf16x6", "bf16x6p", "f16x3"])
def test_am_segmentation_is_exact(torch, G, ctx, oracle, xs_config, gemm):
    """Splitting an utterance over chunks (max_rows) must not change a bit:
    every output element is the same k-ordered MFMA chain whatever the row's
    position."""
    from catears_amd import synth
    model = G.Model(ctx, xs_config).set_gemm(gemm)
    fb = oracle.Fbank()
    feats = [fb.compute(synth.pcm(400 + i, n)) for i, n in enumerate([48000, 16000, 30000])]
    ns = [(len(x) - 1) * 160 + 400 for x in feats]
    x = dev(torch, np.concatenate(feats))
    outs = []
    for max_rows in (4096, 333, 64):
        plan = G.Plan(ctx, ns, model, max_rows=max_rows)
        outs.append(G.am_forward(ctx, model, plan, x).cpu().numpy())
    assert np.array_equal(bits(outs[0]), bits(outs[1]))
    assert np.array_equal(bits(outs[0]), bits(outs[2]))


@pytest.mark.parametrize("gemm", ["fp32", "bf16x6", "bf16x6p", "f16x3"])
def test_am_s_vs_oracle(torch, G, ctx, oracle, s_config, gemm):
    """Benchmark model (TDNN-S, 34.75 MFLOP/frame) on two utterances; the
    oracle's GEMM is numpy fp32 here for speed (any fp32 summation order is
    the reference algorithm; OpenBLAS's order is not pinned either)."""
    from catears_amd import formats, synth
    am = formats.read_am(s_config)
    model = G.Model(ctx, s_config).set_gemm(gemm)
    assert model.num_pdfs == 3456 and model.num_linear == 7
    fb = oracle.Fbank()
    feats = [fb.compute(synth.pcm(500 + i, n)) for i, n in enumerate([48000, 20000])]
    plan = G.Plan(ctx, [48000, 20000], model)
    out = G.am_forward(ctx, model, plan, dev(torch, np.concatenate(feats))).cpu().numpy()
    off = plan.frame_offsets
    for u, x in enumerate(feats):
        ref = oracle.am_whole(am, x, gemm=lambda a, w: a @ w)
        assert np.abs(out[off[u]:off[u + 1]] - ref).max() <= LOGLIK_TOL


def test_split_gemms_are_fp32_accurate(torch, G, ctx, oracle, s_config):
    """The bf16x6 and f16x3 split GEMMs are fp32 GEMMs: on TDNN-S their
    log-likelihood error against an fp64 evaluation of the same network is of
    the fp32-MFMA path's size, and far inside 1e-4.  A single-plane bf16 or
    fp16 GEMM would miss by orders of magnitude."""
    from catears_amd import formats, synth
    am = formats.read_am(s_config)
    fb = oracle.Fbank()
    feats = [fb.compute(synth.pcm(520 + i, n)) for i, n in enumerate([64000, 32000])]
    x = dev(torch, np.concatenate(feats))
    errs = {}
    for gemm in ("fp32", "bf16x6", "f16x3"):
        model = G.Model(ctx, s_config).set_gemm(gemm)
        assert model.gemm == gemm
        plan = G.Plan(ctx, [64000, 32000], model)
        out = G.am_forward(ctx, model, plan, x).cpu().numpy()
        off = plan.frame_offsets
        e = 0.0
        for u, f in enumerate(feats):
            ref = oracle.am_whole(am, f, gemm=lambda a, w: (a.astype(np.float64) @ w.astype(np.float64)).astype(np.float32))
            e = max(e, float(np.abs(out[off[u]:off[u + 1]] - ref).max()))
        errs[gemm] = e
    for gemm in ("bf16x6", "f16x3"):
        assert errs[gemm] <= max(2.0 * errs["fp32"], 2e-5), errs
        assert errs[gemm] <= LOGLIK_TOL / 2, errs
    assert not ctx.overflow()


def test_score_pipeline_with_cmvn(torch, G, ctx, oracle, xs_config, global_stats):
    from catears_amd import formats, synth
    am = formats.read_am(xs_config)
    model = G.Model(ctx, xs_config)
    waves = [synth.pcm(600 + i, n) for i, n in enumerate([32000, 16000, 799])]
    plan = G.Plan(ctx, [len(w) for w in waves], model)
    out = G.score(ctx, model, plan, dev(torch, np.concatenate(waves)), dev(torch, global_stats)).cpu().numpy()
    off = plan.frame_offsets
    fb = oracle.Fbank()
    for u, w in enumerate(waves):
        ref = am_oracle(oracle, am, oracle.cmvn(global_stats, fb.compute(w)))
        assert np.abs(out[off[u]:off[u + 1]] - ref).max() <= LOGLIK_TOL


def test_c3_full_batch_vs_oracle(torch, G, ctx, oracle, s_config):
    """The benchmark's own step at full size: four 10 s utterances packed
    into one 4072-row chunk, fbank -> CMVN (synthetic global stats, as
    bench.py) -> TDNN-S in the default GEMM mode -> minus log prior, against
    the oracle (fbank / CMVN restatement in C, the network in fp64) within the
    north star's 1e-4 on every log-likelihood."""
    from catears_amd import formats, synth
    am = formats.read_am(s_config)
    model = G.Model(ctx, s_config)
    n = 160000
    waves = [synth.pcm(i, n) for i in range(4)]  # bench.py's rank-0 pool seeds
    gstats = synth.cmvn_stats_synthetic()
    plan = G.Plan(ctx, [n] * 4, model)
    assert plan.total_frames == 4 * 998
    out = G.score(ctx, model, plan, dev(torch, np.concatenate(waves)), dev(torch, gstats)).cpu().numpy()
    off = plan.frame_offsets
    fb = oracle.Fbank()
    f64 = lambda a, w: (a.astype(np.float64) @ w.astype(np.float64)).astype(np.float32)
    worst = 0.0
    for u, w in enumerate(waves):
        ref = oracle.am_whole(am, oracle.cmvn(gstats, fb.compute(w)), gemm=f64)
        worst = max(worst, float(np.abs(out[off[u]:off[u + 1]] - ref).max()))
    assert np.isfinite(out).all()
    assert worst <= LOGLIK_TOL, worst


def test_model_rejects_bad_topology(torch, G, ctx, tmp_path):
    from catears_amd import formats
    W = np.ones((40, 8), np.float32)
    layers = [{"kind": "splice", "indices": [-1, 0, 1]}, {"kind": "linear", "W": np.ones((120, 8), np.float32),
                                                          "b": np.zeros(8, np.float32)}]
    p = tmp_path / "bad.nnet"
    p.write_bytes(formats.nnet_bytes(layers, 1, 1))
    pr = tmp_path / "bad.prior"
    pr.write_bytes(formats.vec_bytes(np.full(8, 0.125, np.float32)))
    with pytest.raises(G.CatearsError) as e:
        G.Model(ctx, nnet=str(p), prior=str(pr), left=1, right=1)
    assert e.value.code == -6  # ENOTSUP: splice without its narrow
    p.write_bytes(b"NN02" + b"\x00" * 8 + (1).to_bytes(4, "little") + b"LAY0" + (5).to_bytes(4, "little"))
    with pytest.raises(G.CatearsError) as e:
        G.Model(ctx, nnet=str(p), prior=str(pr), left=0, right=0)
    assert e.value.code == -5 and "unexpected layer type" in str(e.value)
    del W


# ------------------------------------------------------------ linear alg --

@pytest.mark.parametrize("shape", [(5, 3, 2), (100, 100, 1), (1024, 1024, 80), (121, 233, 17),
                                   (4096, 1024, 3072), (300, 3456, 1024)])
def test_sgemm(torch, G, ctx, shape):
    m, n, k = shape
    rng = np.random.default_rng(m + n + k)
    A = rng.uniform(-0.5, 0.5, (m, k)).astype(np.float32)
    B = rng.uniform(1, 2, (k, n)).astype(np.float32)
    C = G.sgemm(ctx, dev(torch, A), dev(torch, B)).cpu().numpy()
    exact = A.astype(np.float64) @ B.astype(np.float64)
    # fp32 fma chain: error << test/gemm_test.cc:104's 1e-2
    assert np.abs(C - exact).max() <= 1e-6 * np.abs(A).sum(1).max() * 2 * k ** 0.5 + 1e-5


@pytest.mark.parametrize("shape", [(5, 3, 2), (100, 100, 1), (1024, 1024, 80), (121, 233, 17),
                                   (257, 300, 1000), (8192, 1024, 3072)])
def test_quantize_and_u8_gemm_bitexact(torch, G, ctx, oracle, shape):
    m, n, k = shape
    rng = np.random.default_rng(3 * m + n)
    A = rng.uniform(-0.5, 0.5, (m, k)).astype(np.float32)
    B = rng.uniform(1, 2, (k, n)).astype(np.float32)
    qa, pa = G.quantize(ctx, dev(torch, A))
    qb, pb = G.quantize(ctx, dev(torch, B))
    oa, sa, za = oracle.quantize(A)
    ob, sb, zb = oracle.quantize(B)
    assert G.params_host(pa) == (sa, za) and G.params_host(pb) == (sb, zb)
    assert np.array_equal(qa.cpu().numpy(), oa) and np.array_equal(qb.cpu().numpy(), ob)
    if m * n * k > 2e9:  # oracle int32 GEMM too slow: check a row/column sample
        ri = rng.choice(m, 16, replace=False)
        ci = np.arange(n)
        ref_i = oracle.gemm_u8u8_i32(oa[ri], za, ob, zb)
        got_i = G.gemm_u8(ctx, qa, pa, qb, pb, out_int32=True).cpu().numpy()[ri][:, ci]
        assert np.array_equal(got_i, ref_i)
        return
    ref_i = oracle.gemm_u8u8_i32(oa, za, ob, zb)
    got_i = G.gemm_u8(ctx, qa, pa, qb, pb, out_int32=True).cpu().numpy()
    assert np.array_equal(got_i, ref_i)
    got_f = G.gemm_u8(ctx, qa, pa, qb, pb).cpu().numpy()
    assert np.array_equal(bits(got_f), bits(oracle.gemm_u8u8f32(oa, sa, za, ob, sb, zb)))


def test_bf16x6_plane_and_fp32_operand_kernels_agree_bitwise(torch, G, ctx, oracle, s_config):
    """CE_GPU_GEMM_BF16X6 (fp32 operands split on the way into LDS) and
    CE_GPU_GEMM_BF16X6_PLANES (planes written by each epilogue, read from
    HBM) form the same six products per element in the same order: the
    log-likelihoods must agree bit for bit (ragged utterances, several
    chunks)."""
    from catears_amd import synth
    fb = oracle.Fbank()
    lens = [64000, 17777, 48000]
    feats = [fb.compute(synth.pcm(540 + i, n)) for i, n in enumerate(lens)]
    x = dev(torch, np.concatenate(feats))
    outs = []
    for gemm in ("bf16x6", "bf16x6p"):
        model = G.Model(ctx, s_config).set_gemm(gemm)
        plan = G.Plan(ctx, lens, model, max_rows=2048)
        outs.append(G.am_forward(ctx, model, plan, x).cpu().numpy())
    assert np.array_equal(bits(outs[0]), bits(outs[1]))


def test_f16x3_overflow_is_flagged(torch, G, ctx, xs_config):
    """Activations beyond the f16x3 range (|x| >= 1.6e7) cannot be stored in
    the two fp16 planes: the context's overflow word reports it; in range,
    it stays clear."""
    model = G.Model(ctx, xs_config).set_gemm("f16x3")
    rng = np.random.default_rng(7)
    x = rng.standard_normal((64, 40)).astype(np.float32)
    assert not ctx.overflow()
    G.nnet_propagate(ctx, model, dev(torch, x))
    assert not ctx.overflow()
    x[10, 3] = 3e7
    G.nnet_propagate(ctx, model, dev(torch, x))
    assert ctx.overflow()
    assert not ctx.overflow()  # read clears it
