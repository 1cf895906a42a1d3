"""The fast fbank mode (ce_gpu_ctx_set_fbank(ctx, CE_GPU_FBANK_FAST),
kernels/fbank_fma.hip): the exact kernel's lane program built with FMA
contraction and a single-precision pre-emphasis, so its products and sums
round differently from the reference's and its bar is the north star's
fbank tolerance rather than bit-exactness.  (Rounds 3-4 ran a four-step
16 x 16 FFT here; the contracted lane program is faster and as accurate.)

Two yardsticks.  (1) The oracle (the reference's fp32 arithmetic): log-mel
within 1e-4 on the reference's speech WAVs (the reference
itself is held to 1e-4 against Kaldi, test/fbank_test.cc:56) and < 1e-4
against the Kaldi dump; within SYNTH_TOL (the sum of the two fp32 errors) on
the synthetic ragged set and C2 set.  (2) The exact result
(pyoracle.fbank_f64, float64 with an exact FFT): the reference's own fp32
rounding puts the oracle up to ~8e-5 from it on the lowest mel band (where
pre-emphasis leaves ~1e-3 of the frame's energy, so the FFT's error relative
to the frame is magnified), so the SURVEY's 3e-5 target is not reachable
against the oracle by any other operation order -- it is checked against the
exact result instead, where the fast mode must be about as accurate as the
reference: max |fast - exact| <= 1.25 max |oracle - exact| on the same
frames, and <= 3e-5 at the 99.9th percentile."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FAST_TOL = 1e-4   # against the oracle (the north star's fbank tolerance)
EXACT_P999 = 3e-5  # against the exact float64 result, 99.9th percentile
# synthetic noise-rich audio leaves the lowest mel band ~1e-3 of a frame's
# energy after pre-emphasis: there the reference's fp32 order alone is up to
# ~1e-4 from the exact result, and the fast mode's fp32 rounding adds its own
SYNTH_TOL = 2e-4


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
def fctx(torch, G):
    c = G.Context(0)
    c.set_fbank("fast")
    return c


def run(torch, G, ctx, waves, dtype=np.float32):
    plan = G.Plan(ctx, [len(w) for w in waves])
    cat = np.concatenate(waves).astype(dtype) if waves else np.zeros(1, dtype)
    feats = torch.empty((max(plan.total_frames, 1), 40), dtype=torch.float32, device="cuda")
    mel = torch.empty_like(feats)
    G.fbank(ctx, plan, torch.from_numpy(np.ascontiguousarray(cat)).cuda(), feats, mel)
    torch.cuda.synchronize()
    return plan, feats.cpu().numpy()[:plan.total_frames], mel.cpu().numpy()[:plan.total_frames]


def test_fast_goldens(torch, G, fctx, oracle):
    waves = [oracle.read_wav(os.path.join(GOLDEN, n)) for n in ("en-us-hello.wav", "en-us-cat.wav")]
    plan, f, _ = run(torch, G, fctx, waves)
    fb = oracle.Fbank()
    off = plan.frame_offsets
    for u, w in enumerate(waves):
        assert np.abs(f[off[u]:off[u + 1]] - fb.compute(w)).max() <= FAST_TOL
    k = np.loadtxt(os.path.join(GOLDEN, "fbankmat_en-us-hello.wav.txt")).reshape(-1, 40)
    assert np.abs(f[:47] - k).max() < 1e-4  # test/fbank_test.cc:56


def test_fast_ragged_edges(torch, G, fctx, oracle):
    from catears_amd import synth
    lengths = [0, 399, 400, 401, 559, 560, 16000, 1, 160000, 33333]
    waves = [synth.pcm(100 + i, n) for i, n in enumerate(lengths)]
    waves.append(np.zeros(16000, np.float32))          # log-floor path
    waves.append(np.full(16000, 32767.0, np.float32))  # DC only
    waves.append(np.full(16001, -32768.0, np.float32))
    plan, f, _ = run(torch, G, fctx, waves)
    fb = oracle.Fbank()
    off = plan.frame_offsets
    for u, w in enumerate(waves):
        of = fb.compute(w)
        assert off[u + 1] - off[u] == len(of)
        if len(of):
            assert np.abs(f[off[u]:off[u + 1]] - of).max() <= SYNTH_TOL, f"utt {u}"
    # the int16 entry point gives the same bits as the float one here too
    _, f16, _ = run(torch, G, fctx, [w.astype(np.int16) for w in waves], np.int16)
    assert np.array_equal(f16.view(np.uint32), f.view(np.uint32))


def test_fast_c2_set(torch, G, fctx, oracle):
    """C2's utterances (10 s synthetic), 200 of them in one launch: against
    the exact result the fast mode is about as accurate as the reference's
    own fp32 order (the oracle); against the oracle within the sum of the two
    fp32 errors (SYNTH_TOL); and a frame does not depend on its neighbours
    (the batch reversed gives the same rows, bit for bit)."""
    from catears_amd import synth
    base = [synth.pcm(5000 + i, 160000) for i in range(20)]
    waves = [base[i % 20] * (1.0 if (i // 20) % 2 == 0 else -1.0) for i in range(200)]
    plan, f, _ = run(torch, G, fctx, waves)
    fb = oracle.Fbank()
    off = plan.frame_offsets
    fast_err, ref_err, vs_oracle = [], [], []
    for u in range(8):
        ex = oracle.fbank_f64(waves[u])
        of = fb.compute(waves[u])
        fast_err.append(np.abs(f[off[u]:off[u + 1]] - ex).ravel())
        ref_err.append(np.abs(of - ex).ravel())
        vs_oracle.append(np.abs(f[off[u]:off[u + 1]] - of).ravel())
    fast_err, ref_err, vs_oracle = map(np.concatenate, (fast_err, ref_err, vs_oracle))
    print(f"vs exact: fast max {fast_err.max():.3g} p99.9 {np.quantile(fast_err, 0.999):.3g}; "
          f"oracle max {ref_err.max():.3g} p99.9 {np.quantile(ref_err, 0.999):.3g}; "
          f"fast vs oracle max {vs_oracle.max():.3g} p99.9 {np.quantile(vs_oracle, 0.999):.3g}")
    assert fast_err.max() <= 1.25 * ref_err.max()
    assert np.quantile(fast_err, 0.999) <= EXACT_P999
    assert vs_oracle.max() <= SYNTH_TOL
    plan_r, f_r, _ = run(torch, G, fctx, waves[::-1])
    for u in range(0, 200, 17):
        v = 199 - u
        assert np.array_equal(f[off[u]:off[u + 1]].view(np.uint32),
                              f_r[plan_r.frame_offsets[v]:plan_r.frame_offsets[v + 1]].view(np.uint32))


def test_mode_switch_and_default(torch, G, oracle):
    from catears_amd import synth
    ctx = G.Context(0)
    w = [synth.pcm(7, 16000)]
    _, fe, me = run(torch, G, ctx, w)  # default: exact
    _, om = oracle.Fbank().compute(w[0], with_mel=True)
    assert np.array_equal(me.view(np.uint32), np.ascontiguousarray(om, np.float32).view(np.uint32))
    ctx.set_fbank("fast")
    _, ff, _ = run(torch, G, ctx, w)
    assert np.abs(ff - fe).max() <= SYNTH_TOL
    ctx.set_fbank("exact")
    _, fe2, _ = run(torch, G, ctx, w)
    assert np.array_equal(fe2.view(np.uint32), fe.view(np.uint32))
    with pytest.raises(KeyError):
        ctx.set_fbank("approximate")
