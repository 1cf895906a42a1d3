"""16-bit PCM ingestion: ce_gpu_fbank_s16 /
ce_gpu_score_s16 read the WAV payload's little-endian int16 samples and do
WaveReader::Process's int16 -> float conversion (src/pcm_reader.cc:148-190,
:174) inside the kernel's loads.  The conversion is exact, so the features
must be bit-identical to the fp32 entry point on the converted floats -- and
through it to the oracle (pre-log mel bit-exact) -- on the reference's WAVs
and on the ragged edge set; the whole scoring path likewise."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

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
def ctx(torch, G):
    return G.Context(0)


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def wav_int16(path):
    """The 16-bit payload exactly as Read16kPcm slices it (file size - 44)."""
    raw = open(path, "rb").read()
    body = raw[44:]
    return np.frombuffer(body[:len(body) // 2 * 2], dtype="<i2").copy()


def both(torch, G, ctx, waves16):
    plan = G.Plan(ctx, [len(w) for w in waves16])
    cat = np.concatenate(waves16) if waves16 else np.zeros(1, np.int16)
    n = max(plan.total_frames, 1)
    out = {}
    for kind, host in (("s16", cat.astype(np.int16)), ("f32", cat.astype(np.float32))):
        pcm = torch.from_numpy(np.ascontiguousarray(host)).cuda()
        feats = torch.empty((n, 40), dtype=torch.float32, device="cuda")
        mel = torch.empty_like(feats)
        G.fbank(ctx, plan, pcm, feats, mel)
        torch.cuda.synchronize()
        out[kind] = (feats.cpu().numpy()[:plan.total_frames], mel.cpu().numpy()[:plan.total_frames])
    return plan, out


def test_s16_goldens_bit_identical(torch, G, ctx, oracle):
    names = ("en-us-hello.wav", "en-us-cat.wav")
    w16 = [wav_int16(os.path.join(GOLDEN, n)) for n in names]
    for n, w in zip(names, w16):  # the oracle's reader gives the same samples
        assert np.array_equal(oracle.read_wav(os.path.join(GOLDEN, n)), w.astype(np.float32))
    plan, out = both(torch, G, ctx, w16)
    assert np.array_equal(bits(out["s16"][0]), bits(out["f32"][0]))
    assert np.array_equal(bits(out["s16"][1]), bits(out["f32"][1]))
    fb = oracle.Fbank()
    off = plan.frame_offsets
    for u, w in enumerate(w16):
        _, om = fb.compute(w.astype(np.float32), with_mel=True)
        assert np.array_equal(bits(out["s16"][1][off[u]:off[u + 1]]), bits(om))
    k = np.loadtxt(os.path.join(GOLDEN, "fbankmat_en-us-hello.wav.txt")).reshape(-1, 40)
    assert np.abs(out["s16"][0][:47] - k).max() < 1e-4  # test/fbank_test.cc:56


def test_s16_ragged_edges_bit_identical(torch, G, ctx):
    from catears_amd import synth
    lengths = [0, 399, 400, 559, 560, 16000, 160000, 1, 1600000]
    waves = [synth.pcm(100 + i, n).astype(np.int16) for i, n in enumerate(lengths)]
    waves.append(np.zeros(16000, np.int16))
    waves.append(np.full(16000, 32767, np.int16))
    waves.append(np.full(16001, -32768, np.int16))   # the int16 minimum
    plan, out = both(torch, G, ctx, waves)
    assert plan.total_frames > 0
    assert np.array_equal(bits(out["s16"][0]), bits(out["f32"][0]))
    assert np.array_equal(bits(out["s16"][1]), bits(out["f32"][1]))


def test_score_s16_matches_score(torch, G, ctx, xs_config, global_stats):
    from catears_amd import synth
    model = G.Model(ctx, xs_config)
    waves = [synth.pcm(300 + i, n).astype(np.int16) for i, n in enumerate([16000, 8000, 560, 33333])]
    plan = G.Plan(ctx, [len(w) for w in waves], model)
    gs = torch.from_numpy(global_stats).cuda()
    cat = np.concatenate(waves)
    a = G.score(ctx, model, plan, torch.from_numpy(cat).cuda(), gs)
    b = G.score(ctx, model, plan, torch.from_numpy(cat.astype(np.float32)).cuda(), gs)
    torch.cuda.synchronize()
    assert np.array_equal(bits(a.cpu().numpy()), bits(b.cpu().numpy()))


def test_fbank_rejects_other_sample_types(torch, G, ctx):
    plan = G.Plan(ctx, [16000])
    with pytest.raises(TypeError):
        G.fbank(ctx, plan, torch.zeros(16000, dtype=torch.int32, device="cuda"))
