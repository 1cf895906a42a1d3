"""The oracle against the reference's own golden vectors and, where the
reference compiles here (oracle/_ref), against the reference itself."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_srfft128_golden(oracle):
    # test/srfft_test.cc:13,144,285 -- 128-point real FFT, |d| < 1e-4
    g = json.load(open(os.path.join(GOLDEN, "srfft128.json")))
    out = oracle.srfft_forward(np.array(g["input"], np.float32))
    exp = np.array(g["expected_prefix"], np.float32)
    assert np.abs(out[:len(exp)] - exp).max() < g["tol"]


@pytest.mark.parametrize("n", [16, 64, 128, 512, 1024])
def test_srfft_bitexact_vs_reference(oracle, n):
    R = oracle.ref_lib()
    if R is None:
        pytest.skip("oracle/_ref not built (reference absent)")
    rng = np.random.default_rng(n)
    for scale in (1.0, 3e4):
        x = (rng.standard_normal(n) * scale).astype(np.float32)
        ours = oracle.srfft_forward(x)
        ref = x.copy()
        h = R.ref_srfft_new(n)
        R.ref_srfft_forward(h, ref, n, np.zeros(n, np.float32))
        R.ref_srfft_free(h)
        assert np.array_equal(bits(ours), bits(ref))


def _kaldi(name):
    return np.loadtxt(os.path.join(GOLDEN, name), dtype=np.float64).reshape(-1, 40)


def test_fbank_vs_kaldi_dump(oracle):
    # test/fbank_test.cc:24-60: 47 x 40 values, |d| < 1e-4
    w = oracle.read_wav(os.path.join(GOLDEN, "en-us-hello.wav"))
    assert len(w) == 7802
    f = oracle.Fbank().compute(w)
    k = _kaldi("fbankmat_en-us-hello.wav.txt")
    assert f.shape == (47, 40) and k.size == 1880
    assert np.abs(f - k).max() < 1e-4


def test_fbank_streaming_equals_oneshot(oracle):
    # test/fbank_test.cc:85-136 feeds 1024-byte chunks; Fbank::Process keeps
    # samples from 160*T on (fbank.cc:306-313), so the frame sequence must be
    # identical to one-shot.  Checked here by re-framing per chunk.
    w = oracle.read_wav(os.path.join(GOLDEN, "en-us-hello.wav"))
    fb = oracle.Fbank()
    oneshot = fb.compute(w)
    buf = np.zeros(0, np.float32)
    rows = []
    for s in range(0, len(w), 512):  # 1024 bytes = 512 int16 samples
        buf = np.concatenate([buf, w[s:s + 512]])
        t = fb.num_frames(len(buf))
        if t:
            rows.append(fb.compute(buf[:(t - 1) * 160 + 400]))
            buf = buf[160 * t:]
    assert np.array_equal(bits(np.concatenate(rows)), bits(oneshot))


def test_cmvn_vs_kaldi_dump(oracle, global_stats):
    # test/cmvn_test.cc:55-76 (made two-sided): apply-cmvn-online dump
    assert global_stats.shape == (41,) and global_stats[40] == 36162480.0
    w = oracle.read_wav(os.path.join(GOLDEN, "en-us-hello.wav"))
    f = oracle.Fbank().compute(w)
    c = oracle.cmvn(global_stats, f)
    k = _kaldi("fbankcmvnmat_en-us-hello.wav.txt")
    assert np.abs(c - k).max() < 1e-4


def test_nnet_layer_kats(oracle):
    kat = json.load(open(os.path.join(GOLDEN, "nnet_kat.json")))
    tol = kat["tol"]
    # LinearLayer(W[out x in], b) stores W^T (nnet.cc:11-20)
    L = kat["linear"]
    W = np.array(L["W_out_by_in"], np.float32).reshape(L["shape"])
    y = oracle.layer_forward({"kind": "linear", "W": W.T.copy(), "b": np.array(L["b"], np.float32)},
                             np.array([L["x"]], np.float32))
    assert np.abs(y[0] - L["y"]).max() < tol
    for name in ("softmax", "relu"):
        y = oracle.layer_forward({"kind": name}, np.array([kat[name]["x"]], np.float32))
        assert np.abs(y[0] - kat[name]["y"]).max() < tol
    L = kat["log_softmax"]
    y = oracle.layer_forward({"kind": "log_softmax"}, np.array(L["x"], np.float32).reshape(L["shape"]))
    assert np.abs(y - np.array(L["y"])).max() < tol
    y = oracle.layer_forward({"kind": "normalize"}, np.array([kat["normalize"]["x"]], np.float32))
    assert abs(float((y.astype(np.float64) ** 2).sum()) - 4.0) < kat["normalize"]["tol"]
    L = kat["splice"]
    y = oracle.layer_forward({"kind": "splice", "indices": L["indices"]},
                             np.array(L["x"], np.float32).reshape(L["shape"]))
    assert np.abs(y - np.array(L["y"])).max() < tol
    L = kat["batchnorm"]
    y = oracle.layer_forward({"kind": "batchnorm", "scale": np.array(L["scale"], np.float32),
                              "offset": np.array(L["offset"], np.float32)},
                             np.array(L["x"], np.float32).reshape(L["shape"]))
    assert np.abs(y - np.array(L["y"])).max() < tol
    L = kat["narrow"]
    x = np.array(L["x"], np.float32).reshape(L["shape"])
    lay = {"kind": "narrow", "left": L["left"], "right": L["right"]}
    assert np.abs(oracle.layer_forward(lay, x) - np.array(L["y_full"])).max() < tol
    y = oracle.layer_forward(lay, x[:L["y_small_rows"]])
    assert np.abs(y - np.array(L["y_small"])).max() < tol


def test_am_chunking_invariance(oracle, xs_config):
    # AM output does not depend on chunk_size because every Splice
    # is followed by the Narrow that drops its clamped rows; the GPU's
    # whole-utterance batching relies on it.
    from catears_amd import formats, synth
    am = formats.read_am(xs_config)
    f = oracle.Fbank().compute(synth.pcm(3, 16000 + 123))
    a = oracle.am_stream(am, f, chunk_size=50)
    b = oracle.am_stream(am, f, chunk_size=7)
    c = oracle.am_whole(am, f)
    assert a.shape == (len(f), 512)
    assert np.array_equal(bits(a), bits(b)) and np.array_equal(bits(a), bits(c))


def test_am_short_utterances(oracle, xs_config):
    from catears_amd import formats, synth
    am = formats.read_am(xs_config)
    f = oracle.Fbank().compute(synth.pcm(4, 16000))
    for t in (0, 1, 2, 5):
        a = oracle.am_stream(am, f[:t], chunk_size=50)
        assert a.shape == (t, 512)
        if t:
            assert np.array_equal(bits(a), bits(oracle.am_whole(am, f[:t])))


@pytest.mark.parametrize("shape", [(5, 3, 2), (100, 100, 1), (121, 233, 17), (64, 96, 300)])
def test_u8_gemm_bitexact_vs_gemmlowp(oracle, shape):
    # test/gemm_test.cc:86-89 shapes; gemmlowp compiled from the reference
    R = oracle.ref_lib()
    if R is None:
        pytest.skip("oracle/_ref not built (reference absent)")
    m, n, k = shape
    rng = np.random.default_rng(m * 7 + n)
    A = rng.uniform(-0.5, 0.5, (m, k)).astype(np.float32)
    B = rng.uniform(1, 2, (k, n)).astype(np.float32)
    qa, sa, za = oracle.quantize(A)
    qb, sb, zb = oracle.quantize(B)
    ours = oracle.gemm_u8u8f32(qa, sa, za, qb, sb, zb)
    ref = np.zeros((m, n), np.float32)
    R.ref_gemm_u8u8f32(m, n, k, qa, sa, za, qb, sb, zb, ref)
    assert np.array_equal(bits(ours), bits(ref))
    # gemm_test.cc:104,120 properties
    exact = A.astype(np.float64) @ B.astype(np.float64)
    assert np.abs(oracle.sgemm(A, B) - exact).max() < 1e-2
    assert np.abs(ours - exact).max() / (ours.max() - ours.min()) < 0.01


def test_quantize_reference_quirks(oracle):
    # max starts at FLT_MIN (matrix.cc:332): an all-negative matrix keeps
    # max = FLT_MIN; the zero point is not clamped.
    x = -np.linspace(1, 2, 12, dtype=np.float32)
    q, s, z = oracle.quantize(x)
    assert np.isclose(s, (np.finfo(np.float32).tiny + 2.0) / 255.0)
    assert z == int(np.round(2.0 / ((np.finfo(np.float32).tiny + 2.0) / 255.0)))
    x = np.linspace(1, 2, 12, dtype=np.float32)
    q, s, z = oracle.quantize(x)
    assert z < 0 and q.min() == 0 and q.max() == 255
