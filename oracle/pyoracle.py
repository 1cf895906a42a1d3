"""ctypes front-end of the C oracle (oracle/oracle.c).  TEST INFRASTRUCTURE ONLY.

Besides thin wrappers this module composes the reference's per-frame
AcousticModel streaming (src/am.cc:115-164) out of the oracle's layer functions,
so the GPU whole-utterance path is checked against the chunked reference
semantics, not against a re-derivation of it.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")


def lib():
    """Load oracle/liboracle.so (built by oracle/Makefile)."""
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = ctypes.CDLL(path)
        vp, ci, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
        L.orc_srfft_new.restype = vp
        L.orc_srfft_new.argtypes = [ci]
        L.orc_srfft_free.argtypes = [vp]
        L.orc_srfft_forward.argtypes = [vp, f32p, f32p]
        L.orc_fbank_new.restype = vp
        L.orc_fbank_free.argtypes = [vp]
        L.orc_fbank_window.restype = ctypes.POINTER(ctypes.c_float)
        L.orc_fbank_window.argtypes = [vp]
        L.orc_fbank_mel.restype = ci
        L.orc_fbank_mel.argtypes = [vp, ci, f32p, ctypes.POINTER(ci)]
        L.orc_fbank_num_frames.restype = ci
        L.orc_fbank_num_frames.argtypes = [cl]
        L.orc_fbank_compute.restype = ci
        L.orc_fbank_compute.argtypes = [vp, f32p, cl, f32p, vp]
        L.orc_cmvn.argtypes = [f32p, f32p, ci, f32p]
        L.orc_sgemm.argtypes = [ci, ci, ci, f32p, ci, f32p, ci, f32p, ci]
        L.orc_linear.argtypes = [ci, ci, ci, f32p, f32p, f32p, f32p]
        L.orc_splice.argtypes = [ci, ci, f32p, ci, i32p, f32p]
        L.orc_relu.argtypes = [cl, f32p]
        L.orc_batchnorm.argtypes = [ci, ci, f32p, f32p, f32p]
        L.orc_log_softmax.argtypes = [ci, ci, f32p]
        L.orc_softmax.argtypes = [ci, ci, f32p]
        L.orc_normalize.argtypes = [ci, ci, f32p]
        L.orc_quant_params.argtypes = [cl, f32p, ctypes.POINTER(ctypes.c_float),
                                       ctypes.POINTER(ctypes.c_int32)]
        L.orc_quantize.argtypes = [cl, f32p, u8p, ctypes.POINTER(ctypes.c_float),
                                   ctypes.POINTER(ctypes.c_int32)]
        L.orc_quantize_apply.argtypes = [cl, f32p, ctypes.c_float, ctypes.c_int32, u8p]
        L.orc_gemm_u8u8_i32.argtypes = [ci, ci, ci, u8p, ctypes.c_int32, u8p, ctypes.c_int32, i32p]
        L.orc_gemm_u8u8f32.argtypes = [ci, ci, ci, u8p, ctypes.c_float, ctypes.c_int32,
                                       u8p, ctypes.c_float, ctypes.c_int32, f32p]
        _LIB = L
    return _LIB


def ref_lib():
    """oracle/_ref/libref.so (reference srfft.cc + gemmlowp), or None."""
    global _REF
    if _REF is None:
        path = os.path.join(HERE, "_ref", "libref.so")
        if not os.path.exists(path):
            return None
        R = ctypes.CDLL(path)
        R.ref_srfft_new.restype = ctypes.c_void_p
        R.ref_srfft_new.argtypes = [ctypes.c_int]
        R.ref_srfft_free.argtypes = [ctypes.c_void_p]
        R.ref_srfft_forward.argtypes = [ctypes.c_void_p, f32p, ctypes.c_int, f32p]
        R.ref_gemm_u8u8f32.argtypes = [ctypes.c_int] * 3 + [u8p, ctypes.c_float, ctypes.c_int32,
                                                             u8p, ctypes.c_float, ctypes.c_int32, f32p]
        _REF = R
    return _REF


# ---------------------------------------------------------------- signal --

def srfft_forward(x):
    x = np.ascontiguousarray(x, np.float32).copy()
    L = lib()
    h = L.orc_srfft_new(len(x))
    try:
        L.orc_srfft_forward(h, x, np.zeros(len(x), np.float32))
    finally:
        L.orc_srfft_free(h)
    return x


class Fbank:
    """Whole-utterance Fbank::Process (src/fbank.cc:265-314)."""

    def __init__(self):
        self._h = lib().orc_fbank_new()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_fbank_free(self._h)
            self._h = None

    @staticmethod
    def num_frames(n):
        return lib().orc_fbank_num_frames(int(n))

    def window(self):
        p = lib().orc_fbank_window(self._h)
        return np.ctypeslib.as_array(p, shape=(400,)).copy()

    def mel_table(self):
        out = []
        for b in range(40):
            w = np.zeros(256, np.float32)
            off = ctypes.c_int()
            n = lib().orc_fbank_mel(self._h, b, w, ctypes.byref(off))
            out.append((off.value, w[:n].copy()))
        return out

    def compute(self, wave, with_mel=False):
        wave = np.ascontiguousarray(wave, np.float32)
        t = self.num_frames(len(wave))
        feats = np.zeros((max(t, 0), 40), np.float32)
        mel = np.zeros((max(t, 0), 40), np.float32) if with_mel else None
        if t > 0:
            lib().orc_fbank_compute(self._h, wave, len(wave), feats,
                                    mel.ctypes.data_as(ctypes.c_void_p) if with_mel else None)
        return (feats, mel) if with_mel else feats


def fbank_f64(wave):
    """Fbank::Process in float64 with an exact FFT (numpy): the reference's
    algorithm (src/fbank.cc:44-245) without its fp32 rounding -- DC removal,
    pre-emphasis, the reference's own Hamming window and mel triangles (from
    the oracle's tables), |rfft|^2, mel dots, floor, log.  The yardstick for
    how far an fp32 fbank (the reference's split-radix order, or the GPU's
    fast mode) is from the exact result."""
    fb = Fbank()
    win = fb.window().astype(np.float64)
    mel = fb.mel_table()
    w = np.asarray(wave, np.float64)
    t = Fbank.num_frames(len(w))
    out = np.zeros((max(t, 0), 40))
    eps = float(np.finfo(np.float32).eps)
    for i in range(t):
        x = w[160 * i:160 * i + 400].copy()
        x -= x.sum() / 400.0
        y = x.copy()
        y[1:] = x[1:] - 0.97 * x[:-1]
        y[0] = x[0] - 0.97 * x[0]
        p = np.abs(np.fft.rfft(np.concatenate([y * win, np.zeros(112)]))) ** 2
        for b, (off, wt) in enumerate(mel):
            out[i, b] = np.log(max(float(np.dot(wt.astype(np.float64), p[off:off + len(wt)])), eps))
    return out


def cmvn(global_stats, feats):
    """Online CMVN over a whole utterance (src/cmvn.cc:100-110 called 0..T-1)."""
    feats = np.ascontiguousarray(feats, np.float32)
    out = np.zeros_like(feats)
    if len(feats):
        lib().orc_cmvn(np.ascontiguousarray(global_stats, np.float32), feats, len(feats), out)
    return out


# ------------------------------------------------------------------ nnet --

def sgemm(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    m, k = a.shape
    n = b.shape[1]
    c = np.zeros((m, n), np.float32)
    lib().orc_sgemm(m, n, k, a, k, b, n, c, n)
    return c


def layer_forward(layer, x, gemm=None):
    """One reference layer's Propagate (src/nnet.cc).  `layer` is a dict as
    produced by catears_amd.model.read_nnet (kind + params)."""
    L = lib()
    kind = layer["kind"]
    x = np.ascontiguousarray(x, np.float32)
    rows = x.shape[0]
    if kind == "linear":
        W, b = layer["W"], layer["b"]  # W: in x out (MAT0 layout)
        if gemm is None:
            y = np.zeros((rows, W.shape[1]), np.float32)
            L.orc_linear(rows, W.shape[0], W.shape[1], x, np.ascontiguousarray(W, np.float32),
                         np.ascontiguousarray(b, np.float32), y)
        else:
            y = gemm(x, W)
            y += b[None, :]
        return y
    if kind == "splice":
        if rows == 0 or x.shape[1] == 0:
            return x  # nnet.cc:55 returns early
        idx = np.asarray(layer["indices"], np.int32)
        y = np.zeros((rows, x.shape[1] * len(idx)), np.float32)
        L.orc_splice(rows, x.shape[1], x, len(idx), idx, y)
        return y
    if kind == "narrow":
        l, r = layer["left"], layer["right"]
        if rows <= l + r:
            return x.copy()
        return x[l:rows - r].copy()
    y = x.copy()
    if kind == "relu":
        L.orc_relu(y.size, y)
    elif kind == "batchnorm":
        L.orc_batchnorm(rows, y.shape[1], y, np.ascontiguousarray(layer["scale"], np.float32),
                        np.ascontiguousarray(layer["offset"], np.float32))
    elif kind == "log_softmax":
        L.orc_log_softmax(rows, y.shape[1], y)
    elif kind == "softmax":
        L.orc_softmax(rows, y.shape[1], y)
    elif kind == "normalize":
        L.orc_normalize(rows, y.shape[1], y)
    else:
        raise ValueError(kind)
    return y


def nnet_propagate(layers, x, gemm=None):
    """Nnet::Propagate (src/nnet.cc:295-307)."""
    for layer in layers:
        x = layer_forward(layer, x, gemm)
    return x


def gemm_u8u8f32_f64(a, sa, zpa, b, sb, zpb):
    """gemm_u8u8f32 (orc_gemm_u8u8f32) for operands too large for its scalar
    loop: each zero-point-shifted product is an integer of magnitude at most
    255^2, so while k * 255^2 < 2^31 the int32 accumulator never wraps and a
    float64 matmul (every partial sum an integer below 2^53) computes it
    exactly; the float stage is the same float(acc) * (sa * sb) in float32
    (an exact integer rounded float64 -> float32 is the int32 -> float
    conversion, both round to nearest even)."""
    k = a.shape[1]
    assert k * 255 * 255 < 2 ** 31, "accumulator could wrap: use gemm_u8u8f32"
    acc = (a.astype(np.float64) - zpa) @ (b.astype(np.float64) - zpb)
    s = np.float32(np.float32(sa) * np.float32(sb))
    return (acc.astype(np.float32) * s).astype(np.float32)


def nnet_propagate_int8(layers, x, exact_f64=False):
    """Nnet::Propagate with every LinearLayer as Quantize + MatMat_U8U8F32 +
    bias (src/matrix.cc:329-420) -- the int8 path of BASELINE config C5, as
    catears_amd runs it (include/catears_gpu.h ce_gpu_model_quantize): the
    activation parameters come from the block entering the Splice (equal to
    those of the spliced block, whose rows it all reads), weights per tensor.
    exact_f64: the u8 GEMMs through gemm_u8u8f32_f64 (same bits, BLAS speed:
    C5-sized blocks)."""
    x = np.ascontiguousarray(x, np.float32)
    pre = None  # block entering the pending Splice
    for layer in layers:
        kind = layer["kind"]
        if kind == "splice":
            pre = x
            x = layer_forward(layer, x)
        elif kind == "linear":
            src = pre if pre is not None else x
            _, sx, zx = quantize(src)
            xq = _quantize_with(x, sx, zx)
            wq, sw, zw = quantize(layer["W"])
            y = (gemm_u8u8f32_f64 if exact_f64 else gemm_u8u8f32)(xq, sx, zx, wq, sw, zw)
            x = (y + np.asarray(layer["b"], np.float32)[None, :]).astype(np.float32)
            pre = None
        else:
            x = layer_forward(layer, x)
            if kind != "narrow":
                pre = None
    return x


def _quantize_with(x, scale, zp):
    """Quantize's elementwise step with given parameters (matrix.cc:378-386)."""
    x = np.ascontiguousarray(x, np.float32)
    q = np.zeros(x.shape, np.uint8)
    if x.size:
        lib().orc_quantize_apply(x.size, x.reshape(-1), scale, zp, q.reshape(-1))
    return q


def am_stream(model, feats, chunk_size=50, gemm=None):
    """AcousticModel::Process per frame + EndOfStream (src/am.cc:115-164).
    `model` has layers, log_prior, left, right.  Returns T x num_pdfs."""
    L, R = model["left"], model["right"]
    buf = []
    outs = []

    def batch(n):
        inp = np.stack(buf[:n + L + R]).astype(np.float32)
        y = nnet_propagate(model["layers"], inp, gemm)
        assert y.shape[0] == n, (y.shape, n)
        return y - model["log_prior"][None, :]  # AddVec(-1.0f): exact negation

    started = False
    for t in range(len(feats)):
        f = feats[t]
        if not started:
            buf.extend([f] * L)
            started = True
        buf.append(f)
        if len(buf) >= L + R + chunk_size:
            outs.append(batch(chunk_size))
            del buf[:chunk_size]
    if buf:
        buf.extend([buf[-1]] * R)
        if len(buf) > L + R:
            outs.append(batch(len(buf) - L - R))
    if not outs:
        return np.zeros((0, model["log_prior"].shape[0]), np.float32)
    return np.concatenate(outs, 0)


def am_whole(model, feats, gemm=None):
    """Whole-utterance equivalent of am_stream: pad L copies of the first frame
    and R of the last, one Propagate (verified equal to am_stream in tests)."""
    L, R = model["left"], model["right"]
    if len(feats) == 0:
        return np.zeros((0, model["log_prior"].shape[0]), np.float32)
    x = np.concatenate([np.repeat(feats[:1], L, 0), feats, np.repeat(feats[-1:], R, 0)], 0)
    y = nnet_propagate(model["layers"], x, gemm)
    return y - model["log_prior"][None, :]


# ------------------------------------------------------------------ int8 --

def quantize(x):
    x = np.ascontiguousarray(x, np.float32)
    q = np.zeros(x.shape, np.uint8)
    s, z = ctypes.c_float(), ctypes.c_int32()
    lib().orc_quantize(x.size, x.reshape(-1), q.reshape(-1), ctypes.byref(s), ctypes.byref(z))
    return q, s.value, z.value


def gemm_u8u8_i32(a, zpa, b, zpb):
    m, k = a.shape
    n = b.shape[1]
    c = np.zeros((m, n), np.int32)
    lib().orc_gemm_u8u8_i32(m, n, k, np.ascontiguousarray(a), zpa, np.ascontiguousarray(b), zpb, c)
    return c


def gemm_u8u8f32(a, sa, zpa, b, sb, zpb):
    m, k = a.shape
    n = b.shape[1]
    c = np.zeros((m, n), np.float32)
    lib().orc_gemm_u8u8f32(m, n, k, np.ascontiguousarray(a), sa, zpa, np.ascontiguousarray(b), sb,
                           zpb, c)
    return c


# --------------------------------------------------------------- decoder --

def decoder_loglikelihood(frame_logp, tid2pdf, rows, trans, am_scale):
    """Decoder::LogLikelihood (src/decoder.cc:97-102): am_scale * frame_logp[
    tid2pdf[trans_id]], a float32 product, for each (frame row, transition
    id) pair: frame_logp is (frames x pdfs), rows / trans index arrays."""
    pdf = np.asarray(tid2pdf, np.int32)[np.asarray(trans)]
    return (np.float32(am_scale) * np.asarray(frame_logp, np.float32)[np.asarray(rows), pdf]).astype(np.float32)


# ------------------------------------------------------------------- wav --

def read_wav(path):
    """Read16kPcm (src/pcm_reader.cc:194-211): RIFF/WAVE, 16-byte fmt chunk,
    PCM, mono 16 kHz, 8/16/32-bit samples converted at raw scale (no /32768).
    The data chunk is taken as file_size - 44 bytes (pcm_reader.cc:204)."""
    import struct
    raw = open(path, "rb").read()
    if raw[0:4] != b"RIFF" or raw[8:12] != b"WAVE" or raw[12:16] != b"fmt ":
        raise ValueError("not a RIFF/WAVE file")
    (sub1,) = struct.unpack("<i", raw[16:20])
    fmt, ch, sr, byte_rate, align, bits = struct.unpack("<hhiihh", raw[20:36])
    if sub1 != 16 or fmt != 1:
        raise ValueError("unsupported fmt chunk")
    if ch != 1 or sr != 16000 or bits not in (8, 16, 32):
        raise ValueError("unsupported format")
    if raw[36:40] != b"data":
        raise ValueError("missing data chunk")
    body = raw[44:]
    dt = {8: np.int8, 16: np.int16, 32: np.int32}[bits]
    n = len(body) // (bits // 8)
    return np.frombuffer(body[:n * (bits // 8)], dtype=dt).astype(np.float32)
