"""ctypes binding of libcatears_hip.so (include/catears_gpu.h).

This is the Python side of the drop-in boundary: the same C-ABI a C++ host
(the reference's ce_stt.cc) links against.  Device memory and streams come
from PyTorch (plumbing only); every compute call goes through the HIP library.
There is no CPU fallback: if the library or a GPU is missing, calls raise.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# CATEARS_HIP_LIB: development override (e.g. an instrumented build)
LIB_PATH = os.environ.get("CATEARS_HIP_LIB") or os.path.join(HERE, "lib", "libcatears_hip.so")

CE_GPU_OK = 0
ERRORS = {-2: "EINVAL", -3: "EHIP", -4: "EIO", -5: "ECORRUPT", -6: "ENOTSUP", -7: "ENOMEM"}

# Every symbol include/catears_gpu.h declares (checked by tests).
ABI = [
    "ce_gpu_last_error", "ce_gpu_version", "ce_gpu_ctx_create", "ce_gpu_ctx_destroy",
    "ce_gpu_ctx_set_stream", "ce_gpu_ctx_synchronize", "ce_gpu_ctx_profile", "ce_gpu_ctx_profile_classes",
    "ce_gpu_ctx_profile_read", "ce_gpu_model_load_config",
    "ce_gpu_model_load", "ce_gpu_model_info", "ce_gpu_model_tid2pdf", "ce_gpu_model_destroy",
    "ce_gpu_fbank_num_frames", "ce_gpu_plan_create", "ce_gpu_plan_info",
    "ce_gpu_plan_frame_offsets", "ce_gpu_plan_destroy", "ce_gpu_fbank", "ce_gpu_cmvn",
    "ce_gpu_am_forward", "ce_gpu_score", "ce_gpu_sgemm", "ce_gpu_quantize",
    "ce_gpu_gemm_u8u8f32", "ce_gpu_gemm_u8u8i32", "ce_gpu_model_load_mem",
    "ce_gpu_nnet_propagate", "ce_gpu_linear", "ce_gpu_splice", "ce_gpu_rowwise",
    "ce_gpu_profile_anchor", "ce_gpu_ctx_profile_intervals", "ce_gpu_model_quantize",
    "ce_gpu_nnet_propagate_blocks", "ce_gpu_loglik_gather", "ce_gpu_loglik_columns",
    "ce_gpu_model_set_gemm", "ce_gpu_model_get_gemm", "ce_gpu_ctx_overflow", "ce_gpu_ctx_set_latency",
    "ce_gpu_fbank_s16", "ce_gpu_score_s16", "ce_gpu_ctx_set_fbank", "ce_gpu_sum_f64", "ce_gpu_ctx_set_wide_tiles",
    "ce_gpu_sum_f64_many", "ce_gpu_trace_mark", "ce_gpu_nnet_check_mem",
]

# ce_gpu_model_set_gemm modes
GEMM_MODES = {"fp32": 0, "bf16x6": 1, "f16x3": 2, "bf16x6p": 3}

_lib = None


class CatearsError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def lib():
    """Load the HIP library; raises ImportError if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: build it with `make` (hipcc, gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    vp, ci, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    pp = ctypes.POINTER(ctypes.c_void_p)
    pi, pi64 = ctypes.POINTER(ci), ctypes.POINTER(i64)
    sig = {
        "ce_gpu_last_error": (ctypes.c_char_p, []),
        "ce_gpu_version": (ctypes.c_char_p, []),
        "ce_gpu_ctx_create": (ci, [ci, vp, pp]),
        "ce_gpu_ctx_destroy": (ci, [vp]),
        "ce_gpu_ctx_set_stream": (ci, [vp, vp]),
        "ce_gpu_ctx_synchronize": (ci, [vp]),
        "ce_gpu_ctx_profile": (ci, [vp, ci]),
        "ce_gpu_ctx_profile_classes": (ci, [vp, ctypes.c_uint]),
        "ce_gpu_ctx_profile_read": (ci, [vp, ci, ctypes.POINTER(ctypes.c_double), pi64]),
        "ce_gpu_model_load_config": (ci, [vp, ctypes.c_char_p, pp]),
        "ce_gpu_model_load": (ci, [vp, ctypes.c_char_p, ctypes.c_char_p, ci, ci, pp]),
        "ce_gpu_model_info": (ci, [vp, pi, pi, pi, pi, pi, pi64]),
        "ce_gpu_model_tid2pdf": (ci, [vp, ctypes.POINTER(ctypes.c_int32), ci, pi]),
        "ce_gpu_model_destroy": (ci, [vp]),
        "ce_gpu_fbank_num_frames": (i64, [i64]),
        "ce_gpu_plan_create": (ci, [vp, vp, pi64, ci, ci, pp]),
        "ce_gpu_plan_info": (ci, [vp, pi, pi64, pi64, pi, pi]),
        "ce_gpu_plan_frame_offsets": (ci, [vp, pi64]),
        "ce_gpu_plan_destroy": (ci, [vp]),
        "ce_gpu_fbank": (ci, [vp, vp, vp, vp, vp]),
        "ce_gpu_fbank_s16": (ci, [vp, vp, vp, vp, vp]),
        "ce_gpu_cmvn": (ci, [vp, vp, vp, vp, vp]),
        "ce_gpu_am_forward": (ci, [vp, vp, vp, vp, vp]),
        "ce_gpu_score": (ci, [vp, vp, vp, vp, vp, vp, vp]),
        "ce_gpu_score_s16": (ci, [vp, vp, vp, vp, vp, vp, vp]),
        "ce_gpu_sgemm": (ci, [vp, ci, ci, ci, vp, ci, vp, ci, vp, ci]),
        "ce_gpu_quantize": (ci, [vp, vp, i64, vp, vp]),
        "ce_gpu_gemm_u8u8f32": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, vp]),
        "ce_gpu_gemm_u8u8i32": (ci, [vp, ci, ci, ci, vp, vp, vp, vp, vp]),
        "ce_gpu_profile_anchor": (ci, [ci, vp]),
        "ce_gpu_trace_mark": (ci, [ci, vp, ci]),
        "ce_gpu_nnet_check_mem": (ci, [vp, i64, pi, pi, pi]),
        "ce_gpu_model_quantize": (ci, [vp, vp]),
        "ce_gpu_nnet_propagate_blocks": (ci, [vp, vp, vp, ci, ctypes.POINTER(ctypes.c_int32), ci, ci, vp]),
        "ce_gpu_ctx_profile_intervals": (ci, [vp, ci, vp, vp, ci, pi]),
        "ce_gpu_model_load_mem": (ci, [vp, vp, i64, vp, ci, ci, ci, pp]),
        "ce_gpu_nnet_propagate": (ci, [vp, vp, vp, ci, ci, ci, vp]),
        "ce_gpu_linear": (ci, [vp, ci, ci, ci, vp, ci, vp, ci, vp, vp, ci]),
        "ce_gpu_splice": (ci, [vp, ci, ci, vp, ci, ctypes.POINTER(ctypes.c_int32), ci, vp]),
        "ce_gpu_rowwise": (ci, [vp, ci, ci, ci, vp, ci, vp, vp]),
        "ce_gpu_loglik_gather": (ci, [vp, vp, ci, ci, ci, vp, ci, vp, vp, ci, ctypes.c_float, vp]),
        "ce_gpu_loglik_columns": (ci, [vp, vp, ci, ci, ci, vp, ci, vp]),
        "ce_gpu_model_set_gemm": (ci, [vp, ci]),
        "ce_gpu_model_get_gemm": (ci, [vp, pi]),
        "ce_gpu_ctx_overflow": (ci, [vp, pi]),
        "ce_gpu_ctx_set_latency": (ci, [vp, ci]),
        "ce_gpu_ctx_set_fbank": (ci, [vp, ci]),
        "ce_gpu_ctx_set_wide_tiles": (ci, [vp, ci]),
        "ce_gpu_sum_f64": (ci, [vp, vp, i64, vp, vp]),
        "ce_gpu_sum_f64_many": (ci, [vp, ci, ctypes.POINTER(vp), pi64, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc):
    if rc != CE_GPU_OK:
        raise CatearsError(rc, lib().ce_gpu_last_error().decode())
    return rc


def _ptr(t):
    """Device pointer of a torch tensor (or None)."""
    if t is None:
        return None
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError("expected a contiguous device tensor")
    return ctypes.c_void_p(t.data_ptr())


class Context:
    """One device + one stream (defaults to torch's current stream)."""

    def __init__(self, device=0, stream=None):
        import torch
        self.device = device
        self._torch_stream = stream if stream is not None else torch.cuda.current_stream(device)
        h = ctypes.c_void_p()
        check(lib().ce_gpu_ctx_create(device, ctypes.c_void_p(self._torch_stream.cuda_stream),
                                      ctypes.byref(h)))
        self.h = h

    def set_stream(self, stream):
        self._torch_stream = stream
        check(lib().ce_gpu_ctx_set_stream(self.h, ctypes.c_void_p(stream.cuda_stream)))

    def synchronize(self):
        check(lib().ce_gpu_ctx_synchronize(self.h))

    def set_latency(self, on=True):
        """Latency mode (ce_gpu_ctx_set_latency): split-K nnet GEMMs for small
        row blocks scored one at a time."""
        check(lib().ce_gpu_ctx_set_latency(self.h, int(bool(on))))

    FBANK_MODES = {"exact": 0, "fast": 1}

    def set_wide_tiles(self, on=True):
        """128 x 128 bf16x6 tiles for every layer (ce_gpu_ctx_set_wide_tiles):
        all CUs per launch, for a batch scored while no other is in flight.
        Same bits as the default tiles."""
        check(lib().ce_gpu_ctx_set_wide_tiles(self.h, int(bool(on))))

    def set_fbank(self, mode="exact"):
        """Fbank kernel of this context (ce_gpu_ctx_set_fbank): "exact" (the
        reference's operation order, bit-exact pre-log energies) or "fast"
        (the same lane program with FMA contraction, ~12 % faster; as close
        to the exact result as the reference's own fp32 order,
        tests/test_gpu_fbank_fast.py)."""
        check(lib().ce_gpu_ctx_set_fbank(self.h, self.FBANK_MODES[mode]))

    def overflow(self):
        """True if an f16x3 GEMM met an out-of-range activation since the
        last call (synchronizes; ce_gpu_ctx_overflow)."""
        v = ctypes.c_int()
        check(lib().ce_gpu_ctx_overflow(self.h, ctypes.byref(v)))
        return bool(v.value)

    PROF_GEMM, PROF_GEMM_GATHER, PROF_FBANK, PROF_CMVN, PROF_FINALIZE, PROF_QUANT = range(6)

    def profile(self, enable=True, classes=None):
        """Time launches (HIP events); `classes`: iterable of PROF_* to time
        (default all)."""
        mask = 0xffffffff if classes is None else sum(1 << c for c in classes)
        check(lib().ce_gpu_ctx_profile_classes(self.h, mask))
        check(lib().ce_gpu_ctx_profile(self.h, int(enable)))

    def profile_read(self, cls):
        """(total_ms, launches) of a kernel class since the last read."""
        ms, n = ctypes.c_double(), ctypes.c_int64()
        check(lib().ce_gpu_ctx_profile_read(self.h, cls, ctypes.byref(ms), ctypes.byref(n)))
        return ms.value, n.value

    def profile_intervals(self, cls):
        """[(start_ms, end_ms)] after the last profile_anchor(), per launch of a class."""
        n = ctypes.c_int()
        rc = lib().ce_gpu_ctx_profile_intervals(self.h, cls, None, None, 0, ctypes.byref(n))
        if rc != CE_GPU_OK and n.value == 0:
            check(rc)
        a = np.zeros(max(n.value, 1), np.float64)
        b = np.zeros_like(a)
        check(lib().ce_gpu_ctx_profile_intervals(self.h, cls, a.ctypes.data_as(ctypes.c_void_p),
                                                 b.ctypes.data_as(ctypes.c_void_p), len(a), ctypes.byref(n)))
        return list(zip(a[:n.value], b[:n.value]))

    def close(self):
        if getattr(self, "h", None):
            lib().ce_gpu_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Model:
    """config_path | (nnet, prior, left, right) files | image= NN02 bytes
    (+ optional prior probabilities, left/right default to the network's)."""

    def __init__(self, ctx, config_path=None, nnet=None, prior=None, left=None, right=None, image=None):
        h = ctypes.c_void_p()
        if config_path is not None:
            check(lib().ce_gpu_model_load_config(ctx.h, config_path.encode(), ctypes.byref(h)))
        elif image is not None:
            pr = None if prior is None else np.ascontiguousarray(prior, np.float32)
            buf = ctypes.create_string_buffer(bytes(image), len(image))
            check(lib().ce_gpu_model_load_mem(
                ctx.h, buf, len(image), None if pr is None else pr.ctypes.data_as(ctypes.c_void_p),
                0 if pr is None else pr.size, -1 if left is None else left, -1 if right is None else right,
                ctypes.byref(h)))
        else:
            check(lib().ce_gpu_model_load(ctx.h, nnet.encode(), prior.encode(), left, right,
                                          ctypes.byref(h)))
        self.h = h
        v = [ctypes.c_int() for _ in range(5)]
        p = ctypes.c_int64()
        check(lib().ce_gpu_model_info(h, *[ctypes.byref(x) for x in v], ctypes.byref(p)))
        self.left, self.right, self.input_dim, self.num_pdfs, self.num_linear = [x.value for x in v]
        self.num_params = p.value

    def quantize(self, ctx):
        """Switch to the int8 path (ce_gpu_model_quantize)."""
        check(lib().ce_gpu_model_quantize(ctx.h, self.h))
        return self

    def set_gemm(self, mode):
        """Matrix-core form of the fp32 Linear layers: "fp32" (fp32 MFMA),
        "bf16x6" (three-plane bf16 split on the way into LDS, six products),
        "bf16x6p" (the same with the planes stored in HBM; bit-identical) or
        "f16x3" (two scaled fp16 planes, three products);
        ce_gpu_model_set_gemm."""
        check(lib().ce_gpu_model_set_gemm(self.h, GEMM_MODES[mode]))
        return self

    @property
    def gemm(self):
        v = ctypes.c_int()
        check(lib().ce_gpu_model_get_gemm(self.h, ctypes.byref(v)))
        return {b: a for a, b in GEMM_MODES.items()}[v.value]

    def tid2pdf(self):
        n = ctypes.c_int()
        check(lib().ce_gpu_model_tid2pdf(self.h, None, 0, ctypes.byref(n)))
        out = np.zeros(n.value, np.int32)
        check(lib().ce_gpu_model_tid2pdf(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                         n.value, ctypes.byref(n)))
        return out

    def close(self):
        if getattr(self, "h", None):
            lib().ce_gpu_model_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def profile_anchor(device, stream):
    """Record the time origin for Context.profile_intervals on `stream`."""
    check(lib().ce_gpu_profile_anchor(device, ctypes.c_void_p(stream.cuda_stream)))


def nnet_check(image):
    """ce_gpu_nnet_check_mem: parse an NN02 image without a device; returns
    (num_layers, left, right) or raises CatearsError with the reference's
    message."""
    buf = bytes(image)
    n, l, r = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    check(lib().ce_gpu_nnet_check_mem(buf, len(buf), ctypes.byref(n), ctypes.byref(l), ctypes.byref(r)))
    return n.value, l.value, r.value


def trace_mark(device, stream, tag):
    """Launch the empty window-marker kernel with `tag` workgroups on `stream`
    (tools/trace_summary.py --window cuts a rocprofv3 kernel trace at it)."""
    check(lib().ce_gpu_trace_mark(device, ctypes.c_void_p(stream.cuda_stream), tag))


def union_ms(intervals):
    """Wall time covered by a set of (start, end) intervals."""
    total, cur_a, cur_b = 0.0, None, None
    for a, b in sorted(intervals):
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                total += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        total += cur_b - cur_a
    return total


def num_frames(n_samples):
    return lib().ce_gpu_fbank_num_frames(int(n_samples))


class Plan:
    def __init__(self, ctx, num_samples, model=None, max_rows=4096):
        ns = np.ascontiguousarray(num_samples, np.int64)
        h = ctypes.c_void_p()
        check(lib().ce_gpu_plan_create(ctx.h, model.h if model else None,
                                       ns.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                       len(ns), max_rows, ctypes.byref(h)))
        self.h = h
        a, d, e = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        b, c = ctypes.c_int64(), ctypes.c_int64()
        check(lib().ce_gpu_plan_info(h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c),
                                     ctypes.byref(d), ctypes.byref(e)))
        self.n_utt, self.total_samples, self.total_frames = a.value, b.value, c.value
        self.n_chunks, self.max_chunk_rows = d.value, e.value
        off = np.zeros(self.n_utt + 1, np.int64)
        check(lib().ce_gpu_plan_frame_offsets(h, off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))))
        self.frame_offsets = off

    def close(self):
        if getattr(self, "h", None):
            lib().ce_gpu_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fbank(ctx, plan, pcm, feats=None, mel=None):
    """Fbank::Process over the plan's utterances; `pcm` is float32 at raw
    int16 scale (ce_gpu_fbank) or int16 (ce_gpu_fbank_s16)."""
    import torch
    if feats is None:
        feats = torch.empty((plan.total_frames, 40), dtype=torch.float32, device=pcm.device)
    fn = lib().ce_gpu_fbank_s16 if pcm.dtype == torch.int16 else lib().ce_gpu_fbank
    if pcm.dtype not in (torch.int16, torch.float32):
        raise TypeError("pcm must be float32 or int16")
    check(fn(ctx.h, plan.h, _ptr(pcm), _ptr(feats), _ptr(mel)))
    return feats


def cmvn(ctx, plan, global_stats, feats, out=None):
    import torch
    if out is None:
        out = torch.empty_like(feats)
    check(lib().ce_gpu_cmvn(ctx.h, plan.h, _ptr(global_stats), _ptr(feats), _ptr(out)))
    return out


def am_forward(ctx, model, plan, feats, out=None):
    import torch
    if out is None:
        out = torch.empty((plan.total_frames, model.num_pdfs), dtype=torch.float32, device=feats.device)
    check(lib().ce_gpu_am_forward(ctx.h, model.h, plan.h, _ptr(feats), _ptr(out)))
    return out


def score(ctx, model, plan, pcm, global_stats=None, ws=None, out=None):
    import torch
    if ws is None:
        ws = torch.empty((2 * plan.total_frames * 40 + 1,), dtype=torch.float32, device=pcm.device)
    if out is None:
        out = torch.empty((plan.total_frames, model.num_pdfs), dtype=torch.float32, device=pcm.device)
    if pcm.dtype not in (torch.int16, torch.float32):
        raise TypeError("pcm must be float32 or int16")
    fn = lib().ce_gpu_score_s16 if pcm.dtype == torch.int16 else lib().ce_gpu_score
    check(fn(ctx.h, model.h, plan.h, _ptr(pcm), _ptr(global_stats), _ptr(ws), _ptr(out)))
    return out


def nnet_propagate(ctx, model, x, subtract_prior=False, out=None):
    """Nnet::Propagate on one padded block (+ the AM's prior subtraction)."""
    import torch
    net_l, net_r = model.left, model.right
    rows = x.shape[0]
    if out is None:
        out = torch.empty((max(rows - net_l - net_r, 0), model.num_pdfs), dtype=torch.float32, device=x.device)
    check(lib().ce_gpu_nnet_propagate(ctx.h, model.h, _ptr(x), rows, x.stride(0), int(subtract_prior), _ptr(out)))
    return out


def nnet_propagate_blocks(ctx, model, x, block_rows, subtract_prior=False, out=None):
    """ce_gpu_nnet_propagate_blocks: independent padded blocks back to back."""
    import torch
    rows = np.ascontiguousarray(block_rows, np.int32)
    n_out = int(rows.sum()) - len(rows) * (model.left + model.right)
    if out is None:
        out = torch.empty((n_out, model.num_pdfs), dtype=torch.float32, device=x.device)
    check(lib().ce_gpu_nnet_propagate_blocks(ctx.h, model.h, _ptr(x), x.stride(0),
                                             rows.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(rows),
                                             int(subtract_prior), _ptr(out)))
    return out


def loglik_gather(ctx, loglik, tid2pdf, rows, trans, am_scale=1.0, out=None):
    """ce_gpu_loglik_gather: am_scale * loglik[rows[i], tid2pdf[trans[i]]]
    (Decoder::LogLikelihood for n pairs); int32 device tensors."""
    import torch
    n = int(rows.numel())
    assert trans.numel() == n and rows.dtype == trans.dtype == tid2pdf.dtype == torch.int32
    if out is None:
        out = torch.empty((n,), dtype=torch.float32, device=loglik.device)
    check(lib().ce_gpu_loglik_gather(ctx.h, _ptr(loglik), loglik.shape[0], loglik.stride(0), loglik.shape[1],
                                     _ptr(tid2pdf),
                                     int(tid2pdf.numel()), _ptr(rows), _ptr(trans), n, float(am_scale),
                                     _ptr(out)))
    return out


def loglik_columns(ctx, loglik, cols, out=None):
    """ce_gpu_loglik_columns: loglik[:, cols] compacted (int32 device cols)."""
    import torch
    assert cols.dtype == torch.int32
    if out is None:
        out = torch.empty((loglik.shape[0], int(cols.numel())), dtype=torch.float32, device=loglik.device)
    check(lib().ce_gpu_loglik_columns(ctx.h, _ptr(loglik), loglik.shape[0], loglik.stride(0), loglik.shape[1],
                                      _ptr(cols), int(cols.numel()), _ptr(out)))
    return out


SUM_PARTS = 1024  # CE_GPU_SUM_PARTS


def sum_f64(x, acc, part):
    """ce_gpu_sum_f64 on torch's current stream: acc (a 0-d float64 device
    tensor) += the float64 sum of the contiguous float32 tensor x; part: a
    float64 device tensor of >= SUM_PARTS elements (scratch, stream-ordered)."""
    import torch
    assert x.dtype == torch.float32 and x.is_contiguous() and x.is_cuda
    assert acc.dtype == torch.float64 and acc.numel() == 1 and part.dtype == torch.float64
    assert part.numel() >= SUM_PARTS
    stream = torch.cuda.current_stream(x.device).cuda_stream
    check(lib().ce_gpu_sum_f64(stream, _ptr(x), x.numel(), _ptr(part), _ptr(acc)))
    return acc


SUM_MAX_BUFS = 16  # CE_GPU_SUM_MAX_BUFS


def sum_f64_many(xs, acc, part):
    """ce_gpu_sum_f64_many on torch's current stream: acc += the float64 sum
    of every contiguous float32 tensor in xs, SUM_MAX_BUFS at a time (one
    launch pair per group)."""
    import torch
    assert acc.dtype == torch.float64 and acc.numel() == 1 and part.dtype == torch.float64
    assert part.numel() >= SUM_PARTS
    stream = torch.cuda.current_stream(acc.device).cuda_stream
    for g in range(0, len(xs), SUM_MAX_BUFS):
        grp = xs[g:g + SUM_MAX_BUFS]
        for x in grp:
            assert x.dtype == torch.float32 and x.is_contiguous() and x.is_cuda
        ptrs = (ctypes.c_void_p * len(grp))(*[_ptr(x) for x in grp])
        ns = (ctypes.c_int64 * len(grp))(*[x.numel() for x in grp])
        check(lib().ce_gpu_sum_f64_many(stream, len(grp), ptrs, ns, _ptr(part), _ptr(acc)))
    return acc


def sgemm(ctx, a, b, c=None):
    import torch
    m, k = a.shape
    n = b.shape[1]
    if c is None:
        c = torch.empty((m, n), dtype=torch.float32, device=a.device)
    check(lib().ce_gpu_sgemm(ctx.h, m, n, k, _ptr(a), a.stride(0), _ptr(b), b.stride(0), _ptr(c),
                             c.stride(0)))
    return c


def quantize(ctx, x):
    """Returns (uint8 tensor, 8-byte device params tensor {f32 scale, i32 zp})."""
    import torch
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    prm = torch.empty(2, dtype=torch.int32, device=x.device)
    check(lib().ce_gpu_quantize(ctx.h, _ptr(x), x.numel(), _ptr(q), _ptr(prm)))
    return q, prm


def params_host(prm):
    """(scale, zero_point) of a device params record."""
    raw = prm.cpu().numpy()
    return float(raw[:1].view(np.float32)[0]), int(raw[1])


def gemm_u8(ctx, a, pa, b, pb, out_int32=False):
    import torch
    m, k = a.shape
    n = b.shape[1]
    if out_int32:
        c = torch.empty((m, n), dtype=torch.int32, device=a.device)
        check(lib().ce_gpu_gemm_u8u8i32(ctx.h, m, n, k, _ptr(a), _ptr(pa), _ptr(b), _ptr(pb), _ptr(c)))
    else:
        c = torch.empty((m, n), dtype=torch.float32, device=a.device)
        check(lib().ce_gpu_gemm_u8u8f32(ctx.h, m, n, k, _ptr(a), _ptr(pa), _ptr(b), _ptr(pb), _ptr(c)))
    return c
