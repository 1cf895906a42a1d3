"""ce_gpu_ctx_set_stream (include/catears_gpu.h): switching a context to a
new stream and then destroying the old one -- the order the header
documents -- leaves the context working, and results do not depend on the
stream they were computed on."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_switch_then_destroy_old_stream():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from catears_amd import gpu, synth
    hip = ctypes.CDLL("libamdhip64.so")
    L = gpu.lib()
    ctx = gpu.Context(0)
    waves = [synth.pcm(11 + i, n) for i, n in enumerate((16000, 400, 33333))]

    def run():
        plan = gpu.Plan(ctx, [len(w) for w in waves])
        pcm = torch.from_numpy(np.concatenate(waves).astype(np.float32)).cuda()
        feats = torch.empty((plan.total_frames, 40), dtype=torch.float32, device="cuda")
        mel = torch.empty_like(feats)
        gpu.fbank(ctx, plan, pcm, feats, mel)
        ctx.synchronize()
        return feats.cpu().numpy()

    ref = run()
    streams = []
    for _ in range(3):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        streams.append(s)
    old = None
    for s in streams:
        gpu.check(L.ce_gpu_ctx_set_stream(ctx.h, s))
        if old is not None:
            assert hip.hipStreamDestroy(old) == 0  # switch first, destroy the old stream afterwards
        old = s
        assert np.array_equal(run().view(np.uint32), ref.view(np.uint32))
    torch_stream = torch.cuda.current_stream()
    gpu.check(L.ce_gpu_ctx_set_stream(ctx.h, ctypes.c_void_p(torch_stream.cuda_stream)))
    assert hip.hipStreamDestroy(old) == 0
    assert np.array_equal(run().view(np.uint32), ref.view(np.uint32))
