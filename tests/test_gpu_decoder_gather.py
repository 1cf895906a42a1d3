"""the decoder's per-frame log-likelihood reads
(Decoder::LogLikelihood, src/decoder.cc:97-102, called per active arc from
ProcessEmitting :327,350) as device gathers -- ce_gpu_loglik_gather for
(frame, transition id) pairs and ce_gpu_loglik_columns for a pdf subset --
against the oracle's restatement.  Both are pure index work: bit-exact."""
import numpy as np
import pytest

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


@pytest.fixture(scope="module")
def scored(torch, G, ctx, xs_config):
    """Real log-likelihood rows of the XS model on two utterances."""
    from catears_amd import synth
    model = G.Model(ctx, xs_config)
    waves = [synth.pcm(70 + i, 16000 * 2 + 333 * i) for i in range(2)]
    plan = G.Plan(ctx, [len(w) for w in waves], model)
    ll = G.score(ctx, model, plan, torch.from_numpy(np.concatenate(waves)).cuda())
    torch.cuda.synchronize()
    return model, ll


def _u32(x):
    return np.ascontiguousarray(x, np.float32).view(np.uint32)


@pytest.mark.parametrize("n,am_scale", [(1, 1.0), (5000, 0.1), (100003, 0.0833)])
def test_loglik_gather_matches_decoder(torch, G, ctx, oracle, scored, n, am_scale):
    model, ll = scored
    tpm = model.tid2pdf()
    rng = np.random.default_rng(n)
    rows = rng.integers(0, ll.shape[0], n).astype(np.int32)
    trans = rng.integers(1, len(tpm), n).astype(np.int32)
    d = lambda a: torch.from_numpy(a).cuda()
    got = G.loglik_gather(ctx, ll, d(tpm), d(rows), d(trans), am_scale).cpu().numpy()
    want = oracle.decoder_loglikelihood(ll.cpu().numpy(), tpm, rows, trans, am_scale)
    assert np.array_equal(_u32(got), _u32(want))


def test_loglik_gather_edges(torch, G, ctx, scored):
    """Empty input is a no-op; out-of-range frames / transition ids give NaN
    (the reference would index out of bounds)."""
    model, ll = scored
    tpm = torch.from_numpy(model.tid2pdf()).cuda()
    e = torch.empty((0,), dtype=torch.int32, device="cuda")
    assert G.loglik_gather(ctx, ll, tpm, e, e).numel() == 0
    rows = torch.tensor([0, -1, ll.shape[0], 3, 3], dtype=torch.int32, device="cuda")
    trans = torch.tensor([1, 1, 1, -5, tpm.numel()], dtype=torch.int32, device="cuda")
    got = G.loglik_gather(ctx, ll, tpm, rows, trans).cpu().numpy()
    assert np.isfinite(got[0]) and np.isnan(got[1:]).all()
    # a corrupt tid2pdf entry (pdf outside the row) also gives NaN, never a
    # read past the row
    bad = torch.tensor([0, ll.shape[1], -1, 2**30], dtype=torch.int32, device="cuda")
    rows = torch.tensor([0, 0, 0, ll.shape[0] - 1], dtype=torch.int32, device="cuda")
    trans = torch.tensor([0, 1, 2, 3], dtype=torch.int32, device="cuda")
    got = G.loglik_gather(ctx, ll, bad, rows, trans).cpu().numpy()
    assert np.isfinite(got[0]) and np.isnan(got[1:]).all()


def test_loglik_columns(torch, G, ctx, scored):
    _, ll = scored
    rng = np.random.default_rng(9)
    cols = np.concatenate([rng.permutation(ll.shape[1])[:97], [0, ll.shape[1] - 1, ll.shape[1], -1]]).astype(np.int32)
    got = G.loglik_columns(ctx, ll, torch.from_numpy(cols).cuda()).cpu().numpy()
    host = ll.cpu().numpy()
    assert got.shape == (ll.shape[0], len(cols))
    assert np.array_equal(_u32(got[:, :-2]), _u32(host[:, cols[:-2]]))
    assert np.isnan(got[:, -2:]).all()
