"""ce_gpu_sum_f64 / ce_gpu_sum_f64_many: the float64 checksum rank 0 folds every gathered
log-likelihood row into (catears_amd/shard.py RowGather, bench.py).  No
reference counterpart: the stand-in for the consumer of the rows gathered to
rank 0.  Checked against numpy's float64 sum of the same
floats (each widened to double, as the kernel does; only the summation order
differs, so agreement to ~1e-15 relative), for aligned and unaligned starts,
ragged lengths and an empty input, and the same bytes give the same bits."""
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


@pytest.mark.parametrize("n,offset", [(1, 0), (3, 0), (5, 1), (1023, 0), (4097, 3), (4072 * 3456, 0),
                                      (998 * 3456 + 7, 1)])
def test_sum_f64_matches_numpy(torch, G, n, offset):
    rng = np.random.default_rng(n)
    host = (rng.normal(-8.0, 3.0, size=n + offset)).astype(np.float32)
    dev = torch.from_numpy(host).cuda()
    x = dev[offset:]  # offset 1 or 3: not 16-byte aligned, the scalar path
    acc = torch.full((), 0.5, dtype=torch.float64, device="cuda")
    part = torch.empty(G.SUM_PARTS, dtype=torch.float64, device="cuda")
    G.sum_f64(x, acc, part)
    want = 0.5 + host[offset:].astype(np.float64).sum()
    got = acc.item()
    assert got == pytest.approx(want, rel=1e-13, abs=1e-9)
    # the same bytes give the same double
    acc2 = torch.full((), 0.5, dtype=torch.float64, device="cuda")
    G.sum_f64(x, acc2, part)
    assert acc2.item() == got


def test_sum_f64_empty_and_errors(torch, G):
    acc = torch.zeros((), dtype=torch.float64, device="cuda")
    part = torch.empty(G.SUM_PARTS, dtype=torch.float64, device="cuda")
    G.sum_f64(torch.empty(0, dtype=torch.float32, device="cuda"), acc, part)
    assert acc.item() == 0.0
    with pytest.raises(G.CatearsError):
        G.check(G.lib().ce_gpu_sum_f64(None, None, 5, None, None))


def test_sum_f64_many_matches_numpy(torch, G):
    """Several buffers in one launch pair (RowGather's per-step fold): aligned,
    unaligned and empty buffers, more than one group of SUM_MAX_BUFS."""
    rng = np.random.default_rng(7)
    sizes = [4072 * 3456, 5, 0, 1023, 998 * 3456 + 3] + [4096 + i for i in range(14)]
    hosts = [rng.normal(-8.0, 3.0, size=n + 1).astype(np.float32) for n in sizes]
    xs = [torch.from_numpy(h).cuda()[i % 2:i % 2 + n] for i, (h, n) in enumerate(zip(hosts, sizes))]
    acc = torch.zeros((), dtype=torch.float64, device="cuda")
    part = torch.empty(G.SUM_PARTS, dtype=torch.float64, device="cuda")
    G.sum_f64_many(xs, acc, part)
    want = sum(h[i % 2:i % 2 + n].astype(np.float64).sum() for i, (h, n) in enumerate(zip(hosts, sizes)))
    assert acc.item() == pytest.approx(want, rel=1e-13, abs=1e-9)
    acc2 = torch.zeros((), dtype=torch.float64, device="cuda")
    G.sum_f64_many(xs, acc2, part)
    assert acc2.item() == acc.item()
