"""bench.py's bookkeeping (no GPU): the algorithmic FLOP and byte counts its
roofline uses, and that the kernel names it quotes traffic for exist in the
newest committed PMC summaries (a renamed kernel would silently drop
roofline.traffic to null)."""
import importlib
import sys

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def bench():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    return importlib.import_module("bench")


def test_flops_per_frame_matches_survey(bench):
    # 2 * (200*1024 + 4*3072*1024 + 1024*1024 + 1024*3456)
    assert bench.FLOPS_PER_FRAME == 34_750_464


def test_split_algorithmic_bytes(bench):
    rows = 4072
    layers = ((256, 1024),) + ((3072, 1024),) * 4 + ((1024, 1024), (1024, 3456))
    want = sum(4 * rows * k + 4 * k * n + 4 * rows * n for k, n in layers) / len(layers)
    assert bench.split_algorithmic_bytes(rows, 4) == pytest.approx(want)
    # planes: 6-byte operands and hidden outputs, fp32 last layer
    want6 = sum(6 * rows * k + 6 * k * n + (4 if i == 6 else 6) * rows * n
                for i, (k, n) in enumerate(layers)) / len(layers)
    assert bench.split_algorithmic_bytes(rows, 6) == pytest.approx(want6)


@pytest.mark.parametrize("workload,kernel", [
    ("c3", "SPLIT_BF16X6"),
    ("c5", "I8"),
])
def test_roofline_kernels_have_committed_traffic(bench, workload, kernel):
    name = bench.SPLIT_ROOFLINE_KERNEL["bf16x6"] if kernel == "SPLIT_BF16X6" else bench.I8_ROOFLINE_KERNEL
    traffic, src = bench.pmc_traffic(name, workload)
    assert src is not None, f"no committed PMC summary for {workload}"
    assert traffic is not None and traffic > 0, f"{name} not in {src}"


@pytest.mark.parametrize("workload,kernel", [
    ("c3", "SPLIT_BF16X6"),
    ("c5", "I8"),
])
def test_roofline_kernels_have_committed_mfma_util(bench, workload, kernel):
    """The rocprof MFMA-utilisation figure (north star) exists for the
    dominant GEMM of C3 and C5 and is a fraction."""
    name = bench.SPLIT_ROOFLINE_KERNEL["bf16x6"] if kernel == "SPLIT_BF16X6" else bench.I8_ROOFLINE_KERNEL
    u = bench.pmc_mfma(name, workload)
    assert u is not None, f"no committed MFMA-utilisation summary for {name} ({workload})"
    assert 0.0 < u["chip"] <= u["active_cus"] <= 1.0
