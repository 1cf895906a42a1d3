"""Scheduling may not change a bit: the reference is a deterministic CPU path
whose per-utterance state lives in its Instance objects
(src/ce_stt.cc:53-60), so a frame's log-likelihoods cannot depend on which
other work ran beside it.  The benchmark's own pipeline -- one front stream
(fbank + CMVN) and three nnet streams, the driver's configuration -- keeps
every batch's fbank output, CMVN output and per-row log-likelihood sums as
the streams produced them; every batch is then re-scored serially on one
stream in the same process and compared bit for bit (bench.py
--verify-serial).  Round 3's exact fbank kernel, which spilled to scratch,
failed this in some runs."""
import os
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(extra):
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    return bench.main(["--steps", "60", "--warmup", "5", "--no-cpu-baseline", "--verify-serial"] + extra)


@pytest.mark.parametrize("extra", [[], ["--pcm", "s16"], ["--fbank", "fast"]], ids=["exact", "exact-s16", "fast"])
def test_pipelined_batches_equal_serial_rescore(extra):
    line = _run(extra)
    v = line["verify"]
    assert v["batches"] == 65
    assert v["differing"] == 0, v["detail"]
    assert line["finite"]


def test_prewarm_changes_no_result():
    """The pre-warm (untimed steps before the W warm-up steps) runs the same
    pipeline on the same inputs: the timed steps' output is bit-identical with
    and without it, and the line reports it beside `warmup`."""
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    base = ["--steps", "6", "--warmup", "2", "--no-cpu-baseline", "--no-profile"]
    off = bench.main(base + ["--prewarm-ms", "0"])
    on = bench.main(base + ["--prewarm-ms", "20"])
    assert off["prewarm"] == {"ms": 0.0, "steps": 0}
    assert on["prewarm"]["ms"] == 20.0 and on["prewarm"]["steps"] >= 10
    assert on["warmup"] == off["warmup"] == 2 and on["steps"] == off["steps"] == 6
    assert on["checksum"] == off["checksum"]
    assert on["finite"] and off["finite"]
