"""BASELINE config C4 end to end on one GPU: bench.py --workload c4 shards a
length-mixed corpus over 2 ranks (gloo, both on device 0 -- the one-GPU
rehearsal of the N-GPU run; the processes are started by torchrun before any
GPU call), packs each rank's utterances into ragged <= 4096-row batches,
scores them and streams every batch to rank 0.  Rank 0's consumed rows --
its own and the peer's, per utterance -- must be bit-identical to one process
scoring the whole corpus alone: sharding and batching may not change a bit
(per-utterance state only, src/ce_stt.cc:53-60; chunk-invariant AM,
src/am.cc:73-80,115-164)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

UTTS = 24  # 24 x 2-18 s (4 min of audio): several ragged batches per rank


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(extra, dump, nproc):
    env = dict(os.environ, PYTHONPATH=ROOT, CATEARS_BENCH_DEVICE="0")
    args = ["bench.py", "--workload", "c4", "--c4-utts", str(UTTS), "--model", "tdnn-xs", "--warmup", "2",
            "--no-cpu-baseline", "--c4-dump", str(dump)] + extra
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args + ["--dist-backend", "gloo"]
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    return json.loads(line[0])


def test_c4_two_ranks_bit_identical_to_one_process(tmp_path):
    from catears_amd.shard import c4_corpus, num_frames
    one = _bench([], tmp_path / "one.npz", 1)
    two = _bench([], tmp_path / "two.npz", 2)
    frames = [num_frames(int(n)) for n in c4_corpus(UTTS)]
    assert one["config"]["frames_total"] == two["config"]["frames_total"] == sum(frames)
    assert two["n_gpus"] == 2 and two["config"]["gather"]
    assert sum(two["config"]["frames_per_rank"]) == sum(frames)
    assert two["config"]["rows_gathered_to_rank0"] == two["config"]["frames_per_rank"][1] > 0
    assert max(two["config"]["batches_per_rank"]) >= 2
    a, b = np.load(tmp_path / "one.npz"), np.load(tmp_path / "two.npz")
    assert sorted(a.files) == sorted(b.files) == sorted(f"u{u}" for u in range(UTTS))
    for k in a.files:
        u = int(k[1:])
        assert a[k].shape == (frames[u], 512)
        assert np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)), k
    # the checksums fold every row of every utterance: equal up to fp64 order
    assert two["checksum"] == pytest.approx(one["checksum"], rel=1e-12)


def _bench_c3(extra, nproc):
    env = dict(os.environ, PYTHONPATH=ROOT, CATEARS_BENCH_DEVICE="0")
    args = ["bench.py", "--model", "tdnn-xs", "--steps", "6", "--warmup", "2", "--pool", "8",
            "--no-cpu-baseline"] + extra
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args + ["--gpus", str(nproc),
                                                                                     "--dist-backend", "gloo"]
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    return json.loads(line[0])


def test_c3_two_ranks_gather_every_row(tmp_path):
    """The driver's N > 1 C3 command (bench.py main: three nnet streams,
    per-batch events, the comm stream, RowGather's receive ring and
    wait_slot), rehearsed with 2 gloo ranks on device 0.  Within the run:
    every batch rank 1 sends (its rows as scored, copied on the stream that
    hands them to the gather) arrives at rank 0 bit for bit, and rank 0's
    checksum folds exactly its own batches and the received ones, warm-up
    included -- no batch lost, duplicated or read before it was written."""
    steps = 6 + 2
    two = _bench_c3(["--c3-dump", str(tmp_path / "d.npz")], 2)
    assert two["n_gpus"] == 2 and two["config"]["gather"] and two["finite"]
    r0, r1 = np.load(tmp_path / "d.rank0.npz"), np.load(tmp_path / "d.rank1.npz")
    assert sorted(r1.files) == sorted(f"r1s{s}" for s in range(steps))
    want = 0.0
    for s in range(steps):
        sent, got, own = r1[f"r1s{s}"], r0[f"r1s{s}"], r0[f"r0s{s}"]
        assert sent.shape == got.shape == own.shape
        assert np.array_equal(sent.view(np.uint32), got.view(np.uint32)), s
        want += float(own.astype(np.float64).sum()) + float(got.astype(np.float64).sum())
    assert two["checksum"] == pytest.approx(want, rel=1e-12)
    # the two ranks score different audio: a gather that dropped the peer's
    # rows (or sent rank 0's twice) would miss by a whole rank's sum
    assert not np.array_equal(r0["r0s0"], r0["r1s0"])
