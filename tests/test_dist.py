"""Multi-rank logic of the benchmark on CPU (gloo, world size 2): the C4
corpus, utterance sharding, batch packing and the streamed variable-length
log-likelihood gather to rank 0."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from catears_amd.shard import (C4_UTTS, RowGather, c4_corpus, exchange_counts, num_frames, pack_batches,
                               shard_utterances)


def test_shard_covers_and_balances():
    lengths = [998] * 9 + [10, 500, 2000, 3, 0]
    for world in (1, 2, 3, 8):
        parts = [shard_utterances(lengths, world, r) for r in range(world)]
        flat = sorted(i for p in parts for i in p)
        assert flat == list(range(len(lengths)))
        loads = [sum(lengths[i] for i in p) for p in parts]
        assert max(loads) - min(loads) <= max(lengths)
    assert shard_utterances(lengths, 2, 0) == shard_utterances(lengths, 2, 0)


def test_shard_weights_give_rank0_its_share():
    """bench.py's sink share: rank 0 weighted 0.62 at 8 ranks gets 0.62 of a
    peer's frames (within one utterance), every utterance exactly once."""
    from catears_amd.shard import c4_corpus
    frames = [num_frames(int(n)) for n in c4_corpus(4000)]
    w = [0.62] + [1.0] * 7
    parts = [shard_utterances(frames, 8, r, weights=w) for r in range(8)]
    assert sorted(i for p in parts for i in p) == list(range(len(frames)))
    loads = [sum(frames[i] for i in p) for p in parts]
    peer = sum(loads[1:]) / 7
    assert abs(loads[0] / peer - 0.62) < 0.01
    assert max(loads[1:]) - min(loads[1:]) <= max(frames)


def test_c4_corpus_is_100h_length_mixed():
    s = c4_corpus()
    assert len(s) == C4_UTTS == 36000
    assert s.sum() == 36000 * 160000                     # exactly 100 h at 16 kHz
    assert s.min() >= 32000 and s.max() <= 288000         # 2 .. 18 s
    assert len(np.unique(s)) > 10000                      # a real length mix
    frames = sum(num_frames(int(n)) for n in s)
    assert abs(frames - 35.93e6) < 0.01 * 35.93e6         # 35.93 M frames
    assert np.array_equal(c4_corpus(), s)                 # seeded


def test_c4_shards_and_batches():
    s = c4_corpus(2000)
    frames = [num_frames(int(n)) for n in s]
    for world in (1, 2, 8):
        seen = []
        loads = []
        for r in range(world):
            mine = shard_utterances(frames, world, r)
            batches = pack_batches([frames[u] for u in mine], 10, 10, 4096)
            for b in batches:
                assert sum(frames[mine[i]] + 20 for i in b) <= 4096
                seen += [mine[i] for i in b]
            loads.append(sum(frames[u] for u in mine))
        assert sorted(seen) == list(range(len(s)))
        assert max(loads) - min(loads) <= max(frames)


def test_pack_batches_edges():
    assert pack_batches([], 1, 1) == []
    assert pack_batches([0, 5, 0], 1, 1, 10) == [[1]]
    # an utterance longer than a batch still gets one (the plan splits it)
    assert pack_batches([3, 20, 3], 1, 1, 10) == [[0], [1], [2]]
    assert pack_batches([3, 3, 3], 1, 1, 10) == [[0, 1], [2]]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows(rank, step, n, width):
    # distinct values in every row and column, so a row lost or moved shows
    return (1000.0 * rank + 10.0 * step + np.arange(n)[:, None] + 0.001 * np.arange(width)[None, :]).astype(np.float32)


# ragged per-rank batch lists: ranks with a step more or fewer than rank 0,
# steps with no rows, a rank with no rows at all (3)
_COUNTS = {0: [5, 3, 4], 1: [2, 6, 0, 1], 2: [8, 1, 1, 7, 2], 3: []}


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        width = 7
        # ragged per-rank batch lists: rank 1 has one step more, and a step
        # with no rows at all
        mine = _COUNTS[rank]
        counts = exchange_counts(mine)
        g = RowGather(counts, width, torch.float32, "cpu", depth=2, keep=True)
        bufs = [torch.empty(8, width) for _ in range(2)]
        steps = max(len(c) for c in counts)
        for s in range(steps):
            slot = s % 2
            g.wait_slot(slot)
            n = mine[s] if s < len(mine) else 0
            if n:
                bufs[slot][:n] = torch.from_numpy(_rows(rank, s, n, width))
            own = bufs[slot][:n] if rank == 0 and n else None
            assert g.submit(s, bufs[slot], own=own) == slot
        total = float(g.drain())
        kept = [(p, s, a.tolist()) for p, s, a in (g.keep or [])]
        q.put((rank, total, g.rows_in, kept))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_row_gather_gloo_ragged(world):
    """RowGather on `world` gloo ranks: with 4, rank 0 posts the receives of
    three peers in one grouped batch_isend_irecv per step (the N = 4 / 8
    shape), peers run out of steps at different times and one peer sends
    nothing."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, total, rows_in, kept = q.get(timeout=120)
        res[r] = (total, rows_in, kept)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    counts = {r: _COUNTS[r] for r in range(world)}
    want = sum(float(_rows(r, s, n, 7).astype(np.float64).sum()) for r in counts for s, n in enumerate(counts[r]) if n)
    assert res[0][0] == pytest.approx(want, rel=1e-12)
    assert res[0][1] == sum(sum(counts[r]) for r in counts if r)
    # every received row, full width, exactly the sender's
    got = {(p, s): np.array(a, np.float32) for p, s, a in res[0][2]}
    assert sorted(got) == sorted((p, s) for p in counts if p for s, n in enumerate(counts[p]) if n)
    for (p, s), a in got.items():
        assert np.array_equal(a, _rows(p, s, counts[p][s], 7))
