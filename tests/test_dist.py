"""Multi-rank logic of the benchmark on CPU (gloo, world size 2): utterance
sharding and the streamed log-likelihood gather to rank 0."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from catears_amd.shard import LoglikGather, shard_utterances


def test_shard_covers_and_balances():
    lengths = [998] * 9 + [10, 500, 2000, 3, 0]
    for world in (1, 2, 3, 8):
        parts = [shard_utterances(lengths, world, r) for r in range(world)]
        flat = sorted(i for p in parts for i in p)
        assert flat == list(range(len(lengths)))
        loads = [sum(lengths[i] for i in p) for p in parts]
        assert max(loads) - min(loads) <= max(lengths)
    assert shard_utterances(lengths, 2, 0) == shard_utterances(lengths, 2, 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, steps, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = LoglikGather((5, 7), torch.float32, "cpu", depth=3)
        bufs = [torch.empty(5, 7) for _ in range(3)]
        for i in range(steps):
            o = i % 3
            g.wait_slot(o)
            bufs[o].fill_(1000.0 * rank + i)  # row 0 sums to 7 * value
            assert g.submit(bufs[o]) == o
        total = g.drain()
        q.put((rank, float(total), g.batches))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_streamed_gather_gloo(world):
    steps = 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict()
    for _ in range(world):
        r, total, batches = q.get(timeout=120)
        res[r] = (total, batches)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = sum(7.0 * (1000.0 * r + i) for r in range(world) for i in range(steps))
    assert res[0][0] == pytest.approx(expect)
    assert all(b == steps for _, b in res.values())
