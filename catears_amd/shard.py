"""Utterance sharding, the C4 corpus and the log-likelihood gather.

Utterances are independent through fbank, CMVN (per-utterance window +
constant global stats) and the TDNN (context never crosses utterances): the
reference keeps every per-utterance state in its own Instance objects
(src/ce_stt.cc:53-60) and the AM's output does not depend on how its rows are
chunked (src/am.cc:73-80,115-164).  A node therefore shards utterances across
GPUs with no data-path collective.  The one exchange is the north star's:
every rank's log-likelihood batches go to rank 0 (RCCL point-to-point over
xGMI when the backend is "nccl"), streamed per batch into a small ring of
receive buffers -- 100 h of TDNN-S posteriors are ~497 GB, more than one GPU's
288 GB, so rank 0 consumes (here: checksums every row of) each batch instead
of storing the run.

Backend-agnostic: the same code runs on CPU tensors with gloo (tests), and
stages CUDA tensors through the host when the backend is gloo (one-GPU
rehearsals of N ranks).
"""
import numpy as np
import torch
import torch.distributed as dist

FRAME_LEN, FRAME_SHIFT = 400, 160   # src/fbank.h:7-13
C4_UTTS = 36000                     # 100 h of 10 s-average utterances
C4_PAIR_SAMPLES = 320000            # two utterances per 20 s pair
C4_MIN_SAMPLES = 32000              # 2 s


def num_frames(n):
    """Fbank frames of n samples (src/fbank.cc:35-42)."""
    return 0 if n < FRAME_LEN else 1 + (n - FRAME_LEN) // FRAME_SHIFT


def c4_corpus(n_utts=C4_UTTS, seed=20250117):
    """Sample counts of the C4 corpus: a seeded length mix of 2-18 s
    utterances in pairs (a, 320000 - a) with a uniform over [2 s, 18 s], so
    the corpus is exactly n_utts x 10 s of audio (100 h at the default
    36 000 utterances) while no two neighbours need have the same length."""
    from .synth import splitmix64
    if n_utts % 2:
        raise ValueError("the C4 corpus is built from pairs of utterances")
    span = C4_PAIR_SAMPLES - 2 * C4_MIN_SAMPLES + 1
    a = C4_MIN_SAMPLES + (splitmix64(seed, n_utts // 2) % np.uint64(span)).astype(np.int64)
    out = np.empty(n_utts, np.int64)
    out[0::2] = a
    out[1::2] = C4_PAIR_SAMPLES - a
    return out


def shard_utterances(lengths, world, rank, weights=None):
    """Longest-first greedy assignment by frame count: returns the indices of
    the utterances rank `rank` scores, ascending (deterministic, balanced
    within one utterance's length).  weights: each rank's relative capacity
    (default equal; bench.py gives rank 0, the gather sink, less)."""
    w = [1.0] * world if weights is None else [float(x) for x in weights]
    assert len(w) == world and all(x > 0 for x in w)
    order = sorted(range(len(lengths)), key=lambda i: (-int(lengths[i]), i))
    load = [0] * world
    owner = [0] * len(lengths)
    for i in order:
        r = min(range(world), key=lambda k: ((load[k] + int(lengths[i])) / w[k], k))
        owner[i] = r
        load[r] += int(lengths[i])
    return [i for i in range(len(lengths)) if owner[i] == rank]


def pack_batches(frames, left, right, max_rows=4096):
    """Consecutive utterances into frame batches of at most `max_rows` packed
    rows (T + L + R per utterance, the layout ce_gpu_plan_create packs):
    returns lists of positions into `frames`.  An utterance longer than a
    batch gets a batch of its own (the plan then splits it into overlapping
    chunks, src/am.cc:73-80)."""
    batches, cur, rows = [], [], 0
    for i, t in enumerate(frames):
        if t <= 0:
            continue  # no frames, no rows (fbank returns 0 x 40)
        need = int(t) + left + right
        if cur and rows + need > max_rows:
            batches.append(cur)
            cur, rows = [], 0
        cur.append(i)
        rows += need
    if cur:
        batches.append(cur)
    return batches


class RowGather:
    """Streams every rank's variable-length row batches to rank 0.

    `counts[r][s]` is the number of rows rank r contributes at step s (0 or
    absent: none), known to every rank from a setup exchange
    (exchange_counts).  submit(s, t) sends this rank's rows of step s (rank
    0: posts the receives of every peer's step-s rows into ring slot s %
    depth, grouped into one batch_isend_irecv, and folds every received row
    -- and, with own=, its own rows -- into a float64 checksum: the stand-in
    for the decoder that would consume them).  A sender must not modify `t`
    until wait_slot(s % depth) returns.  CUDA tensors go through RCCL on the
    "nccl" backend; on gloo they are staged through host memory.
    """

    def __init__(self, counts, width, dtype, device, depth=3, group=None, keep=False):
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.group = group
        self.counts = [list(c) for c in counts]
        self.width = width
        self.depth = depth
        self.device = torch.device(device)
        self.staged = dist.get_backend(group) == "gloo" and self.device.type == "cuda"
        self.pending = [None] * depth  # (works, retire callback) per slot
        self.recv = None
        if self.rank == 0:
            rows = [max(c) if c else 0 for c in self.counts]
            rdev = "cpu" if self.staged else self.device
            self.recv = [[torch.empty((max(rows[p], 1), width), dtype=dtype, device=rdev) for p in range(self.world)]
                         for _ in range(depth)]
        self.sums = [torch.zeros((), dtype=torch.float64, device=self.device) for _ in range(depth)]
        # device folds run ce_gpu_sum_f64 (HBM speed; torch's float64 sum runs
        # at about a third of it): scratch per slot, as a slot's folds are
        # ordered on one stream
        self.parts = None
        if self.device.type == "cuda":
            from catears_amd import gpu
            self.parts = [torch.empty(gpu.SUM_PARTS, dtype=torch.float64, device=self.device) for _ in range(depth)]
        self.rows_in = 0       # rows rank 0 received
        self.batches = 0       # steps retired
        self.keep = [] if keep else None  # (peer, step, host rows) -- tests only

    def rows(self, r, s):
        c = self.counts[r]
        return c[s] if s < len(c) else 0

    def _retire(self, slot):
        pend = self.pending[slot]
        if pend is None:
            return
        works, after, stream = pend
        self.pending[slot] = None
        if stream is None:  # CPU tensors
            for w in works:
                w.wait()
            if after is not None:
                after()
        else:
            # the transfers and rank 0's checksums run on the stream the step
            # was submitted from; the caller's stream then waits for all of
            # it (its buffer may be overwritten after this returns)
            with torch.cuda.stream(stream):
                for w in works:
                    w.wait()
                if after is not None:
                    after()
                ev = torch.cuda.Event()
                ev.record(stream)
            torch.cuda.current_stream(self.device).wait_event(ev)
        self.batches += 1

    def submit(self, s, t=None, own=None):
        slot = s % self.depth
        self._retire(slot)
        ops, after = [], None
        if self.rank != 0:
            n = self.rows(self.rank, s)
            if n:
                assert t is not None and t.shape[0] >= n and t.shape[1] == self.width
                src = t[:n]
                if self.staged:
                    src = src.cpu()
                ops.append(dist.P2POp(dist.isend, src.contiguous(), 0, self.group))
        else:
            bufs = []
            for p in range(1, self.world):
                n = self.rows(p, s)
                if n:
                    b = self.recv[slot][p][:n]
                    bufs.append((p, b))
                    ops.append(dist.P2POp(dist.irecv, b, p, self.group))
            acc, part = self.sums[slot], self.parts[slot] if self.parts is not None else None

            def after():
                # every peer's rows of this step (and rank 0's own) in one fold
                xs = [own] if own is not None else []
                for p, b in bufs:
                    xs.append(b.to(self.device, non_blocking=False) if self.staged else b)
                    self.rows_in += b.shape[0]
                    if self.keep is not None:
                        self.keep.append((p, s, b.cpu().numpy().copy()))
                self._fold(xs, acc, part)
        works = dist.batch_isend_irecv(ops) if ops else []
        stream = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        self.pending[slot] = (works, after, stream)
        return slot

    @staticmethod
    def _fold(xs, acc, part):
        if not xs:
            return
        if xs[0].is_cuda:
            from catears_amd import gpu
            gpu.sum_f64_many([x.contiguous() for x in xs], acc, part)
        else:
            for x in xs:
                acc.add_(torch.sum(x, dtype=torch.float64))

    def wait_slot(self, slot):
        """Order the current stream (NCCL) or the host (gloo) after the
        transfer occupying `slot`; after it that step's input may be
        overwritten and (rank 0) its rows have been consumed."""
        self._retire(slot)

    def drain(self):
        for i in range(self.depth):
            self._retire(i)
        return self.checksum

    @property
    def checksum(self):
        return sum(self.sums[1:], self.sums[0].clone())


def exchange_counts(mine, group=None):
    """Every rank's per-step row counts (and any other picklable per-step
    description, e.g. utterance ids), gathered once at setup so rank 0 can
    post exact-size receives."""
    world = dist.get_world_size(group)
    out = [None] * world
    dist.all_gather_object(out, mine, group=group)
    return out
