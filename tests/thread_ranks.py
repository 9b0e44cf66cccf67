"""W ranks of the REAL multi-GPU step (smash-paper_amd/dist.py
ShardedCounter.step / count_fastq) as W threads of one process on ONE
device (test infrastructure).  Only the transport is replaced: ThreadComm
implements the three collectives the step uses (the key-count exchange,
all_to_all with split sizes, all_gather) with device copies between the
threads' tensors.  Everything else -- the look-ahead search of the next
batch, the two-ahead search after the export, the owner de-dup, the tail
bookkeeping -- is the code `bench.py --gpus N` and `smash_cli count` run.

Each collective synchronises the device before it publishes its input and
after it has copied its output (the ranks' pipelines run on their own
streams), then meets the other threads at a barrier: slow, but every byte
a rank reads was complete when it was published."""
import threading

import numpy as np
import torch

import smashgpu as S
from dist import ShardedCounter, count_fastq, open_fastq


class ThreadWorld:
    def __init__(self, world, timeout=600.0):
        self.world = world
        self.barrier = threading.Barrier(world, timeout=timeout)
        self.slot = [None] * world

    def comm(self, rank):
        return ThreadComm(self, rank)


class ThreadComm:
    def __init__(self, tw, rank):
        self.tw = tw
        self.rank = rank

    def _publish(self, x):
        torch.cuda.synchronize()
        self.tw.slot[self.rank] = x
        self.tw.barrier.wait()

    def _done(self):
        torch.cuda.synchronize()
        self.tw.barrier.wait()   # nobody republishes before every rank has read

    def exchange_counts(self, rows):
        self._publish([list(r) for r in rows])
        got = [self.tw.slot[s][self.rank] for s in range(self.tw.world)]
        self._done()
        return got

    def all_to_all(self, out, inp, out_splits, in_splits):
        self._publish((inp, [int(x) for x in in_splits]))
        o = 0
        for s in range(self.tw.world):
            src, sp = self.tw.slot[s]
            a, n = sum(sp[:self.rank]), sp[self.rank]
            assert n == int(out_splits[s]), (s, n, out_splits)
            if n:
                out[o:o + n].copy_(src[a:a + n])
            o += n
        self._done()

    def all_gather(self, parts, t):
        self._publish(t)
        for s in range(self.tw.world):
            parts[s].copy_(self.tw.slot[s])
        self._done()

    def all_gather_bytes(self, b):
        self.tw.slot[self.rank] = b
        self.tw.barrier.wait()
        got = list(self.tw.slot)
        self.tw.barrier.wait()
        return got


def _run_threads(world, body):
    tw = ThreadWorld(world)
    errs = [None] * world

    def run(r):
        try:
            body(r, tw.comm(r))
        except BaseException as e:   # noqa: BLE001 -- reported below
            errs[r] = e
            tw.barrier.abort()       # the other ranks leave their barrier too

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in errs:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in errs:
        if e is not None:
            raise e


def _summary(pipes, counts):
    total = sum(c.cpu().numpy().astype(np.uint64) for c in counts)
    st = [p.stats() for p in pipes]
    return total, (sum(x.positions for x in st), sum(x.dups for x in st),
                   sum(x.kept for x in st), sum(x.dupe_pairs for x in st))


def make_pipes(ix, world, cs, starts, L, batch, capacity):
    pipes = [S.Pipeline(ix, cs, starts, L, batch, dedup_capacity=capacity)
             for _ in range(world)]
    counts = [torch.zeros(len(starts), dtype=torch.int64, device="cuda") for _ in range(world)]
    return pipes, counts


def run_resident(ix, d_reads, world, per_rank, starts, cs, ahead2=True, capacity=None, runs=1,
                 cross=False):
    """bench.py's sharded step loop, one thread per rank: rank r's pairs are
    d_reads' global pairs [b W B + r B, + B) of batch b (the bench's layout:
    each rank holds its own P pairs, here dealt from one tensor), with the
    next batch searched under this one's exchange and, with ahead2, the one
    after that right after the export.  runs: that many runs over the same
    pairs back to back, each from a reset (a fresh run); cross: as bench.py
    does, a run's last batch issues the next run's first searches and the
    next run's reset keeps them, and the searches wait on no input event
    (smash_pipeline_reads_resident).  Returns the last run's summary (with
    runs > 1: and every run's counts)."""
    n = d_reads.shape[0] // 2
    nb = n // (world * per_rank)
    assert nb * world * per_rank == n
    pipes, counts = make_pipes(ix, world, cs, starts, d_reads.shape[1], per_rank,
                               capacity or n)
    dev = d_reads.device
    per_run = [[None] * world for _ in range(runs)]
    if cross:   # (as bench.py's sharded step: resident reads, no input event)
        for p in pipes:
            p.reads_resident(True)

    def body(r, comm):
        sc = ShardedCounter(pipes[r], r, world, dev, comm=comm)

        def mine(b):   # rank r's batch b, or None past the end
            if b >= nb:
                return None
            lo = b * world * per_rank + r * per_rank
            return d_reads[2 * lo:2 * (lo + per_rank)]

        for run in range(runs):
            sc.reset(keep_search=cross and run > 0)
            counts[r].zero_()
            for b in range(nb):
                more = cross and run + 1 < runs
                nxt = mine(b + 1) if b + 1 < nb else (mine(0) if more else None)
                if not ahead2:
                    nxt2 = None
                elif b + 2 < nb:
                    nxt2 = mine(b + 2)
                else:   # (the next run's batch after nxt, when that is its first)
                    nxt2 = mine(b + 2 - nb) if more and 0 < b + 2 - nb < nb else None
                sc.step(mine(b), per_rank, b * world * per_rank, counts[r],
                        nxt, per_rank if nxt is not None else 0,
                        next2_reads=nxt2, next2_pairs=per_rank if nxt2 is not None else 0)
            per_run[run][r] = counts[r].cpu().numpy().astype(np.uint64)

    _run_threads(world, body)
    if runs == 1:
        return _summary(pipes, counts)
    return _summary(pipes, counts) + ([sum(x) for x in per_run],)


def run_files(ix, paths, world, batch, starts, cs, capacity, shards=True):
    """dist.count_fastq over `world` ranks, each opening the lists as
    smash_cli count does under torchrun (dist.open_fastq: the rank-local
    reader; shards=False: every rank its own whole-input FastqIndex).
    Returns (counts, stats, pairs counted per rank, reader stats per rank)."""
    tw = ThreadWorld(world)
    fqs = [None] * world
    errs = [None] * world

    def opener(r):
        try:
            if shards:
                fqs[r] = open_fastq(ShardedCounter(_NoPipe(), r, world, torch.device("cuda"),
                                                   comm=tw.comm(r)), *paths)
            else:
                fqs[r] = S.FastqIndex(*paths)
        except BaseException as e:   # noqa: BLE001
            errs[r] = e
            tw.barrier.abort()
    th = [threading.Thread(target=opener, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in errs:
        if e is not None:
            raise e
    L = fqs[0].L
    pipes, counts = make_pipes(ix, world, cs, starts, L, batch, capacity)
    done = [0] * world

    def body(r, comm):
        sc = ShardedCounter(pipes[r], r, world, torch.device("cuda"), comm=comm)
        sc.reset()
        done[r] = count_fastq(sc, fqs[r], batch, counts[r])

    _run_threads(world, body)
    total, st = _summary(pipes, counts)
    rstats = [f.stats() if hasattr(f, "stats") else None for f in fqs]
    return total, st, done, rstats


class _NoPipe:
    max_pairs = 0
