"""world_size-2 run of the multi-GPU exchange (smash-paper_amd/dist.py) over
torch.distributed/gloo on the CPU: the pair-key all_to_all, the tail
all_gather and the count all_reduce must reproduce the single-process
chain exactly (global name order = step, rank, pair)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, gold, interleaved_reads, load_bins, load_chrom_sizes


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, per_rank, steps, out_q, runs=1):
    import sys
    for p in ("oracle", "tools", "tests", "smash-paper_amd"):
        sys.path.insert(0, os.path.join(ROOT, p))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gzip, tempfile
    import oracle as O
    from mock_pipeline import OraclePhasePipeline
    from dist import ShardedCounter
    d = tempfile.mkdtemp()
    fa = os.path.join(d, "tiny.fa")
    with gzip.open(gold("tiny.fa.gz"), "rb") as f, open(fa, "wb") as g:
        g.write(f.read())
    oix = O.Index.from_fasta(fa)
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    pipe = OraclePhasePipeline(oix, oix.mappability(), cs, starts, per_rank)
    sc = ShardedCounter(pipe, rank, world, torch.device("cpu"))
    reads = interleaved_reads("s100")
    counts = torch.zeros(len(starts), dtype=torch.int64)

    def mine(s):
        lo = s * world * per_rank + rank * per_rank
        return torch.from_numpy(reads[2 * lo:2 * (lo + per_rank)].copy())

    out = []
    for run in range(runs):
        # (runs > 1: bench.py's back-to-back runs -- a run's last step passes
        # the next run's first batches as its look-ahead, and the next run's
        # reset keeps them)
        sc.reset(keep_search=run > 0)
        counts.zero_()
        for s in range(steps):
            base = s * world * per_rank
            d_reads = mine(s)
            if s + 1 == steps and run + 1 < runs:
                nxt2 = mine(1) if steps > 1 else None
                sc.step(d_reads, per_rank, base, counts, mine(0), per_rank,
                        next2_reads=nxt2, next2_pairs=per_rank if nxt2 is not None else 0)
            elif s + 1 < steps and s % 2 == 0:   # the look-ahead form (next batch's search issued now)
                nxt = mine(s + 1)
                # and the one after (smash_phase_search_ahead)
                nxt2 = mine(s + 2) if s + 2 < steps else None
                sc.step(d_reads, per_rank, base, counts, nxt, per_rank,
                        next2_reads=nxt2, next2_pairs=per_rank if nxt2 is not None else 0)
            else:
                sc.step(d_reads, per_rank, base, counts)
        c = counts.clone()
        dist.all_reduce(c)
        st = torch.tensor([pipe.total, pipe.dups, pipe.kept], dtype=torch.int64)
        dist.all_reduce(st)
        out.append((c.numpy().tolist(), st.tolist()))
    if rank == 0:
        out_q.put(out[0] if runs == 1 else out)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,per_rank,steps", [(2, 250, 2), (2, 97, 3)])
def test_two_rank_exchange_matches_single_process(world, per_rank, steps, tiny_ix):
    import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per_rank, steps, q))
             for r in range(world)]
    for p in procs:
        p.start()
    import queue as _queue
    res = None
    for _ in range(600):
        try:
            res = q.get(timeout=1)
            break
        except _queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        if res is None:
            p.terminate()
    assert res is not None, [p.exitcode for p in procs]
    got_counts, got_stats = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = world * per_rank * steps
    reads = interleaved_reads("s100")[:2 * n]
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    op = O.Pipeline(tiny_ix, tiny_ix.mappability(), cs, starts)
    assert op.run(reads, threads=4) == 0
    assert got_counts == op.counts.tolist()
    assert got_stats == [op.state.total, op.state.dups, op.state.kept]


def _worker_files(rank, world, port, batch, paths, out_q):
    """the file-fed form: every rank indexes the same FASTQ lists
    (smashgpu.FastqIndex) and counts its (step, rank) batches through
    dist.count_fastq, the key counts exchanged on a gloo count group"""
    import sys
    for p in ("oracle", "tools", "tests", "smash-paper_amd"):
        sys.path.insert(0, os.path.join(ROOT, p))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gzip, tempfile
    import oracle as O
    import smashgpu as S
    from mock_pipeline import OraclePhasePipeline
    from dist import ShardedCounter, count_fastq, open_fastq
    d = tempfile.mkdtemp()
    fa = os.path.join(d, "tiny.fa")
    with gzip.open(gold("tiny.fa.gz"), "rb") as f, open(fa, "wb") as g:
        g.write(f.read())
    oix = O.Index.from_fasta(fa)
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    pipe = OraclePhasePipeline(oix, oix.mappability(), cs, starts, batch)
    cg = dist.new_group(backend="gloo")
    sc = ShardedCounter(pipe, rank, world, torch.device("cpu"), count_group=cg)
    fq = open_fastq(sc, *paths, threads=2)   # the rank-local reader (scans all-gathered over gloo)
    assert isinstance(fq, S.FastqShards)
    counts = torch.zeros(len(starts), dtype=torch.int64)
    sc.reset()
    done = count_fastq(sc, fq, batch, counts)
    rs = fq.stats()
    assert rs["pack_pairs"] == done
    dist.all_reduce(counts)
    st = torch.tensor([pipe.total, pipe.dups, pipe.kept, done], dtype=torch.int64)
    dist.all_reduce(st)
    sc_bytes = torch.tensor([rs["scan_bytes"]], dtype=torch.int64)
    parts = [torch.empty_like(sc_bytes) for _ in range(world)]
    dist.all_gather(parts, sc_bytes)
    if rank == 0:
        out_q.put((counts.numpy().tolist(), st.tolist(), [int(x) for x in parts]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,batch", [(2, 300), (2, 173), (3, 256)])
def test_file_fed_ranks_match_single_process(world, batch, tiny_ix, tmp_path):
    """dist.count_fastq over world ranks (gloo, CPU) on the s100 FASTQ pair,
    split over lane files, == the single-process oracle chain on the same
    pairs read by the streaming reader; the last step's shares are short or
    empty."""
    import gzip
    import oracle as O
    import smashgpu as S
    lanes = []
    for m in (1, 2):
        lines = gzip.open(gold("s100_r%d.fq.gz" % m), "rb").read().split(b"\n")
        cut = 4 * 733
        a, b = tmp_path / ("m%d_L1.fq" % m), tmp_path / ("m%d_L2.fq.gz" % m)
        a.write_bytes(b"\n".join(lines[:cut]) + b"\n")
        with gzip.open(b, "wb") as f:
            f.write(b"\n".join(lines[cut:]))
        lanes.append([str(a), str(b)])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker_files, args=(r, world, port, batch, lanes, q))
             for r in range(world)]
    for p in procs:
        p.start()
    import queue as _queue
    res = None
    for _ in range(900):
        try:
            res = q.get(timeout=1)
            break
        except _queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        if res is None:
            p.terminate()
    assert res is not None, [p.exitcode for p in procs]
    got_counts, got_stats, scanned = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # each rank scanned a share, not the whole input (every byte once in all)
    text = sum(len(gzip.open(p, "rb").read()) if p.endswith(".gz") else len(open(p, "rb").read())
               for p in lanes[0] + lanes[1])
    assert sum(scanned) >= text and all(x < text for x in scanned), (scanned, text)
    _, reads = S.read_fastq_pairs(*lanes)
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    op = O.Pipeline(tiny_ix, tiny_ix.mappability(), cs, starts)
    assert op.run(reads, threads=4) == 0
    assert got_counts == op.counts.tolist()
    assert got_stats == [op.state.total, op.state.dups, op.state.kept, reads.shape[0] // 2]


def _worker_keys(rank, world, port, per_rank, steps, cap, plan, out_q):
    """W ranks with the key hash cut to 2 bits (owners 0 and 1 only: a 1.5x
    skew at W = 3) and a key set of `cap` keys: plan = 0 keeps it (the run
    must stop with KeySetFull right after the batch that overflows it),
    plan > 0 lets ShardedCounter size it from the first batch's owner shares"""
    import sys
    for p in ("oracle", "tools", "tests", "smash-paper_amd"):
        sys.path.insert(0, os.path.join(ROOT, p))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["SMASH_KEY_HASH_BITS"] = "2"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gzip, tempfile
    import oracle as O
    from mock_pipeline import OraclePhasePipeline
    from dist import KeySetFull, ShardedCounter
    d = tempfile.mkdtemp()
    fa = os.path.join(d, "tiny.fa")
    with gzip.open(gold("tiny.fa.gz"), "rb") as f, open(fa, "wb") as g:
        g.write(f.read())
    oix = O.Index.from_fasta(fa)
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    pipe = OraclePhasePipeline(oix, oix.mappability(), cs, starts, per_rank, key_capacity=cap)
    sc = ShardedCounter(pipe, rank, world, torch.device("cpu"), plan_pairs=plan, key_slack=8)
    reads = interleaved_reads("s100")
    counts = torch.zeros(len(starts), dtype=torch.int64)
    sc.reset()
    failed = -1
    try:
        for s_ in range(steps):
            base = s_ * world * per_rank
            lo = base + rank * per_rank
            sc.step(torch.from_numpy(reads[2 * lo:2 * (lo + per_rank)].copy()), per_rank, base,
                    counts)
        sc.finish()
    except KeySetFull:
        failed = sc.batch
    f = torch.tensor([failed, len(pipe.seen), pipe.key_capacity], dtype=torch.int64)
    fs = [torch.empty_like(f) for _ in range(world)]
    dist.all_gather(fs, f)
    if failed < 0:
        dist.all_reduce(counts)
        st = torch.tensor([pipe.total, pipe.dups, pipe.kept], dtype=torch.int64)
        dist.all_reduce(st)
    else:
        st = torch.zeros(3, dtype=torch.int64)
    if rank == 0:
        out_q.put(([x.tolist() for x in fs], counts.numpy().tolist(), st.tolist()))
    dist.destroy_process_group()


def _run_keys(world, per_rank, steps, cap, plan):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker_keys, args=(r, world, port, per_rank, steps, cap, plan, q))
             for r in range(world)]
    for p in procs:
        p.start()
    import queue as _queue
    res = None
    for _ in range(600):
        try:
            res = q.get(timeout=1)
            break
        except _queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        if res is None:
            p.terminate()
        p.join(timeout=60)
    assert res is not None, [p.exitcode for p in procs]
    return res


def test_skewed_owner_overflow_stops_at_the_first_batch():
    """SMASH_KEY_HASH_BITS=2 at W = 3: owners 0 and 1 hold every key.  A set
    sized for the uniform share overflows in batch 0, and the step of batch 1
    stops the run (KeySetFull, smash_pipeline_error) -- not the end of the
    pass; rank 2 owns nothing and stops with the others at the same batch."""
    per_rank, steps = 100, 4
    fs, _, _ = _run_keys(3, per_rank, steps, cap=per_rank // 3, plan=0)
    failed = [f[0] for f in fs]
    assert fs[2][1] == 0                          # owner 2 holds no key
    assert max(f[1] for f in fs[:2]) > per_rank // 3
    assert failed == [1, 1, 1], fs                # every rank stops in batch 1's step


def test_key_set_sized_from_plan_and_first_batch_skew(tiny_ix):
    """plan_pairs given: after batch 0's export every owner grows its set to
    its measured share of the run (owners 0 and 1: ~1/2 each, not 1/3), the
    run completes and equals the single-process chain."""
    import oracle as O
    per_rank, steps, world = 100, 4, 3
    n = world * per_rank * steps
    fs, counts, st = _run_keys(world, per_rank, steps, cap=per_rank // 3, plan=n)
    assert all(f[0] < 0 for f in fs), fs
    assert all(f[1] <= f[2] for f in fs)
    assert fs[0][2] > n // 3 and fs[1][2] > n // 3   # grown past the uniform share
    reads = interleaved_reads("s100")[:2 * n]
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    op = O.Pipeline(tiny_ix, tiny_ix.mappability(), cs, starts)
    assert op.run(reads, threads=4) == 0
    assert counts == op.counts.tolist()
    assert st == [op.state.total, op.state.dups, op.state.kept]


def test_two_rank_back_to_back_runs(tiny_ix):
    """bench.py's sharded loop over back-to-back runs (the last step of a run
    passes the next run's first batches as its look-ahead; the next run's
    reset keeps them, dist.ShardedCounter.reset(keep_search=True)): every run
    over gloo equals the single-process chain."""
    import oracle as O
    import queue as _queue
    world, per_rank, steps, runs = 2, 97, 3, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per_rank, steps, q, runs))
             for r in range(world)]
    for p in procs:
        p.start()
    res = None
    for _ in range(600):
        try:
            res = q.get(timeout=1)
            break
        except _queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        if res is None:
            p.terminate()
    assert res is not None, [p.exitcode for p in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = world * per_rank * steps
    reads = interleaved_reads("s100")[:2 * n]
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    op = O.Pipeline(tiny_ix, tiny_ix.mappability(), cs, starts)
    assert op.run(reads, threads=4) == 0
    assert len(res) == runs
    for got_counts, got_stats in res:
        assert got_counts == op.counts.tolist()
        assert got_stats == [op.state.total, op.state.dups, op.state.kept]
