"""Multi-GPU driver of one read -> bin-count batch (one process per GPU).

Reads shard by contiguous pair ranges: in every step rank r owns global pairs
[base + r*B, base + (r+1)*B), so the global name order (samtools sort -n,
SURVEY.md Appendix A.11) is (step, rank, pair).  Everything is per-rank except
the two dependencies the reference's sequential scripts carry:

* smashMEM.py's global first-wins pair de-dup (smashMEM.py:149,217-228): the
  keyed pairs -- a header {hash, length, word offset} plus the key's
  canonical hit words -- are sent to owner rank = (hash >> 1) % world, each
  owner's segment in pair order (all_to_all of the counts, the headers and
  the words); the receive order (source ranks in rank order) is then the
  global pair order, so the owner decides first-wins in receive order over
  the exact keys against its persistent key set and returns one flag per key
  (all_to_all back);
* varbin.py's adjacent de-dup (varbin.py:56-58) compares with the previous
  emitted position: all_gather of every rank's {count, last pos0} gives each
  rank the last position emitted before its shard.

Bin counts stay per rank until the caller's all_reduce.
`pipe` is a smashgpu.Pipeline (device tensors, RCCL) or any object with the
same phase_* methods (the CPU tests drive this code over gloo with an
oracle-backed stand-in).
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

# SMASH_DIST_TIMING=1: wall time per phase of ShardedCounter.step, each phase
# closed by a device synchronisation (diagnostic only: it removes the
# overlap the step otherwise has); ShardedCounter.timing holds the sums
_TIMING = os.environ.get("SMASH_DIST_TIMING", "0") == "1"


class TorchComm:
    """The step's collectives over torch.distributed: device tensors on
    `group` (RCCL on MI355X), the per-batch key counts -- host integers --
    on `count_group` (gloo: no device synchronisation) when one is given."""

    def __init__(self, device, group=None, count_group=None):
        self.device = device
        self.group = group
        self.count_group = count_group

    def exchange_counts(self, rows):
        """rows[o] = [keys, words] this rank sends owner o; returns what every
        source rank sends this one, as rows in rank order"""
        if self.count_group is not None:
            sc = torch.as_tensor(rows, dtype=torch.int64)
            rc = torch.empty_like(sc)
            dist.all_to_all_single(rc, sc, group=self.count_group)
        else:
            sc = torch.as_tensor(rows, dtype=torch.int64).to(self.device)
            rc = torch.empty_like(sc)
            dist.all_to_all_single(rc, sc, group=self.group)
        return rc.cpu().tolist()

    def all_to_all(self, out, inp, out_splits, in_splits):
        dist.all_to_all_single(out, inp, output_split_sizes=out_splits,
                               input_split_sizes=in_splits, group=self.group)

    def all_gather(self, parts, t):
        dist.all_gather(parts, t, group=self.group)

    def all_gather_bytes(self, b):
        """every rank's byte string, in rank order (the ingest scans)"""
        g = self.count_group if self.count_group is not None else self.group
        dev = torch.device("cpu") if self.count_group is not None else self.device
        W = dist.get_world_size(g)
        n = torch.tensor([len(b)], dtype=torch.int64, device=dev)
        ns = [torch.empty_like(n) for _ in range(W)]
        dist.all_gather(ns, n, group=g)
        sizes = [int(x.item()) for x in ns]
        m = max(max(sizes), 1)
        buf = torch.zeros(m, dtype=torch.uint8, device=dev)
        if b:
            buf[:len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8).to(dev)
        parts = [torch.empty_like(buf) for _ in range(W)]
        dist.all_gather(parts, buf, group=g)
        return [bytes(parts[r][:sizes[r]].cpu().numpy().tobytes()) for r in range(W)]


class KeySetFull(RuntimeError):
    """an owner's pair-key set overflowed (SMASH_ERR_NOMEM): counts past this
    batch would count duplicates again, so the run stops here"""


class ShardedCounter:
    def __init__(self, pipe, rank, world, device, group=None, count_group=None, comm=None,
                 plan_pairs=0, key_slack=1 << 20):
        """count_group: a CPU (gloo) process group for the per-batch key
        counts, which are host integers after smash_phase_export: exchanged
        there they cost no device synchronisation (None: over `group`).
        comm: the collectives (default TorchComm(device, group, count_group));
        tests pass an in-process transport to run W ranks of this exact step
        on one device.
        plan_pairs: the pairs of the whole run over all ranks (0: unknown).
        An owner keeps every key it owns for the whole run, so after the
        first batch's export each rank grows its key set to plan_pairs x
        (its share of that batch's keys) x 1.125 + key_slack -- the owner
        skew measured, not assumed uniform.  Either way a set that overflows
        stops the run at the batch after the one that overflowed it
        (KeySetFull), not after the pass."""
        self.pipe = pipe
        self.rank = rank
        self.world = world
        self.device = device
        self.comm = comm if comm is not None else TorchComm(device, group, count_group)
        self.carried = torch.full((1,), -1, dtype=torch.int64, device=device)
        self.max_pairs = pipe.max_pairs
        self.plan_pairs = int(plan_pairs)
        self.key_slack = int(key_slack)
        self.batch = 0          # batches stepped since the last reset
        self.key_need = 0       # the first batch's projection (plan_pairs > 0)
        # exported since construction: keys / words to every owner, and to
        # the other ranks only (the bytes that cross the links)
        self.sent = {"keys": 0, "words": 0, "remote_keys": 0, "remote_words": 0}
        self.timing = {}
        self._t = None

    def _mark(self, name):
        if not _TIMING:
            return
        if self.device.type != "cpu":
            torch.cuda.synchronize(self.device)
        t = time.perf_counter()
        if self._t is not None:
            self.timing[name] = self.timing.get(name, 0.0) + (t - self._t)
        self._t = t

    def reset(self, keep_search=False):
        """a new run over this communicator (fresh key sets, adjacent-dup state
        and stats).  keep_search: the look-ahead searches the previous run's
        last step issued (its next_reads / next2_reads: this run's first
        batches, resident and unmodified) stay valid, so back-to-back runs
        search the next run's first batches under the last batch's exchange"""
        self.pipe.reset(keep_search=keep_search)
        self.carried.fill_(-1)
        self.batch = 0

    def _size_keys(self, sent, received):
        """grow this owner's key set from the first batch's owner shares
        (all ranks take part: the batch's key total is all-gathered)"""
        tot = sum(int.from_bytes(b, "little")
                  for b in self.comm.all_gather_bytes(int(sent).to_bytes(8, "little")))
        if not tot:
            return
        self.key_need = int(self.plan_pairs * received / tot * 1.125) + self.key_slack
        if self.key_need > self.pipe.key_capacity:
            self.pipe.reserve_keys(self.key_need)

    def _raise(self, err, batch, who):
        import smashgpu as S
        msg = ("pipeline data error %d (%s) on %s by batch %d; this rank's key capacity %d"
               % (err, S.ERRORS.get(err, "?"), who, batch, self.pipe.key_capacity))
        if err == S.SMASH_ERR_NOMEM:
            raise KeySetFull(msg + " (raise dedup_capacity / the plan's pair count)")
        raise S.SmashError(msg)

    def finish(self):
        """the run's end, on every rank together: raise (everywhere) if any
        rank's last owner decisions recorded a data error"""
        err = self.pipe.data_error()
        errs = [int.from_bytes(b, "little", signed=True)
                for b in self.comm.all_gather_bytes(int(err).to_bytes(8, "little", signed=True))]
        if min(errs):
            self._raise(min(errs), self.batch - 1,
                        "rank %d" % self.rank if err else "rank %d" % errs.index(min(errs)))

    def check_keys(self, batch=None):
        """this rank alone (a run's end): raise KeySetFull if the owner
        decisions queued so far recorded a full key set (waits for the
        exchange stream only)"""
        err = self.pipe.data_error()
        if err:
            self._raise(err, self.batch - 1 if batch is None else batch, "rank %d" % self.rank)

    def _recv_counts(self, cnt, wcnt, err=0):
        """what every rank sends me: [keys], [words] per source rank, and
        the largest data error any rank reports (every rank sees every
        rank's: all of them stop together)"""
        rcl = self.comm.exchange_counts([[int(a), int(b), int(err)] for a, b in zip(cnt, wcnt)])
        return [x[0] for x in rcl], [x[1] for x in rcl], min(x[2] for x in rcl)

    def step(self, d_reads, n_pairs, step_base, d_counts, next_reads=None, next_pairs=0,
             stride=None, next2_reads=None, next2_pairs=0):
        """One batch: this rank's n_pairs pairs start at global index
        step_base + rank * stride (stride: the nominal batch of every rank,
        default n_pairs; a short last step keeps the (step, rank, pair)
        order with the nominal stride).  next_reads / next_pairs: the rank's
        next batch, whose search the pipeline starts now, so it runs under
        this batch's exchanges; next2_reads / next2_pairs (with next_*): the
        batch after it, searched as soon as this batch's export has returned
        (its set is free then), so the device holds a queued search while
        the host exchanges this batch's keys.  Every batch must stay
        allocated and unmodified until its own step."""
        dev, W, r = self.device, self.world, self.rank
        p = self.pipe
        self._t = None
        self._mark("start")
        if next_pairs:
            p.phase_map_ahead(d_reads, n_pairs, next_reads, next_pairs)
        else:
            p.phase_map(d_reads, n_pairs)
        self._mark("map")
        hdr, words, cnt, wcnt = p.phase_export(W, step_base + r * (n_pairs if stride is None
                                                                     else stride))
        self._mark("export")
        # the last batch's owner decision ran before this export, which
        # synchronised its stream: its data error (a full key set) travels
        # with the key counts, and every rank stops here together
        err = p.data_error() if self.batch else 0
        if next_pairs and next2_pairs and not err:
            p.phase_search_ahead(next2_reads, next2_pairs)
        rcv, rcw, gerr = self._recv_counts(cnt, wcnt, err)
        if gerr:
            self._raise(gerr, self.batch - 1, "rank %d" % self.rank if err else "another rank")
        if self.batch == 0 and self.plan_pairs:
            self._size_keys(sum(int(x) for x in cnt), sum(rcv))
        self._mark("counts")
        snd, sndw = [int(x) for x in cnt], [int(x) for x in wcnt]
        self.sent["keys"] += sum(snd)
        self.sent["words"] += sum(sndw)
        self.sent["remote_keys"] += sum(snd) - snd[r]
        self.sent["remote_words"] += sum(sndw) - sndw[r]
        n_recv, n_words = sum(rcv), sum(rcw)
        recv = torch.empty((max(n_recv, 1), hdr.shape[1]), dtype=torch.int64, device=dev)
        self.comm.all_to_all(recv[:n_recv], hdr[:sum(snd)], rcv, snd)
        recv_words = torch.empty(max(n_words, 1), dtype=torch.int64, device=dev)
        self.comm.all_to_all(recv_words[:n_words], words[:sum(sndw)], rcw, sndw)
        self._mark("all_to_all_keys")
        flags = torch.empty(max(n_recv, 1), dtype=torch.uint8, device=dev)
        p.dedup_owner(recv, n_recv, recv_words, rcv, rcw, flags)
        self._mark("owner")
        back = torch.empty(max(sum(snd), 1), dtype=torch.uint8, device=dev)
        self.comm.all_to_all(back[:sum(snd)], flags[:n_recv], snd, rcv)
        self._mark("all_to_all_flags")
        p.phase_import(back)
        tail = torch.empty(2, dtype=torch.int64, device=dev)
        p.phase_positions(tail)
        self._mark("import_positions")
        parts = [torch.empty(2, dtype=torch.int64, device=dev) for _ in range(W)]
        self.comm.all_gather(parts, tail)
        tails = torch.stack(parts)
        prev = self._prev(tails[:r], self.carried)
        p.phase_bin(prev, d_counts)
        self.carried = self._prev(tails, self.carried)
        self.batch += 1
        self._mark("tails_bin")

    @staticmethod
    def _prev(tails, carried):
        """last pos0 of the latest non-empty shard among `tails` (rank order),
        else the carried value -- on the device, no host sync."""
        if tails.shape[0] == 0:
            return carried.clone()
        nonempty = tails[:, 0] > 0
        idx = torch.arange(tails.shape[0], device=tails.device)
        last = torch.where(nonempty, idx, torch.full_like(idx, -1)).max()
        pick = tails[last.clamp(min=0), 1].reshape(1)
        return torch.where(last >= 0, pick, carried)


def open_fastq(sc, r1_paths, r2_paths, sort_names=False, threads=0, read_len=0):
    """The FASTQ lists of a multi-GPU run, read rank-locally
    (smashgpu.FastqShards: each rank scans ~1/W of the bytes, the scans are
    all-gathered over the communicator, and each batch is read from only
    its own pairs' bytes).  Input the rank-local reader cannot take (not
    strict 4-line FASTQ, or not in name order when sort_names) goes to
    smashgpu.FastqIndex, which every rank builds over the whole input --
    the same decision on every rank, since every rank sees every scan."""
    import smashgpu as S
    try:
        return S.FastqShards(r1_paths, r2_paths, sc.rank, sc.world, sc.comm.all_gather_bytes,
                             threads=threads, read_len=read_len, sort_names=sort_names)
    except S.SmashError as e:
        if getattr(e, "code", None) != S.SMASH_ERR_UNSUPPORTED:
            raise
    return S.FastqIndex(r1_paths, r2_paths, threads=threads, read_len=read_len,
                        sort_names=sort_names)


def count_fastq(sc, index, batch, d_counts, look_ahead=True, pin=True):
    """File-fed multi-GPU run (smash_mapping.sh:19-29 over `world` ranks):
    every rank holds the same plan of both FASTQ lists (open_fastq: the
    rank-local smashgpu.FastqShards, or smashgpu.FastqIndex; pairs in
    samtools sort -n order) and takes, in step s, planned pairs
    [s W batch + rank batch, + batch): the global name order stays (step,
    rank, pair), which is what ShardedCounter's first-wins de-dup and
    adjacent-dup boundary assume.  Every rank runs the same number of steps
    (an empty share in the last one still joins the collectives).  With
    look_ahead the next batch is packed and copied before this one's
    exchange and its search issued with it.  Returns the pairs this rank
    counted."""
    W, r = sc.world, sc.rank
    n, L = index.n, index.L
    steps = (n + W * batch - 1) // (W * batch)
    dev = sc.device
    on_dev = dev.type != "cpu"
    host = [torch.empty((2 * batch, L), dtype=torch.uint8, pin_memory=pin and on_dev)
            for _ in range(2)]
    devb = [torch.empty((2 * batch, L), dtype=torch.uint8, device=dev) for _ in range(2)]

    def share(s):
        lo = min(n, s * W * batch + r * batch)
        return lo, min(n, lo + batch)

    def load(s, k):   # step s's share into device buffer k (host buffer k reused)
        lo, hi = share(s)
        if hi > lo:
            index.pack(lo, hi, host[k])
            devb[k][:2 * (hi - lo)].copy_(host[k][:2 * (hi - lo)], non_blocking=on_dev)
        return hi - lo

    done = 0
    cur = load(0, 0) if steps else 0
    for s in range(steps):
        k = s % 2
        nxt = 0
        if look_ahead and s + 1 < steps:
            if on_dev:
                torch.cuda.current_stream(dev).synchronize()   # host buffer k ^ 1 is free again
            nxt = load(s + 1, k ^ 1)
        sc.step(devb[k][:2 * cur], cur, s * W * batch, d_counts,
                devb[k ^ 1][:2 * nxt] if nxt else None, nxt, stride=batch)
        done += cur
        if not (look_ahead and s + 1 < steps) and s + 1 < steps:
            nxt = load(s + 1, k ^ 1)
        cur = nxt
    sc.finish()
    return done
