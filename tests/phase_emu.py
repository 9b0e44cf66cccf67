"""In-process emulation of W ranks of the multi-GPU phase API on ONE device
(test infrastructure): W pipelines share one index; the collectives of
smash-paper_amd/dist.py (all_to_all of keys and flags, all_gather of tails,
all_reduce of counts) become tensor slicing.  Global order is (step, rank,
pair), as dist.ShardedCounter deals it."""
import numpy as np
import torch

import smashgpu as S
from dist import ShardedCounter


def _rows(reads, a, b, dev):
    """mates [a, b) of `reads` (numpy host array or device tensor) on dev"""
    if isinstance(reads, torch.Tensor):
        return reads[a:b].to(dev)
    return torch.from_numpy(np.ascontiguousarray(reads[a:b])).to(dev)


def _prev(tails, carried):
    return ShardedCounter._prev(tails, carried)


def run_emulated(ix, reads, W, per_rank, steps, starts, cs, ahead=False, capacity=None,
                 ahead2=False):
    """reads: [2n, L] mates (numpy or a device tensor), n = W * per_rank *
    steps pairs in global order.  ahead: each rank's next batch is searched
    by smash_phase_map_ahead; ahead2 (with ahead): and the batch after it by
    smash_phase_search_ahead right after the export.  capacity: each rank's key-set capacity; an
    owner holds every key whose hash it owns over the whole run, ~n/W of the
    pairs, and up to all of them when SMASH_KEY_HASH_BITS cuts the hash to
    a few values.  Default: n.  Returns (summed counts, summed stats)."""
    dev = torch.device("cuda")
    n_all = W * per_rank * steps
    pipes = [S.Pipeline(ix, cs, starts, reads.shape[1], per_rank,
                        dedup_capacity=capacity or n_all) for _ in range(W)]
    for p in pipes:
        p.reset()
    counts = [torch.zeros(len(starts), dtype=torch.int64, device=dev) for _ in range(W)]
    carried = torch.full((1,), -1, dtype=torch.int64, device=dev)
    batches = {}   # (rank, step) -> its reads on the device, kept alive for the run

    def batch(r, s):
        if (r, s) not in batches:
            lo = s * W * per_rank + r * per_rank
            batches[(r, s)] = _rows(reads, 2 * lo, 2 * (lo + per_rank), dev)
        return batches[(r, s)]

    for s in range(steps):
        base = s * W * per_rank
        sends = []
        for r in range(W):
            # ahead: this batch was searched by the previous step's look-ahead
            cur = batch(r, s)
            if ahead and s + 1 < steps:
                # the rank's next batch searched now, on the other search stream
                pipes[r].phase_map_ahead(cur, per_rank, batch(r, s + 1), per_rank)
            else:
                pipes[r].phase_map(cur, per_rank)
            hdr, words, cnt, wcnt = pipes[r].phase_export(W, base + r * per_rank)
            if ahead and ahead2 and s + 2 < steps:
                pipes[r].phase_search_ahead(batch(r, s + 2), per_rank)
            # copies: the export buffers are the pipeline's own
            sends.append((hdr.clone(), words.clone(), [int(c) for c in cnt],
                          [int(c) for c in wcnt]))
        # all_to_all: owner o receives segment o of every rank, rank order
        flags_back = [[None] * W for _ in range(W)]
        for o in range(W):
            hparts, wparts, rc, rw = [], [], [], []
            for r in range(W):
                hdr, words, cnt, wcnt = sends[r]
                h0, w0 = sum(cnt[:o]), sum(wcnt[:o])
                hparts.append(hdr[h0:h0 + cnt[o]])
                wparts.append(words[w0:w0 + wcnt[o]])
                rc.append(cnt[o])
                rw.append(wcnt[o])
            recv = torch.cat(hparts) if sum(rc) else torch.zeros((1, sends[0][0].shape[1]), dtype=torch.int64, device=dev)
            rwords = torch.cat(wparts) if sum(rw) else torch.zeros(1, dtype=torch.int64, device=dev)
            n = sum(rc)
            flags = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
            pipes[o].dedup_owner(recv, n, rwords, rc, rw, flags)
            k = 0
            for r in range(W):
                m = rc[r]
                flags_back[r][o] = flags[k:k + m]
                k += m
        cnts = [x[2] for x in sends]
        tails = []
        for r in range(W):
            back = torch.cat(flags_back[r]) if sum(cnts[r]) else torch.zeros(1, dtype=torch.uint8, device=dev)
            pipes[r].phase_import(back)
            tail = torch.empty(2, dtype=torch.int64, device=dev)
            pipes[r].phase_positions(tail)
            tails.append(tail)
        T = torch.stack(tails)
        for r in range(W):
            pipes[r].phase_bin(_prev(T[:r], carried), counts[r])
        carried = _prev(T, carried)
    total = sum(c.cpu().numpy().astype(np.uint64) for c in counts)
    st = [p.stats() for p in pipes]
    return total, (sum(x.positions for x in st), sum(x.dups for x in st),
                   sum(x.kept for x in st), sum(x.dupe_pairs for x in st))
