"""Multi-GPU phase API on one device: W pipelines ("ranks") share one index;
the collectives of smash-paper_amd/dist.py (all_to_all of keys and flags,
all_gather of tails, all_reduce of counts) are emulated in-process with
tensor slicing.  The result must equal one pipeline over the same pairs in
global order (step, rank, pair).  (dist.py itself is run over real
torch.distributed collectives in tests/test_dist_gloo.py.)"""
import numpy as np
import pytest

from conftest import gold, interleaved_reads, load_bins, load_chrom_sizes

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import smashgpu as S  # noqa: E402
from dist import ShardedCounter  # noqa: E402


@pytest.fixture(scope="module")
def gix(tiny_fa):
    return S.Index.from_fasta(tiny_fa)


def _prev(tails, carried):
    return ShardedCounter._prev(tails, carried)


def run_emulated(ix, reads, W, per_rank, steps, starts, cs, ahead=False, capacity=None):
    """capacity: each rank's key-set capacity.  An owner holds every key whose
    hash it owns over the whole run: ~n/W of the n pairs, but ALL of them
    when the hash is cut to a few bits (SMASH_KEY_HASH_BITS; with 2 bits
    every hash is odd, so owner 1 of 2 gets every key).  Default: n."""
    dev = torch.device("cuda")
    n_all = W * per_rank * steps
    pipes = [S.Pipeline(ix, cs, starts, reads.shape[1], per_rank,
                        dedup_capacity=capacity or n_all) for _ in range(W)]
    for p in pipes:
        p.reset()
    counts = [torch.zeros(len(starts), dtype=torch.int64, device=dev) for _ in range(W)]
    carried = torch.full((1,), -1, dtype=torch.int64, device=dev)
    keep_alive, prev_next = [], [None] * W
    for s in range(steps):
        base = s * W * per_rank
        sends = []
        for r in range(W):
            lo = base + r * per_rank
            d = torch.from_numpy(np.ascontiguousarray(reads[2 * lo:2 * (lo + per_rank)])).to(dev)
            # ahead: this batch was searched by the previous step's look-ahead
            cur = prev_next[r] if (ahead and s > 0) else d
            if ahead and s + 1 < steps:
                # the rank's next batch searched now, on the other search stream
                nlo = lo + W * per_rank
                nxt = torch.from_numpy(np.ascontiguousarray(reads[2 * nlo:2 * (nlo + per_rank)])).to(dev)
                keep_alive.append(nxt)
                pipes[r].phase_map_ahead(cur, per_rank, nxt, per_rank)
                prev_next[r] = nxt
            else:
                pipes[r].phase_map(cur, per_rank)
            hdr, words, cnt, wcnt = pipes[r].phase_export(W, base + r * per_rank)
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
            recv = torch.cat(hparts) if sum(rc) else torch.zeros((1, 5), dtype=torch.int64, device=dev)
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


@pytest.mark.parametrize("W,per_rank,steps,bits,ahead", [(2, 500, 2, 0, False),
                                                         (3, 111, 3, 0, False),
                                                         (4, 250, 1, 0, False),
                                                         (3, 200, 2, 3, False),
                                                         (3, 111, 3, 0, True),
                                                         (2, 300, 3, 2, True)])
def test_phases_equal_single_pipeline(gix, W, per_rank, steps, bits, ahead, monkeypatch):
    """bits > 0: the key hash cut to `bits` bits, so owners see colliding
    keys and must compare the exchanged key words."""
    if bits:
        monkeypatch.setenv("SMASH_KEY_HASH_BITS", str(bits))
    reads = interleaved_reads("s100")
    n = W * per_rank * steps
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    one = S.Pipeline(gix, cs, starts, reads.shape[1], n)
    one.reset()
    c1 = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    one.count_batch(torch.from_numpy(np.ascontiguousarray(reads[:2 * n])).cuda(), n, c1)
    s1 = one.stats()
    total, st = run_emulated(gix, reads, W, per_rank, steps, starts, cs, ahead)
    assert total.tolist() == c1.cpu().numpy().astype(np.uint64).tolist()
    assert st == (s1.positions, s1.dups, s1.kept, s1.dupe_pairs)


@pytest.mark.parametrize("batch", [97, 500, 2000])
def test_count_batches_equals_batch_by_batch(gix, batch):
    """smash_count_batches (searches on two alternating streams, each batch's
    search under the previous one's tail) == smash_count_batch per batch."""
    reads = interleaved_reads("s150")
    n = reads.shape[0] // 2
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    d = torch.from_numpy(np.ascontiguousarray(reads)).cuda()
    out = []
    for together in (False, True):
        pipe = S.Pipeline(gix, cs, starts, reads.shape[1], batch, dedup_capacity=n)
        pipe.reset()
        c = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
        if together:
            pipe.count_batches(d, n, batch, c)
        else:
            for b0 in range(0, n, batch):
                b1 = min(n, b0 + batch)
                pipe.count_batch(d[2 * b0:2 * b1], b1 - b0, c)
        st = pipe.stats()
        out.append((c.cpu().numpy().tolist(), st.positions, st.dups, st.kept, st.dupe_pairs))
    assert out[0] == out[1]


def test_full_key_set_fails_loudly(gix, monkeypatch):
    """The round-2 over-count of [2-300-3-2-True]: with the key set sized for
    one batch (per_rank), owner 1 receives all ~1 770 distinct keys of the run
    (2-bit hashes are all odd) into 1 024 slots.  Once the table is full a key
    cannot be inserted, so a later duplicate of it is not found and its pair
    is counted again; which keys miss the table depends on the race for the
    last slots, hence the intermittent failure.  The library records
    SMASH_ERR_NOMEM; the run must fail, never return those counts."""
    monkeypatch.setenv("SMASH_KEY_HASH_BITS", "2")
    reads = interleaved_reads("s100")
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    with pytest.raises(S.SmashError, match="key set full"):
        run_emulated(gix, reads, 2, 300, 3, starts, cs, True, capacity=300)
