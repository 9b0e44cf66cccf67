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


@pytest.fixture(scope="module")
def gix(tiny_fa):
    return S.Index.from_fasta(tiny_fa)


from phase_emu import run_emulated  # noqa: E402


@pytest.mark.parametrize("W,per_rank,steps,bits,ahead", [(2, 500, 2, 0, False),
                                                         (3, 111, 3, 0, False),
                                                         (4, 250, 1, 0, False),
                                                         (3, 200, 2, 3, False),
                                                         (3, 111, 3, 0, True),
                                                         (2, 300, 3, 2, True),
                                                         (3, 111, 4, 0, 2),
                                                         (2, 250, 4, 2, 2)])
def test_phases_equal_single_pipeline(gix, W, per_rank, steps, bits, ahead, monkeypatch):
    """bits > 0: the key hash cut to `bits` bits, so owners see colliding
    keys and must compare the exchanged key words.  ahead: the next batch's
    search issued with this one's (smash_phase_map_ahead); 2: and the batch
    after it right after this one's export (smash_phase_search_ahead)."""
    if bits:
        monkeypatch.setenv("SMASH_KEY_HASH_BITS", str(bits))
    reads = interleaved_reads("s100")
    n = W * per_rank * steps
    assert 2 * n <= reads.shape[0], "the case needs more pairs than s100 holds"
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    one = S.Pipeline(gix, cs, starts, reads.shape[1], n)
    one.reset()
    c1 = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    one.count_batch(torch.from_numpy(np.ascontiguousarray(reads[:2 * n])).cuda(), n, c1)
    s1 = one.stats()
    total, st = run_emulated(gix, reads, W, per_rank, steps, starts, cs, bool(ahead),
                             ahead2=ahead == 2)
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


SCHEDULES = {"default": {},
             # round 3's first form: ev_free after k_post, k_prep_direct
             "post_gate_kpost": {"SMASH_GATE_POST": "0", "SMASH_PREP_LDS": "0"},
             "one_search": {"SMASH_ONE_SEARCH": "1", "SMASH_PRIO": "0"},
             "gate_prep": {"SMASH_GATE_PREP": "1"}}


@pytest.mark.parametrize("sched", sorted(SCHEDULES))
@pytest.mark.parametrize("batch", [97, 2000])
def test_resident_runs_back_to_back(gix, batch, sched, monkeypatch):
    """smash_count_batches_ready (no input event: the searches of a run start
    under the post stage of the run queued before it), three runs queued
    with no synchronisation, each after a reset and a zeroing of its own
    counts: every run's counts == one run of smash_count_batches, under
    each stream schedule (SMASH_GATE_POST / _PREP, SMASH_ONE_SEARCH,
    SMASH_PREP_LDS, SMASH_PRIO: read at pipeline creation / per launch)."""
    for k, v in SCHEDULES[sched].items():
        monkeypatch.setenv(k, v)
    reads = interleaved_reads("s150")
    n = reads.shape[0] // 2
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    d = torch.from_numpy(np.ascontiguousarray(reads)).cuda()
    torch.cuda.synchronize()
    ref = S.Pipeline(gix, cs, starts, reads.shape[1], batch, dedup_capacity=n)
    ref.reset()
    c0 = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    ref.count_batches(d, n, batch, c0)
    st0 = ref.stats()
    pipe = S.Pipeline(gix, cs, starts, reads.shape[1], batch, dedup_capacity=n)
    cs_ = [torch.zeros(len(starts), dtype=torch.int64, device="cuda") for _ in range(3)]
    for c in cs_:
        pipe.reset()
        pipe.count_batches(d, n, batch, c, resident=True)
    st = pipe.stats()
    for c in cs_:
        assert c.cpu().numpy().tolist() == c0.cpu().numpy().tolist()
    assert (st.positions, st.dups, st.kept, st.dupe_pairs) == (
        st0.positions, st0.dups, st0.kept, st0.dupe_pairs)


def test_full_key_set_fails_loudly(gix, monkeypatch):
    """The round-2 over-count of [2-300-3-2-True]: each emulated rank's key
    set was sized for one batch (1 024 slots), while an owner keeps the keys
    it owns for the whole run, and with owner = hash % W (every hash is odd)
    owner 1 of 2 received all ~1 770 distinct keys.  Once its table was full
    a key could not be inserted, so a later duplicate of it was not found and
    its pair was counted again; which keys missed the table depended on the
    race for the last slots, hence the intermittent failure.  The library
    records SMASH_ERR_NOMEM; the run must fail, never return those counts.
    Here: 512 slots per rank, ~890 keys per owner."""
    monkeypatch.setenv("SMASH_KEY_HASH_BITS", "2")
    reads = interleaved_reads("s100")
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    with pytest.raises(S.SmashError, match="key set full"):
        run_emulated(gix, reads, 2, 150, 6, starts, cs, True, capacity=150)


@pytest.mark.parametrize("s", ["s100", "s150"])
@pytest.mark.parametrize("how", ["rows", "rows_records", "rows_phases"])
def test_native_rows_equal_dense(gix, s, how, monkeypatch):
    """The device's native read layout (smash_read_stride rows, zero padded,
    16-byte aligned): the search copies each mate straight from its row and
    the wave computes its bad mask in LDS (mam_sm.hpp direct rows).  Counts
    and statistics equal the dense [2n, L] input's (k_prep records) for
    count_batches, for the same rows through k_prep (SMASH_DIRECT_ROWS=0:
    records built from strided rows), and through the multi-GPU phase calls;
    the per-read MAM triples of smash_map_batch agree too."""
    reads = interleaved_reads(s)
    n = reads.shape[0] // 2
    L = reads.shape[1]
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    dense = torch.from_numpy(np.ascontiguousarray(reads)).cuda()
    rows = S.to_rows(dense)
    assert rows.shape[1] == S.read_stride(L) and rows.shape[1] % 16 == 0
    assert rows.data_ptr() % 16 == 0 and int(rows[:, L:].abs().sum()) == 0
    if how == "rows_records":
        monkeypatch.setenv("SMASH_DIRECT_ROWS", "0")

    def run(d, stride, batch=173):
        pipe = S.Pipeline(gix, cs, starts, L, batch, dedup_capacity=n, read_stride=stride)
        pipe.reset()
        c = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
        if how == "rows_phases" and stride:
            tail = torch.empty(2, dtype=torch.int64, device="cuda")
            for b0 in range(0, n, batch):
                b1 = min(n, b0 + batch)
                pipe.phase_map(d[2 * b0:2 * b1], b1 - b0)
                hdr, words, cnt, wcnt = pipe.phase_export(1, b0)
                flags = torch.empty(max(int(cnt.sum()), 1), dtype=torch.uint8, device="cuda")
                pipe.dedup_owner(hdr.clone(), int(cnt.sum()), words.clone(), cnt, wcnt, flags)
                pipe.phase_import(flags)
                pipe.phase_positions(tail)
                pipe.phase_bin(None, c)
        else:
            pipe.count_batches(d, n, batch, c)
        st = pipe.stats()
        return c.cpu().numpy().tolist(), (st.positions, st.dups, st.kept, st.dupe_pairs, st.matches)

    assert run(rows, rows.shape[1]) == run(dense, 0)
    # smash_map_batch over rows (stride = the native row) == over dense mates
    cap = L - 20 + 1
    got = []
    for d, stride in ((dense, L), (rows, rows.shape[1])):
        o = torch.zeros(2 * n * cap, dtype=torch.int64, device="cuda")
        nn = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
        S.lib().smash_map_batch(gix.h, S.SMASH_MODE_MAM, 20, S._ptr(d), stride, None, L, 2 * n,
                                S._ptr(o), cap, S._ptr(nn), S.vp(torch.cuda.current_stream().cuda_stream))
        torch.cuda.synchronize()
        got.append((o.cpu().numpy().tolist(), nn.cpu().numpy().tolist()))
    assert got[0] == got[1]
