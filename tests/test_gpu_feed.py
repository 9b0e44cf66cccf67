"""File-fed counting (smash_count_fastq, csrc/feed.hip): FASTQ lists ->
pinned batches -> H2D -> count, overlapped.  Its counts and statistics must
equal the batch path (smash_fastq_read + samtools sort -n order +
smash_count_batch) on the same pairs, for gzip and plain input, one and many
batches, input in name order (streamed) and not (buffered + ordered); and it
must refuse what the batch path refuses."""
import gzip

import numpy as np
import pytest

from conftest import gold, load_bins, load_chrom_sizes

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import smashgpu as S  # noqa: E402


@pytest.fixture(scope="module")
def gix(tiny_fa):
    return S.Index.from_fasta(tiny_fa)


@pytest.fixture(scope="module")
def setup():
    _, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    return cs, starts


def _batch_path(gix, cs, starts, names, reads, batch):
    """smash_cli's batch path: samtools sort -n order, smash_count_batch."""
    order = S.strnum_order(names)
    n = len(names)
    reads = reads.reshape(n, -1)[order].reshape(2 * n, -1)
    pipe = S.Pipeline(gix, cs, starts, reads.shape[1], batch, dedup_capacity=n)
    pipe.reset()
    c = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    for b0 in range(0, n, batch):
        b1 = min(n, b0 + batch)
        pipe.count_batch(torch.from_numpy(np.ascontiguousarray(reads[2 * b0:2 * b1])).cuda(),
                         b1 - b0, c)
    st = pipe.stats()
    return c.cpu().numpy().tolist(), (st.pairs, st.key_pairs, st.dupe_pairs, st.positions,
                                      st.dups, st.kept)


def _feed_path(gix, cs, starts, r1, r2, L, batch, sort_names, n):
    pipe = S.Pipeline(gix, cs, starts, L, batch, dedup_capacity=n)
    pipe.reset()
    c = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    fs = pipe.count_fastq(r1, r2, c, sort_names=sort_names, threads=3)
    st = pipe.stats()
    return c.cpu().numpy().tolist(), (st.pairs, st.key_pairs, st.dupe_pairs, st.positions,
                                      st.dups, st.kept), fs


@pytest.mark.parametrize("s", ["s100", "s150"])
@pytest.mark.parametrize("batch", [5000, 37])
def test_feed_sorted_equals_batch_path(gix, setup, s, batch):
    """sort_names=1 reads every pair, orders them and streams the batches
    (gzip input)."""
    cs, starts = setup
    r1, r2 = [gold("%s_r1.fq.gz" % s)], [gold("%s_r2.fq.gz" % s)]
    names, reads = S.read_fastq_pairs(r1, r2)
    exp = _batch_path(gix, cs, starts, names, reads, batch)
    got_c, got_s, fs = _feed_path(gix, cs, starts, r1, r2, reads.shape[1], batch, True,
                                  len(names))
    assert (got_c, got_s) == exp
    assert fs["pairs"] == len(names)
    assert fs["batches"] == -(-len(names) // batch)


def test_feed_batch_knob_below_max_pairs(gix, setup, monkeypatch):
    """SMASH_FEED_BATCH: file-fed batches smaller than the pipeline's
    max_pairs (bench.py feeds 12.5 M-pair pipelines in 6.25 M-pair batches):
    the same counts and statistics as the batch path at that batch size."""
    cs, starts = setup
    r1, r2 = [gold("s150_r1.fq.gz")], [gold("s150_r2.fq.gz")]
    names, reads = S.read_fastq_pairs(r1, r2)
    exp = _batch_path(gix, cs, starts, names, reads, 41)
    monkeypatch.setenv("SMASH_FEED_BATCH", "41")
    got_c, got_s, fs = _feed_path(gix, cs, starts, r1, r2, reads.shape[1], 5000, True,
                                  len(names))
    assert (got_c, got_s) == exp
    assert fs["batches"] == -(-len(names) // 41)


@pytest.mark.parametrize("gz", [False, True])
def test_feed_streams_input_in_name_order(gix, setup, tmp_path, gz):
    """Pairs rewritten in name order (tools/readgen.py write_fastq): the
    streaming mode (sort_names=0) over many small batches, so the two device
    buffers and three pinned slots cycle."""
    import readgen
    cs, starts = setup
    names, reads = S.read_fastq_pairs([gold("s100_r1.fq.gz")], [gold("s100_r2.fq.gz")])
    n = len(names)
    order = S.strnum_order(names)
    srt = reads.reshape(n, -1)[order].reshape(2 * n, -1)
    ext = ".fq.gz" if gz else ".fq"
    p1, p2 = str(tmp_path / ("a" + ext)), str(tmp_path / ("b" + ext))
    readgen.write_fastq(srt, p1, p2, gz=gz)
    new_names = np.array([b"r%012d/1" % i for i in range(n)], "S16")
    exp = _batch_path(gix, cs, starts, new_names, srt, 29)
    got_c, got_s, fs = _feed_path(gix, cs, starts, [p1], [p2], srt.shape[1], 29, False, n)
    assert (got_c, got_s) == exp
    assert fs["batches"] == -(-n // 29)


def test_feed_refuses_unsorted_stream_and_bad_lengths(gix, setup, tmp_path):
    cs, starts = setup
    r1, r2 = [gold("s100_r1.fq.gz")], [gold("s100_r2.fq.gz")]
    names, reads = S.read_fastq_pairs(r1, r2)
    # the first 200 pairs with names in descending order: r10 > r9 numerically
    u1, u2 = tmp_path / "u1.fq", tmp_path / "u2.fq"
    for path, mate in ((u1, 0), (u2, 1)):
        path.write_bytes(b"".join(b"@r%d\n%s\n+\n%s\n" % (
            200 - q, bytes(reads[2 * q + mate]).upper().replace(b"Z", b"N"),
            b"I" * reads.shape[1]) for q in range(200)))
    pipe = S.Pipeline(gix, cs, starts, reads.shape[1], 64, dedup_capacity=len(names))
    c = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    with pytest.raises(S.SmashError, match="sort -n order"):
        pipe.count_fastq([str(u1)], [str(u2)], c, sort_names=False)
    # ordered (sort_names=1), the same pairs count as the batch path does
    exp = _batch_path(gix, cs, starts, np.array([b"r%d" % (200 - q) for q in range(200)], "S8"),
                      reads[:400], 64)
    got_c, got_s, _ = _feed_path(gix, cs, starts, [str(u1)], [str(u2)], reads.shape[1], 64,
                                 True, 200)
    assert (got_c, got_s) == exp
    pipe2 = S.Pipeline(gix, cs, starts, reads.shape[1] + 1, 64, dedup_capacity=len(names))
    with pytest.raises(S.SmashError, match="read length"):
        pipe2.count_fastq(r1, r2, c, sort_names=True)
    a, b = tmp_path / "a.fq", tmp_path / "b.fq"
    a.write_bytes(b"@p1\n" + b"A" * reads.shape[1] + b"\n+\n\n@p2\n\n+\n\n")
    b.write_bytes(b"@p1\n" + b"C" * reads.shape[1] + b"\n+\n\n@p2\n" + b"C" * reads.shape[1] +
                  b"\n+\n\n")
    with pytest.raises(S.SmashError, match="no bases"):
        pipe.count_fastq([str(a)], [str(b)], c, sort_names=True)
    with pytest.raises(S.SmashError, match="cannot open"):
        pipe.count_fastq(["/nonexistent.fq"], r2, c)
    with gzip.open(gold("s100_r1.fq.gz")) as f:
        assert f.read(1) == b"@"


def _lane_files(tmp_path, srt, lanes, kinds, fasta_lane=None):
    """srt's pairs (name order) as len(lanes) lane files per mate: lane k
    holds pairs [lanes[k], lanes[k + 1]), kind 'gz' or 'fq'; fasta_lane: that
    lane of mate 1 written as FASTA (not strict 4-line FASTQ)"""
    p = [[], []]
    cuts = list(lanes) + [srt.shape[0] // 2]
    for m in (0, 1):
        for k in range(len(lanes)):
            recs = []
            for q in range(cuts[k], cuts[k + 1]):
                seq = bytes(srt[2 * q + m]).upper().replace(b"Z", b"N")
                if fasta_lane == k and m == 0:
                    recs.append(b">r%012d/%d\n%s\n" % (q, m + 1, seq))
                else:
                    recs.append(b"@r%012d/%d\n%s\n+\n%s\n" % (q, m + 1, seq, b"I" * len(seq)))
            body = b"".join(recs)
            f = tmp_path / ("m%d_L%d.%s" % (m, k, kinds[k]))
            f.write_bytes(gzip.compress(body, compresslevel=1) if kinds[k] == "gz" else body)
            p[m].append(str(f))
    return p


@pytest.mark.parametrize("fasta_lane", [None, 0, 2])
def test_feed_gzip_lanes_stream_per_file(gix, setup, tmp_path, fasta_lane):
    """gzip lane lists in name order go through the per-file streaming
    producer (files inflated and indexed on worker threads as the pairs need
    them, batches packed from the files already indexed); a lane that is not
    strict FASTQ hands the rest to the streaming reader (lane 2) or, as the
    first lane, the whole input (lane 0) -- the counts are the batch path's
    either way."""
    cs, starts = setup
    names, reads = S.read_fastq_pairs([gold("s150_r1.fq.gz")], [gold("s150_r2.fq.gz")])
    n = len(names)
    srt = reads.reshape(n, -1)[S.strnum_order(names)].reshape(2 * n, -1)
    p = _lane_files(tmp_path, srt, [0, 100, 200, 350, 500], ["gz", "gz", "fq", "gz", "gz"],
                    fasta_lane)
    new_names = np.array([b"r%012d/1" % i for i in range(n)], "S16")
    exp = _batch_path(gix, cs, starts, new_names, srt, 101)
    got_c, got_s, fs = _feed_path(gix, cs, starts, p[0], p[1], srt.shape[1], 101, False, n)
    assert (got_c, got_s) == exp
    assert fs["pairs"] == n
    if fasta_lane is None:
        assert fs["parallel"] == 1


def test_feed_gzip_lanes_refuse_disorder_and_bad_length(gix, setup, tmp_path):
    cs, starts = setup
    names, reads = S.read_fastq_pairs([gold("s100_r1.fq.gz")], [gold("s100_r2.fq.gz")])
    n = len(names)
    srt = reads.reshape(n, -1)[S.strnum_order(names)].reshape(2 * n, -1)
    rev = srt.reshape(n, -1)[::-1].reshape(2 * n, -1)   # names ascend, reads do not matter
    p = _lane_files(tmp_path, rev, [0, 500], ["gz", "gz"])
    # swap the two lanes of both mates: names out of order at lane 2's first
    p = [p[0][::-1], p[1][::-1]]
    pipe = S.Pipeline(gix, cs, starts, srt.shape[1], 64, dedup_capacity=n)
    c = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    with pytest.raises(S.SmashError, match="sort -n order"):
        pipe.count_fastq(p[0], p[1], c, sort_names=False)
    q = _lane_files(tmp_path, srt[:, :-1].copy(), [0, 300], ["gz", "gz"])
    with pytest.raises(S.SmashError, match="read length"):
        pipe.count_fastq(q[0], q[1], c, sort_names=False)


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_feed_grows_key_set_from_one_batch(gix, setup, s):
    """A gzip input's pair count is unknown before it is inflated, so smash_cli
    starts the key set at one batch and smash_count_fastq grows it (doubling,
    the held keys rehashed into the larger set) before a batch could overflow
    it: counts, duplicates and statistics equal the batch path's with a set
    sized for every pair, over many small batches (several growths)."""
    cs, starts = setup
    r1, r2 = [gold("%s_r1.fq.gz" % s)], [gold("%s_r2.fq.gz" % s)]
    names, reads = S.read_fastq_pairs(r1, r2)
    n, batch = len(names), 23
    exp = _batch_path(gix, cs, starts, names, reads, batch)
    pipe = S.Pipeline(gix, cs, starts, reads.shape[1], batch, dedup_capacity=1)
    cap0 = pipe.key_capacity
    assert cap0 < n
    pipe.reset()
    c = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    pipe.count_fastq(r1, r2, c, sort_names=True, threads=3)
    st = pipe.stats()
    assert st.error == 0
    got = (c.cpu().numpy().tolist(), (st.pairs, st.key_pairs, st.dupe_pairs, st.positions,
                                      st.dups, st.kept))
    assert got == exp
    assert pipe.key_capacity >= n > cap0


def test_reserve_keys_moves_held_keys(gix, setup):
    """smash_pipeline_reserve_keys on a set that holds keys: a second pass of
    the same pairs after the growth finds every keyed pair a duplicate (the
    keys and their records moved), and the counts gain nothing."""
    cs, starts = setup
    names, reads = S.read_fastq_pairs([gold("s150_r1.fq.gz")], [gold("s150_r2.fq.gz")])
    n = len(names)
    d = torch.from_numpy(np.ascontiguousarray(reads)).cuda()
    pipe = S.Pipeline(gix, cs, starts, reads.shape[1], n, dedup_capacity=n)
    pipe.reset()
    c = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    pipe.count_batch(d, n, c)
    st1 = pipe.stats()
    first = c.cpu().numpy().copy()
    pipe.reserve_keys(8 * n)
    assert pipe.key_capacity >= 8 * n
    pipe.count_batch(d, n, c)
    st2 = pipe.stats()
    assert st2.error == 0
    assert st2.dupe_pairs - st1.dupe_pairs == st1.key_pairs
    assert np.array_equal(c.cpu().numpy(), first)
