"""Device parity: every HIP kernel against the oracle / reference goldens.

Marked `gpu` (MI355X).  Index build (SA/ISA/LCP/map.bin), index save/load in
the reference's on-disk format, per-read MAM triples, and the whole
read -> bin-count pipeline (counts + varbin stats) incl. multi-batch state.
"""
import hashlib
import os
import shutil

import numpy as np
import pytest

from conftest import gold, interleaved_reads, load_bins, load_chrom_sizes, read_gz_lines

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import smashgpu as S  # noqa: E402
import oracle as O  # noqa: E402


def _sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def sums():
    return {l.split()[0]: (l.split()[1], int(l.split()[2])) for l in open(gold("tiny_index.sha256"))}


@pytest.fixture(scope="module")
def gix(tiny_fa):
    assert torch.cuda.is_available()
    return S.Index.from_fasta(tiny_fa)


def _arrays(ix):
    i = ix.info
    N = i.N
    SA, ISA = ix.download_sa_isa(plain=True)
    L8 = S.download(i.d_lcp8, N)
    ovf = S.download(i.d_lcp_ovf, 16 * i.n_lcp_overflow, np.uint64).reshape(-1, 2)
    mp = S.download(i.d_map, i.map_bytes)
    T = S.download(i.d_text, N)
    return T, SA, ISA, L8, ovf, mp


def test_device_index_matches_reference(gix, tiny_ix, sums):
    T, SA, ISA, L8, ovf, mp = _arrays(gix)
    assert gix.info.idx_bytes == 4
    assert _sha(T.tobytes()) == sums["rc1.ref.seq.bin"][0]
    assert _sha(SA.tobytes()) == sums["rc1.i4.index.sa.bin"][0]
    assert _sha(ISA.tobytes()) == sums["rc1.i4.index.isa.bin"][0]
    assert _sha(L8.tobytes()) == sums["rc1.i4.index.lcp.vec.bin"][0]
    assert _sha(ovf.tobytes()) == sums["rc1.i4.index.lcp.m.bin:masked"][0]
    assert _sha(mp[2:].tobytes()) == sums["map.bin[2:]"][0]
    assert gix.info.logN == O.lib().orc_logN(gix.info.N)


def test_index_save_load_roundtrip(gix, tiny_fa, tmp_path, sums):
    fa = str(tmp_path / "tiny.fa")
    shutil.copy(tiny_fa, fa)
    gix.save(fa)
    d = fa + ".bin/"
    for name in ("rc1.ref.seq.bin", "rc1.ref.bin", "rc1.i4.index.bin", "rc1.i4.index.sa.bin",
                 "rc1.i4.index.isa.bin", "rc1.i4.index.lcp.vec.bin"):
        assert _sha(open(d + name, "rb").read()) == sums[name][0], name
    m = np.fromfile(d + "rc1.i4.index.lcp.m.bin", np.uint64).reshape(-1, 2)
    assert _sha(m.tobytes()) == sums["rc1.i4.index.lcp.m.bin:masked"][0]
    assert _sha(open(d + "map.bin", "rb").read()[2:]) == sums["map.bin[2:]"][0]
    ix2 = S.Index.load(fa)
    a, b = _arrays(gix), _arrays(ix2)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    # without map.bin the loader recomputes it on the device
    os.remove(d + "map.bin")
    ix3 = S.Index.load(fa)
    assert np.array_equal(_arrays(ix3)[5][2:], a[5][2:])


def _device_reads(reads):
    return torch.from_numpy(np.ascontiguousarray(reads)).cuda()


def run_map(ix, reads, min_len=20, mode=S.SMASH_MODE_MAM):
    n, L = reads.shape
    cap = L - min_len + 1
    d = _device_reads(reads)
    out = torch.zeros(n * cap, dtype=torch.int64, device="cuda")
    nn = torch.zeros(n, dtype=torch.int32, device="cuda")
    S.map_batch(ix, d, n, L, out, cap, nn, min_len=min_len, mode=mode)
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.uint64).reshape(n, cap)
    k = nn.cpu().numpy()
    return [S.unpack_matches(o[i], k[i]) for i in range(n)]


def test_device_accelerators_equal_oracle(gix, tiny_ix):
    """U, and the k-mer table with the (k+2)-mer presence bits of the window
    filter (aux_build.hip k_kfilter) == the oracle's orc_build_ktf; every
    B-mer's presence bit == the oracle's B-mer bitmap (B = k + 2)."""
    i = gix.info
    U = S.download(i.d_uniq, i.N + 64)
    KT = S.download(i.d_kmer, 16 << (2 * i.kmer_k), np.uint64)
    U2, KT2, K2 = tiny_ix.accel()
    assert i.kmer_k == K2
    assert np.array_equal(U[:i.N], U2[:i.N])
    assert np.array_equal(KT, tiny_ix._KTF)
    m40 = np.uint64((1 << 40) - 1)
    assert np.array_equal(KT & m40, KT2)
    assert i.bitmap_b == tiny_ix.acc.B == i.kmer_k + 2 and not i.d_bitmap
    B = i.bitmap_b
    codes = np.arange(1 << (2 * B), dtype=np.uint64)
    bm = (tiny_ix._BM[codes >> np.uint64(6)] >> (codes & np.uint64(63))) & np.uint64(1)
    w0 = KT.reshape(-1, 2)[:, 0]
    kt_bits = (w0[codes >> np.uint64(4)] >> (np.uint64(40) + (codes & np.uint64(15)))) & np.uint64(1)
    assert np.array_equal(bm, kt_bits)
    it = [(i.in_text[c >> 6] >> (c & 63)) & 1 for c in range(256)]
    assert it == list(tiny_ix.acc.in_text)


@pytest.mark.parametrize("s", ["s100", "s150"])
@pytest.mark.parametrize("mode", [S.SMASH_MODE_MAM, S.SMASH_MODE_MAM_PLAIN])
def test_mam_matches_reference(gix, s, mode):
    reads = interleaved_reads(s)
    exp = [[tuple(map(int, x.split(","))) for x in l.split()[2:]]
           for l in read_gz_lines("%s_MAM.txt.gz" % s)]
    got = run_map(gix, reads, mode=mode)
    assert len(got) == len(exp)
    bad = [i for i in range(len(exp)) if got[i] != exp[i]]
    assert not bad, (bad[:5], got[bad[0]] if bad else None, exp[bad[0]] if bad else None)


def make_pipe(ix, L, max_pairs, bins_path=None, cs_path=None):
    _, starts = load_bins(bins_path or gold("tiny_bins.txt"))
    cs = load_chrom_sizes(cs_path or gold("tiny_chrom_sizes.txt"))
    return S.Pipeline(ix, cs, starts, L, max_pairs), starts


def run_pipeline(pipe, reads, nbins, batch=None):
    n_pairs = reads.shape[0] // 2
    batch = batch or n_pairs
    counts = torch.zeros(nbins, dtype=torch.int64, device="cuda")
    pipe.reset()
    for b0 in range(0, n_pairs, batch):
        b1 = min(n_pairs, b0 + batch)
        d = _device_reads(reads[2 * b0:2 * b1])
        pipe.count_batch(d, b1 - b0, counts)
    st = pipe.stats()
    return counts.cpu().numpy().astype(np.uint64), st


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_pipeline_matches_reference_varbin(gix, s):
    reads = interleaved_reads(s)
    pipe, starts = make_pipe(gix, reads.shape[1], reads.shape[0] // 2)
    counts, st = run_pipeline(pipe, reads, len(starts))
    assert st.error == 0
    exp = [int(l.split("\t")[3]) for l in open(gold("%s_varbin.txt" % s))]
    assert counts.tolist() == exp
    g = open(gold("%s_varbin_stats_partial.txt" % s)).read().split("\n")[1].split("\t")
    assert (st.positions, st.dups, st.kept) == (int(g[0]), int(g[1]), int(g[2]))
    assert st.pairs == reads.shape[0] // 2
    # smashMEM.py's own summary and positions (the reference script run on the
    # reference's tagged mapout, tools/make_golden_smashmem.sh)
    summ = read_gz_lines("%s_smashmem.txt.gz" % s)[-1]
    assert summ == "%d dupes\t%d non-dupes" % (st.dupe_pairs, st.key_pairs - st.dupe_pairs)
    pos0, absp = pipe.positions()
    name_at = {v: k for k, v in load_chrom_sizes(gold("tiny_chrom_sizes.txt")).items()}
    got = ["%s %d" % (name_at[a - p], p) for p, a in zip(pos0.tolist(), absp.tolist())]
    assert got == open(gold("%s_positions.txt" % s)).read().splitlines()


@pytest.mark.parametrize("batch", [1, 7, 137, 1000])
def test_pipeline_batches_equal_one_pass(gix, batch):
    reads = interleaved_reads("s100")
    pipe, starts = make_pipe(gix, reads.shape[1], 1000)
    c1, s1 = run_pipeline(pipe, reads, len(starts), batch=1000)
    c2, s2 = run_pipeline(pipe, reads, len(starts), batch=batch)
    assert c1.tolist() == c2.tolist()
    assert s1.as_dict() == s2.as_dict()


def test_pipeline_matches_oracle_per_pair(gix, tiny_ix):
    """Per-pair kept hit lists (smashMEM output before de-dup) == oracle."""
    reads = interleaved_reads("s150")
    n = reads.shape[0] // 2
    pipe, starts = make_pipe(gix, reads.shape[1], n)
    run_pipeline(pipe, reads, len(starts))
    nk, keep, hits = pipe.peek(n)
    mapbin = tiny_ix.mappability()
    offs = np.cumsum([0] + [int(x) for x in tiny_ix.sizes[0::2]][:-1]).astype(np.uint32)
    small = [1 if ("_gl000" in c or "chrM" in c) else 0 for c in tiny_ix.contigs]
    for q in range(n):
        hs = []
        for m in (0, 1):
            P = reads[2 * q + m].tobytes()
            h, _ = tiny_ix.resolve(P, tiny_ix.search(P))
            for x in h:
                O.tag(x, offs, mapbin, small[x.tid])
            hs.append(h)
        exp = O.smash_pair(hs[0], hs[1])
        if exp is None:
            assert nk[q] == -1
            continue
        assert nk[q] == len(exp), q
        got = [(int(w >> 48), int(w & 0xFFFFFFFFFFFF)) for w in hits[q, :nk[q]]]
        assert got == exp, q


@pytest.fixture(scope="module")
def mid():
    import synth
    g = synth.make_genome("mid")
    T, sp, sz, names = O.text_from_contigs(g)
    oix = O.Index(T, sp, sz, names)
    dix = S.Index.create(T, sp, sz, names)
    return g, oix, dix


def test_mid_genome_index_equals_oracle(mid):
    g, oix, dix = mid
    T, SA, ISA, L8, ovf, mp = _arrays(dix)
    assert np.array_equal(SA.astype(np.uint64), oix.SA)
    assert np.array_equal(ISA.astype(np.uint64), oix.ISA)
    assert np.array_equal(L8, np.minimum(oix.LCP, 255).astype(np.uint8))
    big = np.nonzero(oix.LCP >= 255)[0]
    assert np.array_equal(ovf[:, 0], big) and np.array_equal(ovf[:, 1], oix.LCP[big])
    assert np.array_equal(mp[2:], oix.mappability()[2:])


def test_mid_genome_pipeline_equals_oracle(mid, tmp_path):
    import synth
    g, oix, dix = mid
    r1, r2 = synth.make_reads(g, 6000, 150, seed=33)
    reads = np.empty((12000, 150), np.uint8)
    reads[0::2], reads[1::2] = r1, r2
    reads = S.prepare_reads(reads)
    # MAM on every read, both device modes
    got = run_map(dix, reads)
    assert got == run_map(dix, reads, mode=S.SMASH_MODE_MAM_PLAIN)
    for i in range(0, len(reads), 7):
        assert got[i] == oix.search(reads[i].tobytes()), i
    bins_path = str(tmp_path / "bins.txt")
    synth.make_bins(g, 16, bins_path)
    synth.write_index_side_files(str(tmp_path), g)
    cs_path = str(tmp_path / "chrom_sizes.txt")
    pipe, starts = make_pipe(dix, 150, 6000, bins_path, cs_path)
    # per-pair smashMEM output and first-wins keep flags vs the oracle
    counts, st = run_pipeline(pipe, reads, len(starts), batch=6000)
    nk, keep, hits = pipe.peek(6000)
    mapbin = oix.mappability()
    offs = np.cumsum([0] + [int(x) for x in oix.sizes[0::2]][:-1]).astype(np.uint32)
    small = [1 if ("_gl000" in c or "chrM" in c) else 0 for c in oix.contigs]
    seen = set()
    for q in range(6000):
        hs = []
        for m in (0, 1):
            P = reads[2 * q + m].tobytes()
            h, _ = oix.resolve(P, oix.search(P))
            for x in h:
                O.tag(x, offs, mapbin, small[x.tid])
            hs.append(h)
        exp = O.smash_pair(hs[0], hs[1])
        if exp is None:
            assert nk[q] == -1, q
            continue
        got = [(int(w >> 48), int(w & 0xFFFFFFFFFFFF)) for w in hits[q, :max(nk[q], 0)]]
        assert got == exp, (q, got, exp)
        k = tuple(exp)
        assert keep[q] == (k not in seen), (q, exp, keep[q])
        seen.add(k)
    c1 = counts
    counts, st = run_pipeline(pipe, reads, len(starts), batch=2500)
    assert counts.tolist() == c1.tolist()
    op = O.Pipeline(oix, oix.mappability(), load_chrom_sizes(cs_path), starts)
    assert op.run(reads, threads=8) == 0
    assert counts.tolist() == op.counts.tolist()
    assert (st.positions, st.dups, st.kept) == (op.state.total, op.state.dups, op.state.kept)
    assert st.dupe_pairs == op.n_dupe.value


@pytest.mark.parametrize("env", [{"SMASH_POST_LEGACY": "1"}, {"SMASH_POST_CAP": "1"},
                                 {"SMASH_POST_CAP": "3"}])
@pytest.mark.parametrize("s", ["s100", "s150"])
def test_post_paths_agree(gix, s, env, monkeypatch):
    """k_post_fast (register lists), its k_post hand-off for mates above the
    capacity, and the general k_post alone give the same per-pair output."""
    reads = interleaved_reads(s)
    n = reads.shape[0] // 2

    def run():
        pipe, starts = make_pipe(gix, reads.shape[1], n)
        counts, st = run_pipeline(pipe, reads, len(starts))
        nk, keep, hits = pipe.peek(n)
        return counts.tolist(), st.as_dict(), nk.copy(), keep.copy(), \
            [hits[q, :max(nk[q], 0)].tolist() for q in range(n)]

    a = run()
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    b = run()
    assert a[0] == b[0] and a[1] == b[1]
    assert np.array_equal(a[2], b[2]) and np.array_equal(a[3], b[3])
    assert a[4] == b[4]


@pytest.mark.parametrize("bits", [2, 9])
def test_key_set_exact_under_hash_collisions(gix, tiny_ix, bits, monkeypatch):
    """The pair-key set compares the canonical hit words, not the hash: with
    the key hash cut to `bits` bits (most keys collide) the counts, stats and
    keep flags still equal the oracle's, whose set holds the full keys."""
    reads = interleaved_reads("s100")
    n = reads.shape[0] // 2
    monkeypatch.setenv("SMASH_KEY_HASH_BITS", str(bits))
    pipe, starts = make_pipe(gix, reads.shape[1], 700)
    monkeypatch.delenv("SMASH_KEY_HASH_BITS")
    counts, st = run_pipeline(pipe, reads, len(starts), batch=700)
    assert st.error == 0
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    op = O.Pipeline(tiny_ix, tiny_ix.mappability(), cs, starts)
    assert op.run(reads, threads=4) == 0
    assert counts.tolist() == op.counts.tolist()
    assert (st.positions, st.dups, st.kept) == (op.state.total, op.state.dups, op.state.kept)
    assert st.dupe_pairs == op.n_dupe.value


@pytest.mark.parametrize("batch", [7, 1000])
@pytest.mark.parametrize("s", ["s100", "s150"])
def test_fused_positions_bins_agree(gix, s, batch, monkeypatch):
    """k_count_last + k_emit_bin (positions and varbin in one pass; global
    atomics, and 16-bit LDS counters with the default and a tiny flush
    threshold) and the two-kernel path (k_emit, then k_bin over the written positions) give the
    same counts, statistics and, read back after every batch, positions
    (the adjacent de-dup line carried across batches both ways)."""
    reads = interleaved_reads(s)
    n = reads.shape[0] // 2

    def run():
        pipe, starts = make_pipe(gix, reads.shape[1], n)
        counts = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
        pos = []
        for b0 in range(0, n, batch):
            b1 = min(n, b0 + batch)
            pipe.count_batch(_device_reads(reads[2 * b0:2 * b1]), b1 - b0, counts)
            p0, pa = pipe.positions()
            pos.append((p0.tolist(), pa.tolist()))
        return counts.cpu().tolist(), pipe.stats().as_dict(), pos

    a = run()
    monkeypatch.setenv("SMASH_BIN_LDS", "0")   # global bin atomics (k_emit_bin), not LDS
    c = run()
    monkeypatch.setenv("SMASH_BIN_LDS", "1")
    monkeypatch.setenv("SMASH_BIN_FLUSH", "2")   # 16-bit LDS counters flushed every 2
    d = run()
    monkeypatch.delenv("SMASH_BIN_FLUSH")
    monkeypatch.setenv("SMASH_FUSED_BIN", "0")
    b = run()
    assert a[1]["error"] == 0
    assert a == b and a == c and a == d
