"""BASELINE.json's configurations on the device, each against an
independent checker.

C1  chr21-only reference, 10 k x 100 bp, sample_bins/500000: the device
    index equals the REFERENCE's own index files byte for byte
    (tests/golden/c1_index.sha256, oracle/_ref/mummer), and the device bin
    counts equal the REAL varbin.py run on the reference's own mapout
    (tests/golden/c1_varbin_*; tools/make_golden_c1.sh).
hg19 (C2, C3, C5) no CPU suffix sort finishes here, so the device index is
    pinned at full size by an independent device checker (tests/csrc/
    index_check.hip: SA a permutation with ISA its inverse, every adjacent
    pair of suffixes in order at its LCP with the first min(LCP, 255) bytes
    equal, the overflow table exact, sampled overflow entries compared in
    full) plus a host-side sample of the same properties; the oracle then
    runs on that (now pinned) index:
    C2  hg19, 1 M x 100 bp (all 500 k pairs), sample_bins/100000
    C3  hg19, 150 bp, sample_bins/50000: a 100 k-pair sample of the bench's
        workload through the oracle; the full 25 M-pair run by properties
    C4  240 k pairs of the 8-GPU workload (seed 4) over W = 8 and W = 3
        emulated ranks with look-ahead (tests/phase_emu.py) == one pipeline
        == the oracle over all of them
    C5  the map.bin self-scan of every forward base == the index build's
        map.bin, and windows of it == the oracle's longSA::show restatement
idx8 the whole count pipeline with 64-bit SA/ISA (the hg19 element width) on
    the mid genome, against an oracle that builds its own index.
"""
import ctypes as C
import hashlib
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, gold

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import smashgpu as S  # noqa: E402
import oracle as O  # noqa: E402
import synth  # noqa: E402

THREADS = min(16, os.cpu_count() or 1)   # the box's CPU share


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _reads(contigs, n_pairs, L, seed):
    r1, r2 = synth.make_reads(contigs, n_pairs, L, seed=seed)
    reads = np.empty((2 * n_pairs, L), np.uint8)
    reads[0::2], reads[1::2] = r1, r2
    return S.prepare_reads(reads)


def _device_counts(dix, cs, starts, reads, batch, rows=False):
    """rows: the mates in the device's native rows (S.to_rows), the layout
    the bench's batches use -- the search DMAs them straight into LDS, and on
    the packed hg19 index at 150 / 100 bp runs the GEO kernels (mam.hip
    run_sm); dense mates go through k_prep's records and the generic kernel"""
    n = reads.shape[0] // 2
    L = reads.shape[1]
    pipe = S.Pipeline(dix, cs, starts, L, min(batch, n), dedup_capacity=n,
                      read_stride=S.read_stride(L) if rows else 0)
    counts = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    pipe.reset()
    for b0 in range(0, n, batch):
        b1 = min(n, b0 + batch)
        d = torch.from_numpy(reads[2 * b0:2 * b1]).cuda()
        pipe.count_batch(S.to_rows(d, L) if rows else d, b1 - b0, counts)
    st = pipe.stats()
    return counts.cpu().numpy().astype(np.uint64), st, pipe


def _oracle_counts(oix, mp, cs, starts, reads):
    op = O.Pipeline(oix, mp, cs, starts)
    err = op.run(reads, threads=THREADS)
    return op, err


# ---------------------------------------------------------------------------
# C1
# ---------------------------------------------------------------------------
def test_c1_chr21_index_and_counts_equal_reference():
    contigs = synth.make_genome("chr21")
    T, sp, sz, names = S.text_from_contigs(contigs)
    dix = S.Index.create(T, sp, sz, names)
    i = dix.info
    assert i.idx_bytes == 4 and i.N == 96259792
    sums = {l.split()[0]: l.split()[1] for l in open(gold("c1_index.sha256"))}
    assert _sha(S.download(i.d_text, i.N)) == sums["rc1.ref.seq.bin"]
    assert _sha(S.download(i.d_sa, 4 * i.N)) == sums["rc1.i4.index.sa.bin"]
    assert _sha(S.download(i.d_isa, 4 * i.N)) == sums["rc1.i4.index.isa.bin"]
    assert _sha(S.download(i.d_lcp8, i.N)) == sums["rc1.i4.index.lcp.vec.bin"]
    ovf = S.download(i.d_lcp_ovf, 16 * i.n_lcp_overflow, np.uint64)
    assert _sha(ovf) == sums["rc1.i4.index.lcp.m.bin:masked"]
    assert _sha(S.download(i.d_map, i.map_bytes)[2:]) == sums["map.bin[2:]"]
    # 5 000 pairs x 100 bp through the device chain, 500 k bins, chr21 at
    # its hg19 offset
    reads = _reads(contigs, 5000, 100, seed=1)
    src = os.path.join(ROOT, "data", "bins", "50000", "bins.txt")
    rows = []
    for line in open(src):
        c = line.rstrip("\n").split("\t")
        a, ab, b = int(c[1]), int(c[2]), int(c[3])
        for k in range(10):
            rows.append(ab + ((b - a) * k) // 10)
    starts = np.array(rows, np.int64)
    counts, st, _ = _device_counts(dix, {"chr21": 2781598825}, starts, reads, 5000)
    assert st.error == 0
    exp = np.zeros(len(starts), np.uint64)
    lines = open(gold("c1_varbin_nonzero.txt")).read().splitlines()
    assert lines[-1] == "rows %d" % len(starts)
    for l in lines[:-1]:
        b, c = l.split("\t")
        exp[int(b)] = int(c)
    assert np.array_equal(counts, exp)
    g = open(gold("c1_varbin_stats_partial.txt")).read().splitlines()[1].split("\t")
    assert (st.positions, st.dups, st.kept) == (int(g[0]), int(g[1]), int(g[2]))


# ---------------------------------------------------------------------------
# hg19: full-size index properties, then C2 / C3 / C5 against the oracle
# ---------------------------------------------------------------------------
class IchkResult(C.Structure):
    _fields_ = [(n, C.c_ulonglong) for n in (
        "perm_bad", "perm_first", "order_bad", "order_first", "ovf_bad", "ovf_first",
        "full_bad", "full_first", "full_checked", "full_bytes", "rank0_ok")]


def _ichk():
    p = os.path.join(ROOT, "tests", "lib", "libindexcheck.so")
    if not os.path.exists(p):
        pytest.fail("tests/lib/libindexcheck.so not built (__graft_entry__.build())")
    L = C.CDLL(p)
    vp = C.c_void_p
    L.ichk_run.argtypes = [vp, C.c_uint64, vp, vp, C.c_uint32, vp, vp, C.c_uint64, C.c_uint64,
                           C.c_uint64, C.POINTER(IchkResult), C.POINTER(C.c_ulonglong)]
    return L


@pytest.fixture(scope="module")
def hg19():
    contigs = synth.make_genome("hg19")
    T, sp, sz, names = S.text_from_contigs(contigs)
    dix = S.Index.create(T, sp, sz, names)
    return contigs, (T, sp, sz, names), dix


def test_hg19_device_index_properties_full_size(hg19):
    """Every rank of the 6.2e9-suffix index (independent device checker)."""
    _, _, dix = hg19
    i = dix.info
    assert i.idx_bytes == 8 and i.N > (1 << 32)
    r = IchkResult()
    n255 = C.c_ulonglong()
    packed = bool(i.pos_bits)
    dix.pack(False)   # (the checker reads plain elements; the hints are checked below)
    try:
        rc = _ichk().ichk_run(i.d_text, i.N, i.d_sa, i.d_isa, i.idx_bytes, i.d_lcp8, i.d_lcp_ovf,
                              i.n_lcp_overflow, 1024, 1 << 16, C.byref(r), C.byref(n255))
    finally:
        dix.pack(packed)
    assert rc == 0
    assert r.rank0_ok == 1
    assert r.perm_bad == 0, r.perm_first
    assert r.order_bad == 0, r.order_first
    assert r.ovf_bad == 0 and n255.value == i.n_lcp_overflow, (r.ovf_first, n255.value)
    assert r.full_bad == 0 and r.full_checked > 100000, (r.full_first, r.full_checked)


def test_hg19_device_index_host_sample(hg19):
    """The same properties on 2 M random ranks, checked on the host from
    gathered values (no device code involved in the comparison)."""
    _, (T, sp, sz, names), dix = hg19
    i = dix.info
    N = i.N
    rng = np.random.default_rng(19)
    ranks = np.unique(rng.integers(1, N, size=2_000_000)).astype(np.int64)
    SA = S.device_view(i.d_sa, 8 * N, torch.int64)
    ISA = S.device_view(i.d_isa, 8 * N, torch.int64)
    L8 = S.device_view(i.d_lcp8, N, torch.uint8)
    r = torch.from_numpy(ranks).cuda()
    pm = dix.pos_mask
    assert i.pos_bits == 33 and pm == (1 << 33) - 1   # hg19: packed index words
    wa = SA.index_select(0, r - 1).cpu().numpy().view(np.uint64)
    wb = SA.index_select(0, r).cpu().numpy().view(np.uint64)
    a = (wa & np.uint64(pm)).astype(np.int64)
    b = (wb & np.uint64(pm)).astype(np.int64)
    wi = ISA.index_select(0, torch.from_numpy(b).cuda()).cpu().numpy().view(np.uint64)
    back = (wi & np.uint64(pm)).astype(np.int64)
    l8 = L8.index_select(0, r).cpu().numpy().astype(np.int64)
    assert np.array_equal(back, ranks)
    # the packed hints of these words (csrc/pack_index.hip; layout in
    # csrc/common.hpp) restated on the host from T and L8 at the same ranks
    idx = torch.from_numpy(np.concatenate([ranks - 2, ranks - 1, ranks, ranks + 1, ranks + 2])
                           .clip(0, N - 1)).cuda()
    near = L8.index_select(0, idx).cpu().numpy().reshape(5, -1).astype(np.uint64)
    cap = np.minimum(near, 127)
    cap[4][ranks + 2 > N - 1] = 0
    cap[3][ranks + 1 > N - 1] = 0
    sa_hint = wb >> np.uint64(36)
    assert np.array_equal(sa_hint & np.uint64(127), cap[2])
    assert np.array_equal((sa_hint >> np.uint64(7)) & np.uint64(127), cap[3])
    isa_hint = wi >> np.uint64(33)
    for q, row in enumerate((1, 2, 3, 4)):   # L8[r - 1 .. r + 2]
        assert np.array_equal((isa_hint >> np.uint64(7 * q)) & np.uint64(127), cap[row]), q
    K = dix.info.kmer_k
    lut = np.full(256, 255, np.uint8)
    for k, ch in enumerate(b"acgt"):
        lut[ch] = k
    x = b
    tag = (wb >> np.uint64(33)) & np.uint64(7)
    bwt = np.where(x > 0, lut[T[np.maximum(x - 1, 0)]], 255)
    win = np.stack([np.where(x + K + k < N, lut[T[np.minimum(x + K + k, N - 1)]], 255)
                    for k in range(7)])
    dirty = (win == 255).any(0)
    assert np.array_equal(tag[dirty], np.full(dirty.sum(), 5, np.uint64))
    clean = ~dirty
    assert np.array_equal(tag[clean], np.where(bwt[clean] < 4, bwt[clean], 4).astype(np.uint64))
    w50 = wb[clean] >> np.uint64(50)
    for k in range(7):
        assert np.array_equal((w50 >> np.uint64(2 * k)) & np.uint64(3), win[k][clean].astype(np.uint64))
    ovf = S.download(i.d_lcp_ovf, 16 * i.n_lcp_overflow, np.uint64).reshape(-1, 2)
    big = l8 == 255
    pos = np.searchsorted(ovf[:, 0], ranks[big].astype(np.uint64))
    assert np.array_equal(ovf[pos, 0], ranks[big].astype(np.uint64))
    lcp = l8.copy()
    lcp[big] = ovf[pos, 1].astype(np.int64)
    for k in range(0, len(ranks), 997):   # byte compares on the host text
        x, y, l = int(a[k]), int(b[k]), int(lcp[k])
        m = min(l, 4096)
        assert T[x:x + m].tobytes() == T[y:y + m].tobytes(), ranks[k]
        assert np.int8(T[x + l]) < np.int8(T[y + l]), ranks[k]


@pytest.fixture(scope="module")
def hg19_oracle(hg19):
    """The oracle over the device index (pinned by the two tests above)."""
    contigs, (T, sp, sz, names), dix = hg19
    i = dix.info
    N = i.N
    SA, ISA = dix.download_sa_isa(plain=True)
    L8 = S.download(i.d_lcp8, N)
    ovf = S.download(i.d_lcp_ovf, 16 * i.n_lcp_overflow, np.uint64).reshape(-1, 2)
    mp = S.download(i.d_map, i.map_bytes)
    oix = O.Index(T, sp, sz, names, SA=SA, ISA=ISA, L8=L8, ovf=ovf)
    return oix, mp


def _chrom_sizes(contigs):
    out, n = {}, 0
    for name, s in contigs:
        if "_" in name:
            continue
        out[name] = n
        n += len(s)
    return out


@pytest.mark.parametrize("cfg,rows", [("c2", False), ("c2", True), ("c3", False), ("c3", True)])
def test_hg19_counts_equal_oracle(hg19, hg19_oracle, cfg, rows, tmp_path):
    """C2 whole / a C3 sample against the oracle, from dense mates (generic
    search kernel) and from native rows (the GEO 100 / GEO 150 kernels)"""
    contigs, _, dix = hg19
    oix, mp = hg19_oracle
    src = os.path.join(ROOT, "data", "bins", "50000", "bins.txt")
    if cfg == "c2":     # all of C2: 1 M mates x 100 bp, the 100 000-bin split
        n, L, seed = 500_000, 100, 2
        path = str(tmp_path / "bins100k.txt")
        synth.split_bins(src, 2, path)
    else:               # a 100 k-pair sample of C3's 150 bp workload, 50 000 bins
        n, L, seed, path = 100_000, 150, 3, src
    starts = np.array([int(l.split("\t")[2]) for l in open(path)], np.int64)
    reads = _reads(contigs, n, L, seed)
    cs = _chrom_sizes(contigs)
    counts, st, pipe = _device_counts(dix, cs, starts, reads, 40_000, rows=rows)
    assert st.error == 0
    assert pipe.map_hints == bool(dix.info.pos_bits)
    op, err = _oracle_counts(oix, mp, cs, starts, reads)
    assert err == 0
    assert np.array_equal(counts, op.counts)
    assert (st.positions, st.dups, st.kept) == (op.state.total, op.state.dups, op.state.kept)
    assert st.dupe_pairs == op.n_dupe.value
    assert st.kept > n   # SMASH reads: several kept segments per pair


def test_c3_full_run_properties(hg19):
    """The C3 run as stated, 25 M pairs (50 M mates) in 2 batches of 12.5 M
    (the bench's split), and again in 4 of 6.25 M and 15 of 1.7 M, with one key
    set and the adjacent-dup state carried: the counts sum to ReadsKept,
    every pair is accounted for, and every batch split gives the same counts
    and stats (the oracle cannot run 50 M reads here)."""
    contigs, _, dix = hg19
    cs = _chrom_sizes(contigs)
    src = os.path.join(ROOT, "data", "bins", "50000", "bins.txt")
    starts = np.array([int(l.split("\t")[2]) for l in open(src)], np.int64)
    import readgen
    P = 25_000_000
    g = readgen.Generator(dix, contigs, 150, seed=3)
    d_reads = g.generate(P)
    outs = []
    torch.cuda.empty_cache()
    for batch in (12_500_000, 6_250_000, 1_700_000):
        pipe = S.Pipeline(dix, cs, starts, 150, batch, dedup_capacity=P)
        counts = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
        pipe.reset()
        for b0 in range(0, P, batch):
            b1 = min(P, b0 + batch)
            pipe.count_batch(d_reads[2 * b0:2 * b1], b1 - b0, counts)
        st = pipe.stats()
        assert st.error == 0 and st.pairs == P
        assert int(counts.sum().item()) == st.kept
        assert st.positions == st.kept + st.dups
        outs.append((counts.cpu().numpy(), st.as_dict()))
        del pipe
    for c, d in outs[1:]:
        assert np.array_equal(outs[0][0], c) and outs[0][1] == d


# ---------------------------------------------------------------------------
# C4's logic at C4's shape on one device: hg19, 150 bp SMASH reads (seed 4),
# sample_bins/50000, ranks emulated in-process (tests/phase_emu.py)
# ---------------------------------------------------------------------------
C4_PAIRS = 240_000


@pytest.fixture(scope="module")
def c4_run(hg19, hg19_oracle):
    """240 k pairs of C4's workload, their single-pipeline counts and the
    oracle's counts over all of them."""
    import readgen
    contigs, _, dix = hg19
    oix, mp = hg19_oracle
    cs = _chrom_sizes(contigs)
    src = os.path.join(ROOT, "data", "bins", "50000", "bins.txt")
    starts = np.array([int(l.split("\t")[2]) for l in open(src)], np.int64)
    d_reads = readgen.Generator(dix, contigs, 150, seed=4).generate(C4_PAIRS)
    one = S.Pipeline(dix, cs, starts, 150, C4_PAIRS, dedup_capacity=C4_PAIRS)
    one.reset()
    c1 = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
    one.count_batch(d_reads, C4_PAIRS, c1)
    s1 = one.stats()
    op, err = _oracle_counts(oix, mp, cs, starts, d_reads.cpu().numpy())
    assert err == 0
    single = (c1.cpu().numpy().astype(np.uint64), (s1.positions, s1.dups, s1.kept, s1.dupe_pairs))
    orc = (op.counts.copy(), (op.state.total, op.state.dups, op.state.kept, op.n_dupe.value))
    return dix, cs, starts, d_reads, single, orc


@pytest.mark.parametrize("W,per_rank,steps,bits,ahead2", [(8, 10_000, 3, 0, True),
                                                          (3, 20_000, 4, 0, True),
                                                          (3, 20_000, 4, 0, False),
                                                          (8, 10_000, 3, 18, True)])
def test_c4_sharded_equals_single_and_oracle(c4_run, W, per_rank, steps, bits, ahead2,
                                             monkeypatch):
    """W ranks (look-ahead search on, as dist.ShardedCounter runs it: the
    next batch with this one, ahead2: the one after right after the export) over
    the same 240 k pairs dealt in (step, rank, pair) order: counts and
    stats equal one pipeline's and the oracle's (smashMEM.py:217-228
    first-wins across ranks, varbin.py:56-58 across shard boundaries).
    bits: the key hash cut to 18 bits, so ~100 k keys collide in it and
    the owners must compare the exchanged key words."""
    from phase_emu import run_emulated
    dix, cs, starts, d_reads, single, orc = c4_run
    assert W * per_rank * steps == C4_PAIRS
    if bits:
        monkeypatch.setenv("SMASH_KEY_HASH_BITS", str(bits))
    total, st = run_emulated(dix, d_reads, W, per_rank, steps, starts, cs, ahead=True,
                             ahead2=ahead2)
    assert orc[1][3] > 100          # duplicate pairs across ranks and steps occur
    assert np.array_equal(total, orc[0]) and st == orc[1]
    assert np.array_equal(single[0], orc[0]) and single[1] == orc[1]


def test_c5_mappability_scan_full_genome(hg19, hg19_oracle):
    contigs, _, dix = hg19
    oix, mp = hg19_oracle
    total = int(sum(dix.contig_sizes))
    out = torch.empty(2 * total, dtype=torch.uint8, device="cuda")
    cc = torch.zeros(len(dix.contigs), dtype=torch.int64, device="cuda")
    S.mappability_scan(dix, 0, total, 36, out, None, None, 0, None, cc)
    dev = out.cpu().numpy()
    assert np.array_equal(dev, mp[2:])        # == the index build's map.bin
    rng = np.random.default_rng(5)
    n_uniq = 0
    for g0 in [0] + [int(x) for x in rng.integers(0, total - 300_000, size=4)]:
        m, u = oix.mappability_range(g0, g0 + 300_000, 36)
        assert np.array_equal(m, dev[2 * g0:2 * (g0 + 300_000)]), g0
        r = dev[2 * g0 + 1:2 * (g0 + 300_000):2]
        assert u == int(((r >= 1) & (r <= 36)).sum())
        n_uniq += u
    assert int(cc.sum().item()) == int(((dev[1::2] >= 1) & (dev[1::2] <= 36)).sum())


def test_c5_prepare_rebuilds_u_full_genome(hg19, hg19_oracle, monkeypatch):
    """C5 from the index arrays at full size (smash_mappability_prepare,
    csrc/uniq_build.hip: 369 level-1 buckets in 12 chunks at hg19): U
    poisoned and rebuilt from SA + L8 by the partition passes equals the
    gather form's U (ISA -> L8, the definition) byte for byte, and the scan
    over it equals the index build's map.bin (built from the exact LCP,
    longSA.cpp:612-690); one rank's eighth (its own window only, the rest of U
    poisoned) equals its slice."""
    contigs, _, dix = hg19
    oix, mp = hg19_oracle
    total = int(sum(dix.contig_sizes))
    N = dix.info.N
    U = S.device_view(dix.info.d_uniq, N + 64, torch.uint8)
    monkeypatch.setenv("SMASH_UNIQ_GATHER", "1")
    S.mappability_prepare(dix, 0, total)
    torch.cuda.synchronize()
    monkeypatch.delenv("SMASH_UNIQ_GATHER")
    gathered = U[:N].clone()
    U[:N].fill_(0x55)
    S.mappability_prepare(dix, 0, total)
    torch.cuda.synchronize()
    assert torch.equal(U[:N], gathered)
    # (SMASH_UPART_2S=1: the pass-2/3 chunks alternating over two streams)
    monkeypatch.setenv("SMASH_UPART_2S", "1")
    U[:N].fill_(0x55)
    S.mappability_prepare(dix, 0, total)
    torch.cuda.synchronize()
    monkeypatch.delenv("SMASH_UPART_2S")
    assert torch.equal(U[:N], gathered)
    del gathered
    out = torch.empty(2 * total, dtype=torch.uint8, device="cuda")
    S.mappability_scan(dix, 0, total, 36, out, None, None, 0, None, None)
    want = torch.from_numpy(mp[2:]).cuda()
    assert torch.equal(out, want)
    keep = U[:N].clone()
    try:
        g0, g1 = total * 3 // 8, total * 4 // 8
        lo, hi = S.mappability_window(dix, g0, g1)
        assert hi - lo < N // 4
        U[:N].fill_(0xAA)
        S.mappability_prepare(dix, g0, g1)
        part = torch.empty(2 * (g1 - g0), dtype=torch.uint8, device="cuda")
        S.mappability_scan(dix, g0, g1, 36, part, None, None, 0, None, None)
        torch.cuda.synchronize()
        assert torch.equal(U[lo:hi], keep[lo:hi])
        assert torch.equal(part, want[2 * g0:2 * g1])
    finally:
        U[:N].copy_(keep)
        S.mappability_prepare(dix, 0, total)
        torch.cuda.synchronize()
        S.mappability_release(dix)   # (the scratch HBM: the later tests' pipelines need it)


def test_c3_mem_hg19_equals_oracle(hg19, hg19_oracle):
    """-maxmatch (memsam's MEM mode, csrc/mem.hip, smash_match_batch) at hg19
    on 20 k of C3's 150 bp SMASH reads: every read's MEM count equals the
    oracle's restatement of longSA::findMEM (longSA.cpp:395-490), and the
    records of the first 4 000 reads equal it in emission order."""
    import readgen
    contigs, _, dix = hg19
    oix, _ = hg19_oracle
    P, L, cap = 10_000, 150, 1024
    n = 2 * P
    d = readgen.Generator(dix, contigs, L, seed=77).generate(P)
    out = torch.zeros(n * cap * 2, dtype=torch.int64, device="cuda")
    nn = torch.zeros(n, dtype=torch.int32, device="cuda")
    S.match_batch(dix, d, n, L, out, cap, nn, mode="MEM")
    torch.cuda.synchronize()
    h = d.cpu().numpy()
    got_n = nn.cpu().numpy()
    tot, per, _ = O.mem_batch(oix, h, threads=THREADS)
    assert got_n.tolist() == per.tolist()
    assert tot > n                                  # several MEMs per SMASH read
    # (a read inside a repeat family has thousands to millions: its records
    # are cut at cap, its count is still exact -- compare the records of the
    # others; 91% of these reads have <= 1 024 MEMs, profiles/r05/ab3)
    assert (got_n <= cap).mean() > 0.8
    o = out.view(n, 2 * cap)[:4000].cpu().numpy().view(np.uint64)
    compared = 0
    for i in range(4000):
        if got_n[i] <= cap:
            assert S.unpack_records(o[i], got_n[i], cap) == oix.search(h[i].tobytes(),
                                                                       mode="MEM"), i
            compared += 1
    assert compared > 3000


# ---------------------------------------------------------------------------
# idx8 on the mid genome: the 64-bit search and chain vs an independent oracle
# ---------------------------------------------------------------------------
def test_idx8_pipeline_equals_independent_oracle(monkeypatch, tmp_path):
    g = synth.make_genome("mid")
    T, sp, sz, names = O.text_from_contigs(g)
    oix = O.Index(T, sp, sz, names)            # the oracle's own suffix sort
    monkeypatch.setenv("SMASH_IDX_BYTES", "8")
    dix = S.Index.create(T, sp, sz, names)
    monkeypatch.delenv("SMASH_IDX_BYTES")
    i = dix.info
    assert i.idx_bytes == 8
    dsa, disa = dix.download_sa_isa(plain=True)
    assert np.array_equal(dsa, oix.SA.astype(np.uint64))
    assert np.array_equal(disa, oix.ISA.astype(np.uint64))
    # the packed words (mid is far below 2^33) equal the host restatement
    sys.path.insert(0, os.path.join(ROOT, "tools", "sm_emu"))
    import sm_emu
    assert i.pos_bits == 33
    psa, pisa = dix.download_sa_isa(plain=False)
    hsa, hisa = sm_emu.pack_words(oix.T, oix.SA, oix.ISA, oix.L8, i.kmer_k)
    assert np.array_equal(psa, hsa) and np.array_equal(pisa, hisa)
    reads = _reads(g, 6000, 150, seed=88)
    # MAM triples of every 5th read
    n = reads.shape[0]
    cap = 150 - 20 + 1
    d = torch.from_numpy(reads).cuda()
    o = torch.zeros(n * cap, dtype=torch.int64, device="cuda")
    nn = torch.zeros(n, dtype=torch.int32, device="cuda")
    S.map_batch(dix, d, n, 150, o, cap, nn)
    torch.cuda.synchronize()
    w = o.cpu().numpy().view(np.uint64).reshape(n, cap)
    k = nn.cpu().numpy()
    for r in range(0, n, 5):
        assert S.unpack_matches(w[r], k[r]) == oix.search(reads[r].tobytes()), r
    bins_path = str(tmp_path / "bins.txt")
    synth.make_bins(g, 16, bins_path)
    synth.write_index_side_files(str(tmp_path), g)
    cs = {l.split("\t")[0]: int(l.split("\t")[2]) for l in open(tmp_path / "chrom_sizes.txt")}
    starts = np.array([int(l.split("\t")[2]) for l in open(bins_path)], np.int64)
    counts, st, pipe = _device_counts(dix, cs, starts, reads, 2500)
    # the device-built map and the index's own tag offsets: the searches
    # hand the post stage each forward match's right map.bin byte
    assert pipe.map_hints
    assert st.error == 0
    op, err = _oracle_counts(oix, oix.mappability(), cs, starts, reads)
    assert err == 0
    assert np.array_equal(counts, op.counts)
    assert (st.positions, st.dups, st.kept) == (op.state.total, op.state.dups, op.state.kept)
    assert st.dupe_pairs == op.n_dupe.value
    # the same per-pair hit lists (one batch, all pairs) with the hints off
    n = reads.shape[0] // 2
    peek = []
    for env in ("1", "0"):
        monkeypatch.setenv("SMASH_MAP_HINT", env)
        c2, st2, p2 = _device_counts(dix, cs, starts, reads, n)
        assert p2.map_hints == (env == "1")
        assert np.array_equal(c2, counts) and st2.as_dict() == st.as_dict()
        peek.append(p2.peek(n))
    monkeypatch.delenv("SMASH_MAP_HINT")
    (nk1, keep1, h1), (nk2, keep2, h2) = peek
    assert np.array_equal(nk1, nk2) and np.array_equal(keep1, keep2)
    for q in np.nonzero(nk1 > 0)[0]:
        assert np.array_equal(h1[q, :nk1[q]], h2[q, :nk1[q]]), q


# ---------------------------------------------------------------------------
# The REAL multi-GPU driver (dist.ShardedCounter.step, dist.count_fastq) on
# C4's workload: W ranks as threads of this process (tests/thread_ranks.py:
# only the transport differs), and one rank over a real RCCL process group
# (the collectives SCALE runs, to itself) -- against the oracle
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("W,per_rank,bits,ahead2", [(8, 10_000, 0, True),
                                                    (3, 20_000, 0, True),
                                                    (3, 20_000, 0, False),
                                                    (8, 10_000, 18, True)])
def test_c4_real_driver_threads_equal_oracle(c4_run, W, per_rank, bits, ahead2, monkeypatch):
    """ShardedCounter.step itself, as bench.py's sharded loop calls it (next
    batch searched with this one, the one after right after the export),
    W ranks over the 240 k pairs == the oracle (smashMEM.py:217-228 first-wins
    across ranks and steps, varbin.py:56-58 across shard boundaries)."""
    from thread_ranks import run_resident
    dix, cs, starts, d_reads, single, orc = c4_run
    if bits:
        monkeypatch.setenv("SMASH_KEY_HASH_BITS", str(bits))
    total, st = run_resident(dix, d_reads, W, per_rank, starts, cs, ahead2=ahead2)
    assert orc[1][3] > 100
    assert st == orc[1], (st, orc[1], single[1])
    assert np.array_equal(total, orc[0])


@pytest.mark.parametrize("W,per_rank,bits,runs", [(3, 20_000, 0, 2), (8, 10_000, 18, 3)])
def test_c4_back_to_back_runs_cross_search(c4_run, W, per_rank, bits, runs, monkeypatch):
    """bench.py's sharded loop over back-to-back runs: each run's last batch
    issues the next run's first two searches (next_reads / next2_reads), and
    the next run's reset keeps them (smash_pipeline_reset_ex,
    SMASH_RESET_KEEP_SEARCH) -- every run's counts and the last run's stats
    == the oracle's (a fresh smashMEM.py + varbin.py run each time)."""
    from thread_ranks import run_resident
    dix, cs, starts, d_reads, single, orc = c4_run
    if bits:
        monkeypatch.setenv("SMASH_KEY_HASH_BITS", str(bits))
    total, st, per_run = run_resident(dix, d_reads, W, per_rank, starts, cs, runs=runs,
                                      cross=True)
    assert st == orc[1], (st, orc[1])
    for k, c in enumerate(per_run):
        assert np.array_equal(c, orc[0]), k


def test_c4_real_driver_variants(c4_run, monkeypatch):
    """The W = 8 driver, and one pipeline over 24 batches (the key records
    written by one launch and compared by later ones), with each kernel form
    the knobs select (SMASH_COOP_COPY=0: per-lane key-word copies instead of
    the wave-cooperative ones; SMASH_BIN_LDS=0: global bin atomics) == the
    oracle, all reported before the first failure is raised (a failing form
    is then named by the others)."""
    from thread_ranks import run_resident
    dix, cs, starts, d_reads, single, orc = c4_run
    res = {}
    for name, env in [("coop0", {"SMASH_COOP_COPY": "0"}), ("binglobal", {"SMASH_BIN_LDS": "0"}),
                      ("default", {})]:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        total, st = run_resident(dix, d_reads, 8, 10_000, starts, cs)
        res[name] = (st, bool(np.array_equal(total, orc[0])))
        for k in env:
            monkeypatch.delenv(k)
    for name, env in [("single_batches", {}), ("single_batches_coop0", {"SMASH_COOP_COPY": "0"})]:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        one = S.Pipeline(dix, cs, starts, 150, 10_000, dedup_capacity=C4_PAIRS)
        one.reset()
        c1 = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
        for b0 in range(0, C4_PAIRS, 10_000):
            one.count_batch(d_reads[2 * b0:2 * (b0 + 10_000)], 10_000, c1)
        s1 = one.stats()
        res[name] = ((s1.positions, s1.dups, s1.kept, s1.dupe_pairs),
                     bool(np.array_equal(c1.cpu().numpy().astype(np.uint64), orc[0])))
        for k in env:
            monkeypatch.delenv(k)
    print("variants:", res, "oracle:", orc[1], "single:", single[1],
          "single counts == oracle:", bool(np.array_equal(single[0], orc[0])))
    assert all(st == orc[1] and eq for st, eq in res.values()), (res, orc[1], single[1])


@pytest.fixture(scope="module")
def c4_fastq(c4_run, tmp_path_factory):
    """C4's 240 k pairs as FASTQ lane files (names r%09d in order): 3 plain
    lanes and 2 gzip lanes per mate."""
    import readgen
    _, _, _, d_reads, _, _ = c4_run
    h = d_reads.cpu().numpy()
    d = tmp_path_factory.mktemp("c4fq")
    cut = 2 * 150_000
    a1, a2 = readgen.write_fastq_lanes(h[:cut], str(d / "plain"), 3)
    b1, b2 = readgen.write_fastq_lanes(h[cut:], str(d / "gz"), 2, gz=True, q0=cut // 2)
    return a1 + b1, a2 + b2


@pytest.mark.parametrize("W,batch", [(3, 30_000), (8, 7_000)])
def test_c4_real_driver_files_threads_equal_oracle(c4_run, c4_fastq, W, batch):
    """dist.count_fastq (every rank its own FastqIndex of the lane lists,
    look-ahead packing, short and empty last shares) == the oracle."""
    from thread_ranks import run_files
    dix, cs, starts, _, _, orc = c4_run
    total, st, done, rs = run_files(dix, c4_fastq, W, batch, starts, cs, capacity=C4_PAIRS)
    assert sum(done) == C4_PAIRS
    assert np.array_equal(total, orc[0]) and st == orc[1]
    # rank-local: each rank packed only its own pairs
    assert [r["pack_pairs"] for r in rs] == done


def _port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_c4_real_driver_rccl_world1_equals_oracle(c4_run, c4_fastq, monkeypatch):
    """One rank over a real nccl (RCCL) process group plus the gloo count
    group, exactly as bench.py --gpus N and smash_cli count set them up:
    the bench's step loop (4 batches, next / next-two search), the same
    with the key hash cut to 18 bits, and dist.count_fastq from the lane
    files -- all == the oracle."""
    import torch.distributed as tdist
    from dist import ShardedCounter, count_fastq, open_fastq
    from thread_ranks import _NoPipe
    dix, cs, starts, d_reads, _, orc = c4_run
    dev = torch.device("cuda", 0)
    tdist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _port(), rank=0,
                             world_size=1, device_id=dev)
    try:
        cg = tdist.new_group(backend="gloo")
        B = 60_000
        nb = C4_PAIRS // B
        for bits in (0, 18):
            if bits:
                monkeypatch.setenv("SMASH_KEY_HASH_BITS", str(bits))
            pipe = S.Pipeline(dix, cs, starts, 150, B, dedup_capacity=C4_PAIRS)
            counts = torch.zeros(len(starts), dtype=torch.int64, device=dev)
            sc = ShardedCounter(pipe, 0, 1, dev, count_group=cg)
            sc.reset()
            for b in range(nb):   # bench.py's sharded loop at world 1
                b0, b1 = b * B, (b + 1) * B
                n0, n1 = b1, min(C4_PAIRS, b1 + B)
                m0, m1 = n1, min(C4_PAIRS, n1 + B)
                sc.step(d_reads[2 * b0:2 * b1], B, b0, counts,
                        d_reads[2 * n0:2 * n1] if n1 > n0 else None, n1 - n0,
                        next2_reads=d_reads[2 * m0:2 * m1] if m1 > m0 else None,
                        next2_pairs=m1 - m0)
            tdist.all_reduce(counts)
            s = pipe.stats()
            assert np.array_equal(counts.cpu().numpy().astype(np.uint64), orc[0]), bits
            assert (s.positions, s.dups, s.kept, s.dupe_pairs) == orc[1], bits
            del pipe
        monkeypatch.delenv("SMASH_KEY_HASH_BITS")
        fq = open_fastq(ShardedCounter(_NoPipe(), 0, 1, dev, count_group=cg), *c4_fastq)
        assert fq.n == C4_PAIRS and isinstance(fq, S.FastqShards)
        pipe = S.Pipeline(dix, cs, starts, fq.L, 70_000, dedup_capacity=C4_PAIRS)
        counts = torch.zeros(len(starts), dtype=torch.int64, device=dev)
        sc = ShardedCounter(pipe, 0, 1, dev, count_group=cg)
        sc.reset()
        assert count_fastq(sc, fq, 70_000, counts) == C4_PAIRS
        tdist.all_reduce(counts)
        s = pipe.stats()
        assert np.array_equal(counts.cpu().numpy().astype(np.uint64), orc[0])
        assert (s.positions, s.dups, s.kept, s.dupe_pairs) == orc[1]
    finally:
        tdist.destroy_process_group()


class _ProductionRun:
    """C3 at the bench's production batch size: 12.6 M pairs of the bench's
    workload (seed 3000, 150 bp, sample_bins/50000) counted as bench.py counts
    a run -- smash_count_batches_ready over batches of 12.5 M pairs (the
    bench's fit_batch choice on one GPU: 3.28e9 hit words per batch, within
    smash_pipeline_max_batch's 2^32 bound), one key set and the adjacent-dup
    state carried into the second, short batch; the oracle's whole chain over
    the same 25.2 M reads is advanced in PARTS parts by the tests below (each
    ~25 s of oracle time on 16 threads, so no test runs silent for minutes;
    the oracle's state carries across its calls)."""
    P, B, PARTS = 12_600_000, 12_500_000, 10

    def __init__(self, hg19, hg19_oracle):
        import readgen
        contigs, _, dix = hg19
        oix, mp = hg19_oracle
        cs = _chrom_sizes(contigs)
        src = os.path.join(ROOT, "data", "bins", "50000", "bins.txt")
        starts = np.array([int(l.split("\t")[2]) for l in open(src)], np.int64)
        P, B = self.P, self.B
        assert B <= S.pipeline_max_batch(150)
        torch.cuda.empty_cache()
        d_reads = readgen.Generator(dix, contigs, 150, seed=3000).generate(P)
        pipe = S.Pipeline(dix, cs, starts, 150, B, dedup_capacity=P + P // 8 + (1 << 20))
        counts = torch.zeros(len(starts), dtype=torch.int64, device="cuda")
        pipe.reset()
        pipe.count_batches(d_reads, P, B, counts, resident=True)
        self.st = pipe.stats()
        self.got = counts.cpu().numpy().astype(np.uint64)
        self.h = d_reads.cpu().numpy()
        del d_reads, pipe
        torch.cuda.empty_cache()
        self.op = O.Pipeline(oix, mp, cs, starts)
        self.done = 0

    def advance(self, k):
        """the oracle over parts 0..k (in order; the ones done are kept)"""
        P, step = self.P, -(-self.P // self.PARTS)
        while self.done <= k:
            a, b = self.done * step, min(P, (self.done + 1) * step)
            assert self.op.run(self.h[2 * a:2 * b], threads=THREADS) == 0
            self.done += 1


@pytest.fixture(scope="module")
def c3_production(hg19, hg19_oracle):
    return _ProductionRun(hg19, hg19_oracle)


@pytest.mark.parametrize("part", range(_ProductionRun.PARTS - 1))
def test_c3_production_batch_oracle_part(c3_production, part):
    c3_production.advance(part)
    assert c3_production.op.state.total > 0


def test_c3_production_batch_equals_oracle(c3_production):
    """the device run at the production batch == the oracle's whole chain
    over the same 12.6 M pairs (smashMEM.py:147-228, varbin.py:52-92)"""
    r = c3_production
    r.advance(r.PARTS - 1)
    st, op = r.st, r.op
    assert st.pairs == r.P
    assert np.array_equal(r.got, op.counts)
    assert (st.positions, st.dups, st.kept) == (op.state.total, op.state.dups, op.state.kept)
    assert st.dupe_pairs == op.n_dupe.value and st.dupe_pairs > 1000
