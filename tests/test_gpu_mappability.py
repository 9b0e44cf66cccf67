"""The mappability self-scan (BASELINE config C5) on the device:
smash_mappability_scan's map.bin bytes against the reference's map.bin
(`mummer -rcref -mappability`, hashed in tests/golden/tiny_index.sha256) and
the oracle's restatement of longSA::show, for any split of the genome into
ranges (the multi-GPU partition), with 4- and 8-byte ISA; the unique-k-mer
counts per contig and per bin against numpy over the oracle's map.  Marked
`gpu`."""
import hashlib
import os

import numpy as np
import pytest

from conftest import gold

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import smashgpu as S  # noqa: E402
import oracle as O  # noqa: E402


def scan(ix, begin, end, k, off=None, starts=None):
    dev = "cuda"
    out = torch.zeros(max(2 * (end - begin), 1), dtype=torch.uint8, device=dev)
    nc = len(ix.contigs)
    cc = torch.zeros(nc, dtype=torch.int64, device=dev)
    if starts is not None:
        db = torch.from_numpy(np.ascontiguousarray(starts, np.int64)).to(dev)
        bc = torch.zeros(len(starts), dtype=torch.int64, device=dev)
        S.mappability_scan(ix, begin, end, k, out, off, db, len(starts), bc, cc)
    else:
        bc = None
        S.mappability_scan(ix, begin, end, k, out, None, None, 0, None, cc)
    torch.cuda.synchronize()
    return (out.cpu().numpy()[:2 * (end - begin)], cc.cpu().numpy(),
            None if bc is None else bc.cpu().numpy())


def expected_counts(mp, sizes, k, off, starts):
    right = mp[1::2]
    uniq = (right >= 1) & (right <= k)
    cc, bc = [], np.zeros(len(starts), np.int64)
    g = 0
    for q, S_ in enumerate(sizes):
        u = uniq[g:g + S_]
        cc.append(int(u.sum()))
        if off is not None and off[q] >= 0:
            a = off[q] + np.nonzero(u)[0]
            b = np.searchsorted(starts, a, side="right") - 1
            b[b < 0] = len(starts) - 1
            np.add.at(bc, b, 1)
        g += S_
    return np.array(cc), bc


def test_tiny_map_equals_reference(tiny_fa):
    ix = S.Index.from_fasta(tiny_fa)
    total = sum(ix.contig_sizes)
    mp, _, _ = scan(ix, 0, total, 36)
    sums = {l.split()[0]: l.split()[1] for l in open(gold("tiny_index.sha256"))}
    assert hashlib.sha256(mp.tobytes()).hexdigest() == sums["map.bin[2:]"]


@pytest.fixture(scope="module", params=[4, 8])
def mid(request, tmp_path_factory):
    import synth
    g = synth.make_genome("mid")
    T, sp, sz, names = O.text_from_contigs(g)
    oix = O.Index(T, sp, sz, names)
    old = os.environ.get("SMASH_IDX_BYTES")
    os.environ["SMASH_IDX_BYTES"] = str(request.param)
    try:
        dix = S.Index.create(T, sp, sz, names)
    finally:
        if old is None:
            os.environ.pop("SMASH_IDX_BYTES")
        else:
            os.environ["SMASH_IDX_BYTES"] = old
    d = tmp_path_factory.mktemp("mid%d" % request.param)
    synth.write_index_side_files(str(d), g)
    synth.make_bins(g, 16, str(d / "bins.txt"))
    cs = S.read_chrom_sizes(str(d / "chrom_sizes.txt"))
    off = np.array([cs.get(c, -1) if "_" not in c and c != "chrM" else -1
                    for c in dix.contigs], np.int64)
    _, starts = S.read_bins(str(d / "bins.txt"))
    return oix, dix, off, starts


@pytest.mark.parametrize("k", [20, 36])
def test_mid_scan_equals_oracle(mid, k):
    oix, dix, off, starts = mid
    total = sum(dix.contig_sizes)
    omap = oix.mappability()
    mp, cc, bc = scan(dix, 0, total, k, off, starts)
    assert np.array_equal(mp, omap[2:])
    ecc, ebc = expected_counts(omap[2:], dix.contig_sizes, k, off, starts)
    assert cc.tolist() == ecc.tolist()
    assert bc.tolist() == ebc.tolist()
    # the index's own map.bin agrees
    assert np.array_equal(S.download(dix.info.d_map, dix.info.map_bytes)[2:], omap[2:])


@pytest.mark.parametrize("parts", [2, 3, 8])
def test_mid_scan_any_partition(mid, parts):
    oix, dix, off, starts = mid
    total = sum(dix.contig_sizes)
    rng = np.random.default_rng(parts)
    cuts = [0] + sorted(int(x) for x in rng.integers(1, total, parts - 1)) + [total]
    full, fcc, fbc = scan(dix, 0, total, 36, off, starts)
    maps, cc, bc = [], 0, 0
    for a, b in zip(cuts[:-1], cuts[1:]):
        m, c1, b1 = scan(dix, a, b, 36, off, starts)
        maps.append(m)
        cc = cc + c1
        bc = bc + b1
    assert np.array_equal(np.concatenate(maps), full)
    assert np.array_equal(cc, fcc) and np.array_equal(bc, fbc)


def host_uniq(oix):
    """U[x] = min(255, max(LCP[ISA[x]], LCP[ISA[x] + 1])) on the host from the
    oracle's own index (longSA.cpp:628-641 before the +1 and the edge rules)"""
    L8 = oix.L8.astype(np.int64)
    Lp = np.append(L8[1:], 0)
    isa = oix.ISA.astype(np.int64)
    return np.maximum(L8[isa], Lp[isa]).astype(np.uint8)


@pytest.mark.parametrize("form", ["partition", "partition_chunk1", "partition_nt512", "gather"])
def test_prepare_rebuilds_u_from_the_suffix_array(mid, form, monkeypatch):
    """smash_mappability_prepare (C5's preparation from SA + L8,
    csrc/uniq_build.hip): U poisoned on the device, rebuilt for the whole
    genome, equals the host's U from the oracle's ISA + LCP, and the scan over
    it equals the oracle's map.bin (longSA.cpp:612-690); SMASH_UNIQ_GATHER=1
    runs the gather form for A/B; partition_chunk1 the partition with one
    level-1 bucket per pass-2/3 chunk; partition_nt512 passes 1 and 2 in
    tiles of 8 192 entries."""
    oix, dix, off, starts = mid
    if form == "gather":
        monkeypatch.setenv("SMASH_UNIQ_GATHER", "1")
    if form == "partition_chunk1":
        monkeypatch.setenv("SMASH_UPART_E2MB", "1")
    if form == "partition_nt512":
        monkeypatch.setenv("SMASH_UPART_NT", "512")
        monkeypatch.setenv("SMASH_UPART_NT2", "512")
    N = dix.info.N
    U = S.device_view(dix.info.d_uniq, N + 64, torch.uint8)
    want = host_uniq(oix)
    assert np.array_equal(U[:N].cpu().numpy(), want)     # the index build's
    U[:N].fill_(0x55)
    total = sum(dix.contig_sizes)
    S.mappability_prepare(dix, 0, total)
    torch.cuda.synchronize()
    assert np.array_equal(U[:N].cpu().numpy(), want)
    mp, _, _ = scan(dix, 0, total, 36, off, starts)
    assert np.array_equal(mp, oix.mappability()[2:])


@pytest.mark.parametrize("parts", [3, 8])
def test_prepare_per_partition(mid, parts):
    """Each part of a partition of the forward bases (a rank's share of C5)
    rebuilds only its window (its forward and reverse-complement positions)
    and scans it: poisoned U outside the rebuilt windows is never read, the
    concatenated maps equal the oracle's."""
    oix, dix, off, starts = mid
    total = sum(dix.contig_sizes)
    N = dix.info.N
    U = S.device_view(dix.info.d_uniq, N + 64, torch.uint8)
    want = torch.from_numpy(host_uniq(oix)).cuda()
    rng = np.random.default_rng(100 + parts)
    cuts = [0] + sorted(int(x) for x in rng.integers(1, total, parts - 1)) + [total]
    omap = oix.mappability()[2:]
    try:
        for a, b in zip(cuts[:-1], cuts[1:]):
            lo, hi = S.mappability_window(dix, a, b)
            assert 0 <= lo < hi <= N
            U[:N].fill_(0xAA)
            S.mappability_prepare(dix, a, b)
            torch.cuda.synchronize()
            assert torch.equal(U[lo:hi], want[lo:hi]), (a, b, lo, hi)
            m, _, _ = scan(dix, a, b, 36, off, starts)
            assert np.array_equal(m, omap[2 * a:2 * b]), (a, b)
    finally:
        U[:N].copy_(want)
        S.mappability_prepare(dix, 0, total)   # (the directory too)
        torch.cuda.synchronize()
        S.mappability_release(dix)
