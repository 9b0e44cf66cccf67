"""Device parity of memsam's other search modes: -maxmatch (MEM, findMEM) and
-mum (MUM), plus MAM through the unpacked smash_match_batch records.

Pinned to the reference's own per-read triples (tests/golden/s{100,150}_
{MAM,MUM,MEM}.txt.gz, written by the compiled reference through
oracle/ref_harness.cpp) in emission order, and to the oracle's restatement on
a repeat-rich mid-size genome with 4- and 8-byte SA/ISA, including reads made
of repeats (thousands of MEMs), N runs and text separators.  Marked `gpu`.
"""
import os

import numpy as np
import pytest

from conftest import interleaved_reads, read_gz_lines

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import smashgpu as S  # noqa: E402
import oracle as O  # noqa: E402


def run_match(ix, reads, mode, cap=512, min_len=20):
    n, L = reads.shape
    d = torch.from_numpy(np.ascontiguousarray(reads)).cuda()
    out = torch.zeros(n * cap * 2, dtype=torch.int64, device="cuda")
    nn = torch.zeros(n, dtype=torch.int32, device="cuda")
    S.match_batch(ix, d, n, L, out, cap, nn, mode=mode, min_len=min_len)
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.uint64).reshape(n, 2 * cap)
    k = nn.cpu().numpy()
    return [S.unpack_records(o[i], k[i], cap) for i in range(n)], k


@pytest.fixture(scope="module")
def gix(tiny_fa):
    return S.Index.from_fasta(tiny_fa)


@pytest.mark.parametrize("s", ["s100", "s150"])
@pytest.mark.parametrize("mode", ["MAM", "MUM", "MEM"])
def test_modes_match_reference_triples(gix, s, mode):
    reads = interleaved_reads(s)
    exp = [[tuple(map(int, x.split(","))) for x in l.split()[2:]]
           for l in read_gz_lines("%s_%s.txt.gz" % (s, mode))]
    got, n = run_match(gix, reads[:len(exp)], mode, cap=16384)
    assert max(n) <= 16384
    bad = [i for i in range(len(exp)) if got[i] != exp[i]]
    assert not bad, (bad[:5], got[bad[0]] if bad else None, exp[bad[0]] if bad else None)


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_mum_packed_equals_records(gix, s):
    reads = interleaved_reads(s)
    n, L = reads.shape
    cap = L
    d = torch.from_numpy(reads).cuda()
    out = torch.zeros(n * cap, dtype=torch.int64, device="cuda")
    nn = torch.zeros(n, dtype=torch.int32, device="cuda")
    S.map_batch(gix, d, n, L, out, cap, nn, mode=S.SMASH_MODE_MUM)
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.uint64).reshape(n, cap)
    k = nn.cpu().numpy()
    packed = [S.unpack_matches(o[i], k[i]) for i in range(n)]
    rec, _ = run_match(gix, reads, "MUM")
    assert packed == rec


def test_mem_rejected_by_packed_entry(gix):
    reads = interleaved_reads("s100")[:4]
    d = torch.from_numpy(reads).cuda()
    out = torch.zeros(4 * 100, dtype=torch.int64, device="cuda")
    nn = torch.zeros(4, dtype=torch.int32, device="cuda")
    with pytest.raises(S.SmashError):
        S.map_batch(gix, d, 4, 100, out, 100, nn, mode=S.SMASH_MODE_MEM)


def _edge_reads(T, L, n, rng):
    out = np.empty((n, L), np.uint8)
    N = len(T)
    for i in range(n):
        kind = i % 5
        if kind == 0:                              # a stretch of one repeat family copy
            p = int(rng.integers(0, N - L - 1))
            r = bytearray(T[p:p + L].tobytes())
        elif kind == 1:                            # low complexity (many MEMs)
            r = bytearray((b"ac" * L)[:L]) if i % 2 else bytearray(b"a" * L)
        elif kind == 2:                            # chimeric, 20-60 bp pieces
            r = bytearray()
            while len(r) < L:
                p = int(rng.integers(0, N - 80))
                r += T[p:p + int(rng.integers(20, 61))].tobytes()
            r = r[:L]
        else:                                      # mutated copy with N / separators
            p = int(rng.integers(0, N - L - 1))
            r = bytearray(T[p:p + L].tobytes())
            for _ in range(int(rng.integers(0, 6))):
                r[int(rng.integers(0, L))] = int(rng.choice(list(b"acgtnz`$")))
        out[i] = np.frombuffer(bytes(r[:L]), np.uint8)
    return out


@pytest.fixture(scope="module", params=[4, 8])
def mid(request):
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
    assert dix.info.idx_bytes == request.param
    return T, oix, dix


@pytest.mark.parametrize("L", [100, 150])
@pytest.mark.parametrize("mode", ["MEM", "MUM"])
def test_modes_equal_oracle_mid_genome(mid, mode, L):
    T, oix, dix = mid
    rng = np.random.default_rng(L + len(mode))
    reads = _edge_reads(T[:-1], L, 400, rng)
    cap = 4096
    got, n = run_match(dix, reads, mode, cap=cap)
    for i in range(len(reads)):
        exp = oix.search(reads[i].tobytes(), mode)
        assert n[i] == len(exp), (i, mode)
        assert got[i] == exp[:cap], (i, mode, reads[i].tobytes()[:40])


@pytest.mark.parametrize("defer", ["0", "2", "64"])
@pytest.mark.parametrize("cap", [37, 4096])
def test_mem_deferred_collect_equal_oracle(mid, defer, cap, monkeypatch):
    """collectMEMs calls over >= SMASH_MEM_DEFER ranks run as wave jobs
    (csrc/mem.hip k_mem_jobs) and their records are placed around the lane's
    own (k_mem_fix): the records, cut at cap, and the counts equal the
    oracle's for every threshold (0: none deferred; 2: nearly every call)."""
    T, oix, dix = mid
    monkeypatch.setenv("SMASH_MEM_DEFER", defer)
    rng = np.random.default_rng(7)
    reads = _edge_reads(T[:-1], 150, 300, rng)
    got, n = run_match(dix, reads, "MEM", cap=cap)
    for i in range(len(reads)):
        exp = oix.search(reads[i].tobytes(), "MEM")
        assert n[i] == len(exp), (i, defer, cap)
        assert got[i] == exp[:cap], (i, defer, cap)


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_mem_deferred_matches_reference_triples(gix, s, monkeypatch):
    """the reference's own MEM triples with nearly every collectMEMs call
    deferred to the wave jobs (SMASH_MEM_DEFER=2)"""
    monkeypatch.setenv("SMASH_MEM_DEFER", "2")
    reads = interleaved_reads(s)
    exp = [[tuple(map(int, x.split(","))) for x in l.split()[2:]]
           for l in read_gz_lines("%s_MEM.txt.gz" % s)]
    got, n = run_match(gix, reads[:len(exp)], "MEM", cap=16384)
    bad = [i for i in range(len(exp)) if got[i] != exp[i]]
    assert not bad, (bad[:5], got[bad[0]] if bad else None, exp[bad[0]] if bad else None)
