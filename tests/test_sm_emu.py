"""The device MAM state machine (smash-paper_amd/csrc/mam_sm.hpp: k_prep +
k_mam_sm) compiled for the host as a single-lane emulation (tools/sm_emu) and
checked on the CPU: against the reference's MAM goldens, against the oracle's
restatement of longSA::MAM on edge reads and read lengths, for both SA/ISA
widths.  The GPU tests (test_gpu_parity.py) run the same kernel on MI355X;
this suite pins its control flow without a GPU."""
import os
import sys

import numpy as np
import pytest

from conftest import interleaved_reads, read_gz_lines

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools", "sm_emu"))
import sm_emu  # noqa: E402


@pytest.fixture(scope="module")
def emu(tiny_ix):
    tiny_ix.accel()
    # plain 4-byte, plain 8-byte, and the packed 8-byte words (the device's
    # hg19 index: the search's hints in the SA / ISA words, csrc/common.hpp)
    return sm_emu.Emu(tiny_ix), sm_emu.Emu(tiny_ix, wide=True), sm_emu.Emu(tiny_ix, packed=True)


@pytest.mark.parametrize("s", ["s100", "s150"])
@pytest.mark.parametrize("wide", [0, 1, 2])
@pytest.mark.parametrize("lin", [2, 1])
@pytest.mark.parametrize("bm_dual", ["0", "1", "2", "3"])
def test_state_machine_matches_reference_goldens(emu, s, wide, lin, bm_dual, monkeypatch):
    """lin: L8 blocks scanned per side of a run before bisecting (1 forces
    the bisection path on every run longer than one block); bm_dual: the (F)
    filter loads both B-mer words in one iteration."""
    monkeypatch.setenv("SMASH_SM_BM_DUAL", bm_dual)
    exp = [[tuple(map(int, x.split(","))) for x in l.split()[2:]]
           for l in read_gz_lines("%s_MAM.txt.gz" % s)]
    got, iters = emu[wide].map(interleaved_reads(s), lin_blocks=lin)
    bad = [i for i in range(len(exp)) if got[i] != exp[i]]
    assert not bad, (bad[:5], got[bad[0]] if bad else None, exp[bad[0]] if bad else None)
    assert iters.min() > 0


def _edge_reads(ix, L, n, rng):
    T = ix.T[:ix.N]
    out = np.empty((n, L), np.uint8)
    for i in range(n):
        p = int(rng.integers(0, ix.N - L - 1))
        r = bytearray(T[p:p + L].tobytes())
        for _k in range(int(rng.integers(0, 5))):
            r[int(rng.integers(0, L))] = int(rng.choice(list(b"acgtnz`$N")))
        out[i] = np.frombuffer(bytes(r), np.uint8)
    return out


@pytest.mark.parametrize("L", [15, 32, 33, 100, 128, 129, 150, 255])
@pytest.mark.parametrize("direct", ["1", "0"])
def test_state_machine_edge_reads(emu, tiny_ix, L, direct, monkeypatch):
    """bytes absent from the text, 'n' (present), windows at the read end,
    homopolymers; read lengths around the record/bad-mask boundaries.
    direct: the reads as native rows (the bad mask computed from the LDS
    row, mam_sm.hpp row_bad_mask) or as k_prep records."""
    monkeypatch.setenv("SMASH_SM_DIRECT", direct)
    rng = np.random.default_rng(L)
    reads = _edge_reads(tiny_ix, L, 120, rng)
    extra = [b"z" * L, b"n" * L, b"a" * L, (b"acgt" * 64)[:L], (b"c" * (L // 2) + b"z" + b"c" * L)[:L]]
    reads = np.concatenate([reads, np.array([np.frombuffer(x, np.uint8) for x in extra])])
    for e in (emu[0], emu[2]):
        # (tiny index: K 9, B 11, so min_len 22 / 24 put the filter's window
        # spread D at 11 / 13, where its second entry no longer fits fk)
        for ml, lin in ((20, 2), (12, 2), (30, 2), (20, 1), (12, 1), (22, 2), (24, 2)):
            got, _ = e.map(reads, min_len=ml, lin_blocks=lin)
            for i in range(len(reads)):
                assert got[i] == tiny_ix.search(reads[i].tobytes(), min_len=ml), (e.packed, ml, lin, i)


def test_state_machine_on_mid_genome():
    import oracle as O
    import synth
    g = synth.make_genome("mid")
    ix = O.Index(*O.text_from_contigs(g))
    ix.accel()
    r1, r2 = synth.make_reads(g, 1500, 150, seed=45)
    reads = np.empty((3000, 150), np.uint8)
    reads[0::2], reads[1::2] = r1, r2
    reads[reads == ord("N")] = ord("Z")
    lo = np.arange(256, dtype=np.uint8)
    lo[65:91] += 32
    reads = lo[reads]
    for emu in (sm_emu.Emu(ix), sm_emu.Emu(ix, packed=True)):
        for lin in (2, 1):
            got, _ = emu.map(reads, lin_blocks=lin)
            for i in range(len(reads)):
                assert got[i] == ix.search(reads[i].tobytes()), (emu.packed, lin, i)


def test_packed_words_cut_lines_on_mid_genome():
    """The packed SA / ISA words (csrc/common.hpp) leave every match as it is
    and cut the random lines per read: the BWT character, the L8 bytes around
    a rank and 7 window bases come with the element the search loads anyway."""
    import oracle as O
    import synth
    g = synth.make_genome("mid")
    ix = O.Index(*O.text_from_contigs(g))
    ix.accel()
    r1, r2 = synth.make_reads(g, 1000, 150, seed=46)
    reads = np.empty((2000, 150), np.uint8)
    reads[0::2], reads[1::2] = r1, r2
    lo = np.arange(256, dtype=np.uint8)
    lo[65:91] += 32
    reads = lo[np.where(reads == ord("N"), ord("Z"), reads).astype(np.uint8)]
    plain, packed = sm_emu.Emu(ix, wide=True), sm_emu.Emu(ix, packed=True)
    a, ia = plain.map(reads)
    b, ib = packed.map(reads)
    assert a == b
    la = sum(v[1] for v in plain.counters.values())
    lb = sum(v[1] for v in packed.counters.values())
    assert lb < 0.9 * la, (la / len(reads), lb / len(reads))
    assert packed.counters["lcp"][1] < 0.5 * plain.counters["lcp"][1]
    assert ib.sum() < ia.sum()


@pytest.mark.parametrize("pf", ["0", "1"])
def test_request_accounting(emu, pf, monkeypatch):
    """tools/sm_emu's request count (bench.py roofline: requests_per_read):
    every probe is at least one request, every line transition one of them,
    speculative loads only with the binary-search prefetch (SMASH_SM_PF)."""
    monkeypatch.setenv("SMASH_SM_PF", pf)
    e = emu[1]
    got, _ = e.map(interleaved_reads("s150"))
    lines = sum(v[1] for v in e.counters.values())
    probes = sum(v[0] for v in e.counters.values())
    allr, spec = e.requests
    assert lines <= allr and spec <= allr
    assert (spec > 0) == (pf == "1")
    assert allr <= probes + spec + len(got) * 4   # + the record lines per read
    print("requests/read %.1f (spec %.1f) probes/read %.1f lines/read %.1f" % (
        allr / len(got), spec / len(got), probes / len(got), lines / len(got)))


@pytest.mark.parametrize("L,stride", [(15, 15), (32, 32), (33, 35), (100, 100), (128, 128),
                                      (129, 131), (150, 150), (151, 153), (255, 255)])
@pytest.mark.parametrize("var", [False, True])
def test_prep_direct_equals_lds(L, stride, var):
    """k_prep_direct (the pipeline's default record builder, no LDS) writes
    every word of every record, equal to k_prep's: ACGT and other bytes,
    'N' and case, odd strides (unaligned reads), per-read lengths, the input's
    last read (no load past its last word)."""
    import ctypes as C
    rng = np.random.default_rng(L * 7 + stride + var)
    n = 97
    alphabet = np.frombuffer(b"acgtacgtacgtnNAZ$`", np.uint8)
    buf = alphabet[rng.integers(0, len(alphabet), n * stride)].astype(np.uint8)
    lens = rng.integers(1, L + 1, n).astype(np.uint16) if var else None
    if var:
        lens[:3] = (L, 1, 32 if L >= 32 else L)
    in_text = np.zeros(256, bool)
    for b in b"acgtn":
        in_text[b] = True
    it = sm_emu.in_text_words(in_text)
    g_chunks_max = 4 * (2 + 68)   # words per record, generous
    a = np.zeros(n * g_chunks_max, np.uint32)
    b = np.zeros(n * g_chunks_max, np.uint32)
    rc = sm_emu.lib().sm_emu_prep(
        buf.ctypes.data_as(C.c_void_p), C.c_uint64(stride),
        lens.ctypes.data_as(C.c_void_p) if var else None, C.c_uint32(L), C.c_uint64(n),
        it.ctypes.data_as(C.c_void_p), a.ctypes.data_as(C.c_void_p), b.ctypes.data_as(C.c_void_p))
    assert rc > 0
    w = n * rc
    assert not (a[:w] == 0xDEADBEEF).any()
    bad = np.nonzero(a[:w] != b[:w])[0]
    assert bad.size == 0, (bad[:8] // rc, bad[:8] % rc, a[bad[:8]], b[bad[:8]])
