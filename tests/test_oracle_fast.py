"""The accelerated search (device SMASH_MODE_MAM, restated in the oracle as
orc_mam_fast) must emit exactly the reference's MAM triples: checked against
the golden vectors and against orc_mam on a larger synthetic genome (CPU)."""
import os
import sys

import numpy as np
import pytest

import oracle as O
from conftest import interleaved_reads, read_gz_lines

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_fast_search_matches_reference_goldens(tiny_ix, s):
    tiny_ix.accel()
    exp = [[tuple(map(int, x.split(","))) for x in l.split()[2:]]
           for l in read_gz_lines("%s_MAM.txt.gz" % s)]
    reads = interleaved_reads(s)
    for i, e in enumerate(exp):
        assert tiny_ix.search_fast(reads[i].tobytes()) == e, i
        assert tiny_ix.search_v3(reads[i].tobytes()) == e, i


def test_v3_on_edge_reads(tiny_ix):
    """reads with bytes absent from the text, 'n' (present in the text),
    all-N, min_len windows at the read end, a palindrome."""
    tiny_ix.accel()
    T = tiny_ix.T[:tiny_ix.N]
    rng = np.random.default_rng(5)
    cases = []
    for _ in range(300):
        p = int(rng.integers(0, tiny_ix.N - 200))
        r = bytearray(T[p:p + 120].tobytes())
        for _k in range(int(rng.integers(0, 4))):
            r[int(rng.integers(0, 120))] = int(rng.choice(list(b"acgtnz`$N")))
        cases.append(bytes(r))
    cases += [b"z" * 100, b"n" * 100, b"a" * 100, b"acgt" * 30]
    for P in cases:
        for ml in (20, 12, 30):
            assert tiny_ix.search_v3(P, min_len=ml) == tiny_ix.search(P, min_len=ml)


def test_fast_search_equals_plain_on_mid_genome():
    import synth
    g = synth.make_genome("mid")
    ix = O.Index(*O.text_from_contigs(g))
    U, KT, K = ix.accel()
    assert K == O.lib().orc_accel_k(ix.N)
    r1, r2 = synth.make_reads(g, 3000, 150, seed=44)
    reads = np.empty((6000, 150), np.uint8)
    reads[0::2], reads[1::2] = r1, r2
    reads[reads == ord("N")] = ord("Z")
    lo = np.arange(256, dtype=np.uint8); lo[65:91] += 32
    reads = lo[reads]
    c1, c2 = O.OrcCounters(), O.OrcCounters()
    for i in range(len(reads)):
        P = reads[i].tobytes()
        exp = ix.search(P)
        assert ix.search_fast(P) == exp, i
        assert ix.search_v3(P) == exp, i
    n1, k1 = O.map_only(ix, reads, threads=4, count=True)
    n2, k2 = O.map_only_fast(ix, reads, threads=4, count=True)
    n3, k3 = O.map_only_v3(ix, reads, threads=4, count=True)
    assert n1 == n2 == n3
    assert k3.lines() < k2.lines() < k1.lines()     # the point of the accelerators


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_device_mem_probes_match_reference_goldens(tiny_ix, s):
    """orc_mem_dev (csrc/mem.hip's probe sequence: the k-mer table from the
    root, 8-byte singleton compares) emits the compiled reference's -maxmatch
    triples in order, like orc_mem; the threaded batch agrees read by read
    and counts fewer probe lines than the reference's sequence."""
    tiny_ix.accel()
    exp = [[tuple(map(int, x.split(","))) for x in l.split()[2:]]
           for l in read_gz_lines("%s_MEM.txt.gz" % s)]
    reads = interleaved_reads(s)[:len(exp)]
    for i, e in enumerate(exp):
        assert tiny_ix.search(reads[i].tobytes(), mode="MEM_DEV") == e, i
    t0, p0, c0 = O.mem_batch(tiny_ix, reads, threads=3, count=True)
    t1, p1, c1 = O.mem_batch(tiny_ix, reads, threads=3, device_probes=True, count=True)
    assert t0 == t1 == sum(len(e) for e in exp)
    assert p0.tolist() == p1.tolist() == [len(e) for e in exp]
    lines = lambda c: c.sa_lines + c.isa_lines + c.ref_lines + c.lcp_lines + c.kt_lines
    assert lines(c1) < lines(c0)


def test_device_mem_probes_on_edge_reads(tiny_ix):
    tiny_ix.accel()
    T = tiny_ix.T[:tiny_ix.N]
    rng = np.random.default_rng(6)
    cases = [b"z" * 100, b"n" * 100, b"a" * 100, b"acgt" * 30]
    for _ in range(200):
        p = int(rng.integers(0, tiny_ix.N - 200))
        r = bytearray(T[p:p + 120].tobytes())
        for _k in range(int(rng.integers(0, 4))):
            r[int(rng.integers(0, 120))] = int(rng.choice(list(b"acgtnz`$N")))
        cases.append(bytes(r))
    for P in cases:
        for ml in (20, 12, 30):
            assert tiny_ix.search(P, mode="MEM_DEV", min_len=ml) == \
                tiny_ix.search(P, mode="MEM", min_len=ml)


def test_device_mem_probes_packed_words():
    """mem.hip over packed 8-byte SA words decides find_Lmaximal from the
    word's BWT tag instead of a text byte (csrc/mem.hip left_max); the
    oracle's restatement of that probe sequence (orc_mem_dev over an index
    with pos_mask) gives the reference's MEMs with fewer text lines."""
    import synth
    sys.path.insert(0, os.path.join(ROOT, "tools", "sm_emu"))
    import sm_emu
    g = synth.make_genome("mid")
    T, sp, sz, names = O.text_from_contigs(g)
    ix = O.Index(T, sp, sz, names)
    ix.accel()
    sa, isa = sm_emu.pack_words(ix.T, ix.SA, ix.ISA, ix.L8, ix.acc.K)
    pix = O.Index(ix.T, sp, sz, names, SA=sa, ISA=isa, L8=ix.L8, ovf=ix.ovf, padded_text=True,
                  pos_mask=sm_emu.POS_MASK)
    assert pix.SA.dtype == np.uint64
    pix.accel()
    rng = np.random.default_rng(11)
    N = ix.N
    reads = []
    for i in range(120):                      # genome slices: repeat copies give many MEMs
        p = int(rng.integers(0, N - 151))
        r = bytearray(ix.T[p:p + 150].tobytes())
        if i % 3 == 0:
            r[int(rng.integers(0, 150))] = ord("g")
        reads.append(bytes(r))
    R = np.frombuffer(b"".join(reads), np.uint8).reshape(len(reads), 150)
    for r in reads:
        assert pix.search(r, mode="MEM_DEV") == ix.search(r, mode="MEM")
    _, per_a, ca = O.mem_batch(ix, R, device_probes=True, count=True)
    _, per_b, cb = O.mem_batch(pix, R, device_probes=True, count=True)
    assert (per_a == per_b).all() and per_a.sum() > len(reads)
    assert cb.ref_lines < ca.ref_lines
