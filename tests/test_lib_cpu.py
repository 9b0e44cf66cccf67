"""CPU-side checks of the product library (no GPU needed): it loads, exports
every entry point include/smash_gpu.h declares, and its host-side FASTA
builder (smash_text_from_fasta) reproduces the reference text byte for byte."""
import hashlib
import os
import re

import numpy as np

from conftest import ROOT, gold

import smashgpu as S


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "smash_gpu.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(smash_[a-z0-9_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    L = S.lib()
    syms = declared_symbols()
    assert len(syms) >= 20
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    assert sorted(S.EXPORTS) == syms


def test_text_from_fasta_matches_reference(tiny_fa):
    T, sp, sz, names = S.text_from_fasta(tiny_fa)
    sums = {l.split()[0]: l.split()[1] for l in open(gold("tiny_index.sha256"))}
    assert hashlib.sha256(T.tobytes()).hexdigest() == sums["rc1.ref.seq.bin"]
    import oracle as O
    T2, sp2, sz2, n2 = O.text_from_fasta(tiny_fa)
    assert np.array_equal(sp, sp2) and np.array_equal(sz, sz2) and names == n2


def test_text_from_contigs_equals_fasta(tiny_fa):
    import synth
    T, sp, sz, names = S.text_from_contigs(synth.make_genome("tiny"))
    T2, sp2, sz2, n2 = S.text_from_fasta(tiny_fa)
    assert np.array_equal(T, T2) and np.array_equal(sp, sp2) and names == n2


def test_fasta_edge_cases(tmp_path):
    """blank lines, spaces, lowercase, no trailing newline (last line is
    dropped by the reference's getline/eof handling, fasta.cpp:195-226)."""
    import oracle as O
    cases = [b">a x\nACGT\n\nacgN\n>b\nTTTT\n",
             b">a\n  AC GT  \n>b\nGG\n",
             b">a\nACGT\n>b\nGG",
             b">only\nRYKMBDHVN\n"]
    for i, c in enumerate(cases):
        p = tmp_path / ("f%d.fa" % i)
        p.write_bytes(c)
        a = S.text_from_fasta(str(p))
        b = O.text_from_fasta(str(p))
        assert a[0].tobytes() == b[0].tobytes(), c
        assert list(a[1]) == list(b[1]) and list(a[2]) == list(b[2]) and a[3] == b[3]


def _ref_bin_image(fasta_size, T, sp, sz, names):
    """rc?.ref.bin as Sequence::Sequence writes it (fasta.cpp:265-277)."""
    b = bytearray()
    for v in (fasta_size, len(T), len(sp)):
        b += int(v).to_bytes(8, "little")
    for s, z, n in zip(sp, sz, names):
        b += int(s).to_bytes(8, "little") + int(z).to_bytes(8, "little")
        b += len(n).to_bytes(8, "little") + n.encode()
    b += max(len(n) for n in names).to_bytes(8, "little")
    return bytes(b)


def test_text_from_fasta_forward_layout_matches_reference(tiny_fa):
    """`mummer` without -rcref (fasta.cpp:160-169): c1 ` c2 ` ... cn $, one
    entry per contig; the text and the whole rc0.ref.bin (sizes, start
    positions, names) equal the reference's own (tests/golden/
    tiny_index_rc0.sha256, tools/make_golden_r03.sh)."""
    sums = {l.split()[0]: l.split()[1] for l in open(gold("tiny_index_rc0.sha256"))}
    T, sp, sz, names = S.text_from_fasta(tiny_fa, rcref=False)
    assert hashlib.sha256(T.tobytes()).hexdigest() == sums["rc0.ref.seq.bin"]
    img = _ref_bin_image(os.path.getsize(tiny_fa), T, sp, sz, names)
    assert hashlib.sha256(img).hexdigest() == sums["rc0.ref.bin"]
    # and the -rcref layout's image of rc1.ref.bin
    T1, sp1, sz1, n1 = S.text_from_fasta(tiny_fa)
    sums1 = {l.split()[0]: l.split()[1] for l in open(gold("tiny_index.sha256"))}
    if "rc1.ref.bin" in sums1:
        img1 = _ref_bin_image(os.path.getsize(tiny_fa), T1, sp1, sz1, n1)
        assert hashlib.sha256(img1).hexdigest() == sums1["rc1.ref.bin"]


def test_fasta_forward_layout_edge_cases(tmp_path):
    """The forward-only text is the -rcref text's forward contigs joined by
    '`' (no separator after the last one), on the edge-case files above; a
    last line without a newline is read with eof set and its bytes after the
    first land in the text with no contig entry (fasta.cpp:195-240), in
    both layouts."""
    cases = [b">a x\nACGT\n\nacgN\n>b\nTTTT\n",
             b">a\n  AC GT  \n>b\nGG\n",
             b">a\nACGT\n>b\nGG",
             b">only\nRYKMBDHVN\n",
             b">a\nAC\n>b\nGG\n>c\nT\n"]
    for i, c in enumerate(cases):
        p = tmp_path / ("f%d.fa" % i)
        p.write_bytes(c)
        T1, sp1, sz1, n1 = S.text_from_fasta(str(p))
        T0, sp0, sz0, n0 = S.text_from_fasta(str(p), rcref=False)
        fw = [T1[int(sp1[k]):int(sp1[k] + sz1[k])].tobytes() for k in range(0, len(sp1), 2)]
        end = int(sp1[-1] + sz1[-1])
        tail = T1[end + 1:-1].tobytes()
        want = b"`".join(fw) + (b"`" + tail if tail else b"") + b"$"
        assert T0.tobytes() == want, c
        assert n0 == n1[0::2] and list(sz0) == list(sz1[0::2])
        assert list(sp0) == [sum(len(f) + 1 for f in fw[:k]) for k in range(len(fw))]


def test_pipeline_refuses_batches_past_the_32bit_word_bound():
    """max_pairs * 2 * slots must stay below 2^32 (the batch's u32 position
    offsets and the export's packed keys << 32 | words prefix,
    csrc/pipeline.hip k_export_count): smash_pipeline_create refuses a larger
    batch with SMASH_ERR_ARG before it touches the index or the device."""
    import ctypes as C
    assert S.pipeline_max_batch(150, 20) == ((1 << 32) - 1) // (2 * 131) == 16_393_004
    assert S.pipeline_max_batch(100, 20) == ((1 << 32) - 1) // (2 * 81)
    assert S.pipeline_max_batch(255, 20) == ((1 << 32) - 1) // (2 * 236)
    assert S.pipeline_max_batch(19, 20) == 0 and S.pipeline_max_batch(256, 20) == 0
    assert 12_500_000 <= S.pipeline_max_batch(150, 20)   # the bench's C3 batch fits

    class FakeIndex:   # never dereferenced past the size check
        buf = C.create_string_buffer(4096)
        h = C.cast(buf, C.c_void_p)
        contigs = ["chr1", "chr2"]
        contig_sizes = [1000, 1000]

    starts = np.array([0, 500, 1000], np.int64)
    for L, B in ((150, 16_393_005), (150, 25_000_000), (250, 12_500_000)):
        assert B > S.pipeline_max_batch(L, 20)
        try:
            S.Pipeline(FakeIndex(), {"chr1": 0, "chr2": 1000}, starts, L, B)
        except S.SmashError as e:
            assert "(-1)" in str(e) and "bad configuration" in str(e), e
        else:
            raise AssertionError("batch of %d pairs at %d bp accepted" % (B, L))
