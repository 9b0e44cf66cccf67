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
