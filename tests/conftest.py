"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else is CPU."""
import gzip
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools"),
          os.path.join(ROOT, "smash-paper_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def gold(name):
    return os.path.join(GOLD, name)


def read_gz_lines(name):
    with gzip.open(gold(name), "rt") as f:
        return [l.rstrip("\n") for l in f]


@pytest.fixture(scope="session")
def tiny_fa(tmp_path_factory):
    d = tmp_path_factory.mktemp("tiny")
    p = d / "tiny.fa"
    with gzip.open(gold("tiny.fa.gz"), "rb") as f:
        p.write_bytes(f.read())
    return str(p)


@pytest.fixture(scope="session")
def tiny_ix(tiny_fa):
    import oracle as O
    return O.Index.from_fasta(tiny_fa)


def fastq_reads(name):
    """Sequences of a gzipped FASTQ, as raw bytes."""
    lines = read_gz_lines(name)
    return [lines[i].encode() for i in range(1, len(lines), 4)]


def interleaved_reads(prefix):
    """[2*n, L] uint8, lowercased with N->z (fastqs_to_sam replaceN +
    NewQuery::extend), mates interleaved r1,r2,r1,..."""
    import oracle as O
    r1 = fastq_reads(prefix + "_r1.fq.gz")
    r2 = fastq_reads(prefix + "_r2.fq.gz")
    L = len(r1[0])
    out = np.empty((2 * len(r1), L), np.uint8)
    for i, (a, b) in enumerate(zip(r1, r2)):
        out[2 * i] = np.frombuffer(O.lower_read(a), np.uint8)
        out[2 * i + 1] = np.frombuffer(O.lower_read(b), np.uint8)
    return out


def load_bins(path):
    rows = [l.rstrip("\n").split("\t") for l in open(path)]
    return rows, np.array([int(r[2]) for r in rows], np.int64)


def load_chrom_sizes(path):
    out = {}
    for l in open(path):
        c = l.rstrip("\n").split("\t")
        out[c[0]] = int(c[2])
    return out
