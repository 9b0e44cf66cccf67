"""Deterministic synthetic genomes, SMASH reads and bin tables.

Input generator for tests, golden fixtures and bench.py.  No
network, no real genome: genomes are numpy-generated from a seed, shaped like
the reference's targets:

* ``tiny``  -- 5 contigs (~330 kb) with N runs, an Alu-like family, a
  segmental duplication, a tandem repeat, a reverse-complement palindrome, a
  ``chrM`` and a ``_gl000`` contig (exercises mappability_tag's small_chr
  rule, mappability_tag.cpp:82-83, and varbin's chromosome filter,
  varbin.py:38-49).
* ``chr21`` -- one 48,129,895 bp contig, leading 9.41 Mb N run.
* ``hg19``  -- chr1..chr22, chrX, chrY with hg19 lengths taken from
  ``data/bins/50000/bins.txt`` plus chrM (16,571 bp); N runs over every
  >1 Mb bin of that table (the real assembly gaps sit there) and 10 kb
  telomere gaps.

All genomes also carry interspersed repeats (300 bp "Alu", 6 kb "L1"),
20 kb segmental duplications and short tandem repeats so that suffix-array
intervals are non-trivial.

Reads follow the SMASH mode of SURVEY.md §8d: each mate is a concatenation
of segments of uniform length [20,60] from independent loci and strands,
1 % substitutions, a few reads with an ``N``, ~1 % exact duplicate pairs
(pair de-dup, smashMEM.py:217-228).  Names are ``r%09d`` so that
``samtools sort -n`` order equals generation order.
"""
from __future__ import annotations

import os
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
DATA = os.path.join(ROOT, "data")

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)
_COMP = np.arange(256, dtype=np.uint8)
for a, b in zip(b"ACGTNacgtn", b"TGCANtgcan"):
    _COMP[a] = b


def revcomp(seq: np.ndarray) -> np.ndarray:
    return _COMP[seq[::-1]]


def _mutate(rng, seq: np.ndarray, rate: float) -> np.ndarray:
    out = seq.copy()
    if rate <= 0 or len(out) == 0:
        return out
    m = rng.random(len(out)) < rate
    k = int(m.sum())
    if k:
        # substitute with a different base
        cur = np.searchsorted(ACGT, out[m]).clip(0, 3)
        out[m] = ACGT[(cur + rng.integers(1, 4, size=k)) % 4]
    return out


def hg19_lengths(bins_path: str | None = None):
    """(name, length) of the 24 major hg19 contigs, from the bins table."""
    bins_path = bins_path or os.path.join(DATA, "bins", "50000", "bins.txt")
    lens = {}
    order = []
    with open(bins_path) as f:
        for line in f:
            c = line.rstrip("\n").split("\t")
            if c[0] not in lens:
                order.append(c[0])
            lens[c[0]] = int(c[3])
    return [(c, lens[c]) for c in order]


def _big_bins(bins_path=None, min_len=1_000_000):
    bins_path = bins_path or os.path.join(DATA, "bins", "50000", "bins.txt")
    out = {}
    with open(bins_path) as f:
        for line in f:
            c = line.rstrip("\n").split("\t")
            if int(c[4]) > min_len:
                out.setdefault(c[0], []).append((int(c[1]), int(c[3])))
    return out


def _inject_repeats(rng, contigs, nmask, scale):
    """Interspersed repeats / segmental dups / tandem repeats, in place.

    Never writes over N runs (nmask) so that N runs stay exact."""
    total = sum(len(s) for _, s in contigs)
    lens = np.array([len(s) for _, s in contigs], dtype=np.float64)
    p = lens / lens.sum()

    def place(length):
        while True:
            ci = int(rng.choice(len(contigs), p=p))
            L = len(contigs[ci][1])
            if L <= length + 2:
                continue
            st = int(rng.integers(0, L - length))
            if not nmask[ci][st:st + length].any():
                return ci, st

    fams = [
        (300, int(total / 10000 * scale), 0.02, 0.20),   # Alu-like
        (6000, int(total / 500000 * scale), 0.05, 0.20),  # L1-like
    ]
    for flen, copies, dlo, dhi in fams:
        element = ACGT[rng.integers(0, 4, size=flen)]
        for _ in range(copies):
            e = element
            if flen > 1000:  # 5' truncation like L1
                e = e[int(rng.integers(0, flen - 500)):]
            e = _mutate(rng, e, float(rng.uniform(dlo, dhi)))
            if rng.random() < 0.5:
                e = revcomp(e)
            ci, st = place(len(e))
            contigs[ci][1][st:st + len(e)] = e
    # segmental duplications (20 kb, 1-2 % divergence)
    for _ in range(max(1, int(total / 2_500_000 * scale))):
        sl = 20000
        ci, st = place(sl)
        src = contigs[ci][1][st:st + sl].copy()
        src = _mutate(rng, src, float(rng.uniform(0.01, 0.02)))
        if rng.random() < 0.5:
            src = revcomp(src)
        cj, sj = place(sl)
        contigs[cj][1][sj:sj + sl] = src
    # short tandem repeats
    for _ in range(int(total / 50000 * scale)):
        per = int(rng.integers(1, 7))
        n = int(rng.integers(50, 500))
        unit = ACGT[rng.integers(0, 4, size=per)]
        tr = np.tile(unit, n // per + 1)[:n]
        ci, st = place(n)
        contigs[ci][1][st:st + n] = tr


def make_genome(kind: str = "tiny", seed: int | None = None):
    """Returns [(name, uint8 ASCII array 'ACGTN')] in FASTA order."""
    if kind == "tiny":
        seed = 7 if seed is None else seed
        rng = np.random.default_rng(seed)
        spec = [("chr1", 120000), ("chr2", 90000), ("chrX", 60000),
                ("chrM", 16571), ("chr1_gl000191_random", 40000)]
        contigs = [(n, ACGT[rng.integers(0, 4, size=L)]) for n, L in spec]
        nmask = [np.zeros(len(s), bool) for _, s in contigs]
        # N runs: telomeric on chr1, interior on chr2 and chrX
        for ci, a, b in [(0, 0, 2000), (0, 60000, 65000), (1, 40000, 52000),
                         (2, 59000, 60000)]:
            contigs[ci][1][a:b] = ord("N")
            nmask[ci][a:b] = True
        _inject_repeats(rng, contigs, nmask, scale=20.0)
        # a perfect reverse-complement palindrome (never unique in the
        # doubled text)
        half = ACGT[rng.integers(0, 4, size=60)]
        pal = np.concatenate([half, revcomp(half)])
        contigs[0][1][30000:30120] = pal
        return contigs
    if kind == "mid":
        # ~3.2 Mbp, for device-vs-oracle parity at a size the C oracle
        # indexes in seconds
        seed = 5 if seed is None else seed
        rng = np.random.default_rng(seed)
        spec = [("chr1", 1400000), ("chr2", 1000000), ("chr3", 600000),
                ("chrX", 200000), ("chrM", 16571), ("chr4_gl000193_random", 30000)]
        contigs = [(n, ACGT[rng.integers(0, 4, size=L)]) for n, L in spec]
        nmask = [np.zeros(len(s), bool) for _, s in contigs]
        for ci, a, b in [(0, 0, 10000), (0, 700000, 760000), (1, 300000, 301000),
                         (2, 590000, 600000)]:
            contigs[ci][1][a:b] = ord("N")
            nmask[ci][a:b] = True
        _inject_repeats(rng, contigs, nmask, scale=10.0)
        return contigs
    if kind == "chr21":
        seed = 21 if seed is None else seed
        rng = np.random.default_rng(seed)
        L = 48129895
        s = ACGT[rng.integers(0, 4, size=L)]
        s[:9411193] = ord("N")
        nmask = [np.zeros(L, bool)]
        nmask[0][:9411193] = True
        contigs = [("chr21", s)]
        _inject_repeats(rng, contigs, nmask, scale=1.0)
        return contigs
    if kind == "hg19":
        seed = 19 if seed is None else seed
        rng = np.random.default_rng(seed)
        big = _big_bins()
        contigs, nmask = [], []
        for name, L in hg19_lengths() + [("chrM", 16571)]:
            s = ACGT[rng.integers(0, 4, size=L)]
            m = np.zeros(L, bool)
            if name != "chrM":
                for a, b in [(0, 10000), (L - 10000, L)]:
                    m[a:b] = True
                for a, b in big.get(name, []):
                    a2, b2 = a + 50000, b - 50000
                    if b2 > a2:
                        m[a2:b2] = True
            s[m] = ord("N")
            contigs.append((name, s))
            nmask.append(m)
        _inject_repeats(rng, contigs, nmask, scale=1.0)
        return contigs
    raise ValueError(kind)


def write_fasta(path, contigs, width=60):
    with open(path, "wb") as f:
        for name, s in contigs:
            f.write(b">" + name.encode() + b"\n")
            b = s.tobytes()
            for i in range(0, len(b), width):
                f.write(b[i:i + width] + b"\n")


def _allowed_intervals(contigs, margin=500, minlen=80):
    """Non-N stretches, shrunk by `margin` from N runs and contig ends."""
    out = []
    for ci, (name, s) in enumerate(contigs):
        isn = np.concatenate([[True], s == ord("N"), [True]])
        d = np.diff(isn.astype(np.int8))
        starts = np.nonzero(d == -1)[0]
        ends = np.nonzero(d == 1)[0]
        for a, b in zip(starts, ends):
            a2, b2 = a + margin, b - margin
            if b2 - a2 >= minlen:
                out.append((ci, a2, b2))
    return out


def make_reads(contigs, n_pairs: int, read_len: int = 100, seed: int = 1,
               err: float = 0.01, dup_frac: float = 0.01,
               n_frac: float = 0.005, seg=(20, 60), exclude=("chrM",),
               chunk: int = 200000):
    """SMASH-mode paired reads.  Returns (r1, r2): uint8 [n_pairs, read_len].

    Fully vectorised (chunks of `chunk` pairs) so that 50 M-pair inputs are
    generated in minutes."""
    rng = np.random.default_rng(seed)
    ivs = [iv for iv in _allowed_intervals(contigs)
           if contigs[iv[0]][0] not in exclude and "_" not in contigs[iv[0]][0]]
    coff = np.cumsum([0] + [len(s) for _, s in contigs])
    G = np.concatenate([s for _, s in contigs])
    iv_a = np.array([coff[c] + a for c, a, _ in ivs], dtype=np.int64)
    iv_b = np.array([coff[c] + b for c, _, b in ivs], dtype=np.int64)
    w = (iv_b - iv_a).astype(np.float64)
    w /= w.sum()
    max_segs = read_len // seg[0] + 1
    r1 = np.empty((n_pairs, read_len), dtype=np.uint8)
    r2 = np.empty((n_pairs, read_len), dtype=np.uint8)
    cols = np.arange(read_len, dtype=np.int64)[None, :]
    for p0 in range(0, n_pairs, chunk):
        npair = min(chunk, n_pairs - p0)
        nm = 2 * npair
        seglen = rng.integers(seg[0], seg[1] + 1, size=(nm, max_segs)).astype(np.int64)
        ivi = rng.choice(len(ivs), size=(nm, max_segs), p=w)
        a, b = iv_a[ivi], iv_b[ivi]
        st = a + (rng.random((nm, max_segs)) *
                  np.maximum(b - a - seglen, 1)).astype(np.int64)
        strand = rng.random((nm, max_segs)) < 0.5
        cum = np.cumsum(seglen, axis=1)
        sid = np.zeros((nm, read_len), dtype=np.int64)
        for k in range(max_segs - 1):
            sid += cols >= cum[:, k:k + 1]
        rows = np.arange(nm)[:, None]
        base = np.concatenate([np.zeros((nm, 1), np.int64), cum[:, :-1]], axis=1)
        off = cols - base[rows, sid]
        L = seglen[rows, sid]
        S = st[rows, sid]
        rc = strand[rows, sid]
        pos = np.where(rc, S + L - 1 - off, S + off)
        out = G[pos]
        out = np.where(rc, _COMP[out], out).astype(np.uint8)
        flat = out.reshape(-1)
        mut = rng.random(flat.shape[0]) < err
        cur = np.searchsorted(ACGT, flat[mut]).clip(0, 3)
        flat[mut] = ACGT[(cur + rng.integers(1, 4, size=int(mut.sum()))) % 4]
        nn = np.nonzero(rng.random(nm) < n_frac)[0]
        out[nn, rng.integers(0, read_len, size=len(nn))] = ord("N")
        r1[p0:p0 + npair] = out[0::2]
        r2[p0:p0 + npair] = out[1::2]
    # exact duplicate pairs (copy of an earlier pair)
    if n_pairs > 10 and dup_frac > 0:
        d = np.nonzero(rng.random(n_pairs) < dup_frac)[0]
        d = d[d > 0]
        src = (rng.random(len(d)) * d).astype(np.int64)
        r1[d] = r1[src]
        r2[d] = r2[src]
    return r1, r2


def write_fastq(path, reads: np.ndarray, mate: int):
    q = b"I" * reads.shape[1]
    with open(path, "wb") as f:
        for i in range(reads.shape[0]):
            f.write(b"@r%09d %d:N:0\n" % (i, mate))
            f.write(reads[i].tobytes() + b"\n+\n" + q + b"\n")


def write_index_side_files(fa_bin_dir, contigs):
    """chrom_sizes.txt and sam_header.txt exactly as index_setup.sh:28,31."""
    os.makedirs(fa_bin_dir, exist_ok=True)
    n = 0
    with open(os.path.join(fa_bin_dir, "chrom_sizes.txt"), "w") as f:
        for name, s in contigs:
            if "_" in name:
                continue
            f.write("%s\t%d\t%d\n" % (name, len(s), n))
            n += len(s)
    with open(os.path.join(fa_bin_dir, "sam_header.txt"), "w") as f:
        for name, s in contigs:
            f.write("@SQ\tSN:%s\tLN:%d\n" % (name, len(s)))


def make_bins(contigs, per_contig_bins=8, path=None):
    """Variable-width bins (6-column bins.txt, binning.sh:22-24) for a
    synthetic genome: each non-'_', non-chrM contig split into bins of
    pseudo-random widths.  abspos offsets follow chrom_sizes order."""
    rng = np.random.default_rng(99)
    rows = []
    off = 0
    for name, s in contigs:
        if "_" in name:
            continue
        L = len(s)
        if name != "chrM":
            cuts = np.sort(rng.choice(np.arange(1, L), size=per_contig_bins - 1,
                                      replace=False))
            starts = np.concatenate([[0], cuts])
            stops = np.concatenate([cuts, [L]])
            for a, b in zip(starts, stops):
                rows.append((name, int(a), int(a + off), int(b), int(b - a), 1000))
        off += L
    if path:
        with open(path, "w") as f:
            for r in rows:
                f.write("%s\t%d\t%d\t%d\t%d\t%d\n" % r)
    return rows


def split_bins(src_path, factor, dst_path):
    """Synthesize a finer bin table by splitting each bin into `factor`
    equal sub-bins (100000 = 50000 split in 2, 500000 = split
    in 10; the upstream files are missing, .MISSING_LARGE_BLOBS:1-4)."""
    with open(src_path) as f, open(dst_path, "w") as g:
        for line in f:
            c = line.rstrip("\n").split("\t")
            a, ab, b = int(c[1]), int(c[2]), int(c[3])
            L = b - a
            for k in range(factor):
                s = a + (L * k) // factor
                e = a + (L * (k + 1)) // factor
                g.write("%s\t%d\t%d\t%d\t%d\t%s\n" % (c[0], s, ab + (s - a), e, e - s, c[5]))
