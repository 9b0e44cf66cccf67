"""Pin the C oracle to the UPSTREAM reference's own outputs (tests/golden/,
made by tools/make_golden.sh from the compiled reference + varbin.py).

Every stage of the chain is checked: text layout, SA/ISA/LCP/map.bin bytes,
per-read MAM/MUM/MEM triples, prepare_matches + mappability_tag SAM fields,
smashMEM (the REFERENCE's smashMEM.py run over tools/pysam_shim,
tools/make_golden_smashmem.sh) and varbin counts.  CPU only.
"""
import hashlib
import re

import numpy as np
import pytest

import oracle as O
from conftest import (gold, interleaved_reads, load_bins, load_chrom_sizes,
                      read_gz_lines)


def _sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def sums():
    out = {}
    for l in open(gold("tiny_index.sha256")):
        name, h, size = l.split()
        out[name] = (h, int(size))
    return out


def test_text_layout(tiny_ix, sums):
    # rc1.ref.seq.bin is the raw doubled text (fasta.cpp:267)
    T = tiny_ix.T[:tiny_ix.N].tobytes()
    assert (_sha(T), len(T)) == sums["rc1.ref.seq.bin"]
    assert T[-1:] == b"$"
    assert tiny_ix.contigs == ["chr1", "chr2", "chrX", "chrM", "chr1_gl000191_random"]


def test_text_from_contigs_matches_fasta(tiny_ix):
    import synth
    g = synth.make_genome("tiny")
    T, sp, sz, names = O.text_from_contigs(g)
    assert np.array_equal(T, tiny_ix.T[:tiny_ix.N])
    assert np.array_equal(sp, tiny_ix.startpos)
    assert np.array_equal(sz, tiny_ix.sizes)


def test_sa_isa_lcp_bytes(tiny_ix, sums):
    # 32-bit index flavour (`mummer`, size.h) since N < 2^31
    assert (_sha(tiny_ix.SA.astype(np.uint32).tobytes()), 4 * tiny_ix.N) == sums["rc1.i4.index.sa.bin"]
    assert (_sha(tiny_ix.ISA.astype(np.uint32).tobytes()), 4 * tiny_ix.N) == sums["rc1.i4.index.isa.bin"]
    vec = np.minimum(tiny_ix.LCP, 255).astype(np.uint8)
    assert (_sha(vec.tobytes()), tiny_ix.N) == sums["rc1.i4.index.lcp.vec.bin"]
    # overflow table: item_t{size_t idx; uint32 val} padded to 16 B, sorted;
    # the 4 padding bytes are uninitialised upstream, hence the masked hash
    big = np.nonzero(tiny_ix.LCP >= 255)[0]
    m = np.zeros((len(big), 2), np.uint64)
    m[:, 0] = big
    m[:, 1] = tiny_ix.LCP[big]
    assert _sha(m.tobytes()) == sums["rc1.i4.index.lcp.m.bin:masked"][0]


def test_mappability_bytes(tiny_ix, sums):
    mp = tiny_ix.mappability()
    h, size = sums["map.bin[2:]"]
    assert len(mp) == size
    assert _sha(mp[2:].tobytes()) == h


def _parse_triples(lines):
    out = []
    for l in lines:
        f = l.split()
        out.append([tuple(map(int, x.split(","))) for x in f[2:]])
    return out


@pytest.mark.parametrize("s", ["s100", "s150"])
@pytest.mark.parametrize("mode", ["MAM", "MUM", "MEM"])
def test_search_triples(tiny_ix, s, mode):
    exp = _parse_triples(read_gz_lines("%s_%s.txt.gz" % (s, mode)))
    reads = interleaved_reads(s)
    assert len(exp) <= len(reads)
    for i, e in enumerate(exp):
        got = tiny_ix.search(reads[i].tobytes(), mode)
        assert got == e, (i, mode)


def _expected_lines(ix, name, reads_pair, mapbin, offsets, small):
    """Reduced SAM records (fields 1-9 + tags) the reference would print for
    one pair: prepare_matches/set_nomap/set_mate/print_matches
    (query.cpp:231-415) + mappability_tag L0/R0 (mappability_tag.cpp:93-124)."""
    res = []
    for k, P in enumerate(reads_pair):
        m = ix.search(P)
        hits, best = ix.resolve(P, m)
        res.append((hits, best))
    lines = []
    contigs = ix.contigs
    for k in (0, 1):
        hits, best = res[k]
        ohits, obest = res[1 - k]
        flag0 = 65 if k == 0 else 129
        mate_unmapped = obest is None
        if mate_unmapped:
            flag0 |= 8
            mate = best
        else:
            mate = obest
        mate_s = "%s\t%d\t0" % (contigs[mate[0]], mate[1] + 1) if mate else "*\t0\t0"
        if not hits:
            rn = "%s\t%d" % (contigs[mate[0]], mate[1] + 1) if mate else "*\t0"
            lines.append("%s\t%d\t%s\t0\t*\t%s\tXM:i:0\tNH:i:0" % (name, flag0 | 4, rn, mate_s))
            continue
        for i, h in enumerate(hits):
            O.tag(h, offsets, mapbin, small[h.tid])
            flag = flag0 | (16 if h.rc else 0) | (256 if h.hi else 0)
            t = ["XM:i:%d" % h.n_matches, "XU:i:%d" % h.n_unique,
                 "XE:i:%d" % h.n_matched, "XS:A:%s" % ("-" if h.rc else "+"),
                 "NH:i:%d" % h.nh, "HI:i:%d" % h.hi]
            if i > 0:
                p = hits[i - 1]
                t += ["cc:Z:%s" % contigs[p.tid], "cp:i:%d" % (p.pos + 1),
                      "xo:A:%s" % ("=" if p.rc == h.rc else "!"),
                      "xc:Z:%s" % p.cigar.decode()]
            if i + 1 < len(hits):
                n = hits[i + 1]
                t += ["CC:Z:%s" % contigs[n.tid], "CP:i:%d" % (n.pos + 1),
                      "XO:A:%s" % ("=" if n.rc == h.rc else "!"),
                      "XC:Z:%s" % n.cigar.decode()]
            t += ["L0:i:%d" % h.L0, "R0:i:%d" % h.R0]
            lines.append("%s\t%d\t%s\t%d\t50\t%s\t%s\t%s" % (
                name, flag, contigs[h.tid], h.pos + 1, h.cigar.decode(), mate_s,
                "\t".join(t)))
    return lines


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_resolve_and_tag_match_mapout(tiny_ix, s):
    gold_lines = read_gz_lines("%s_mapout_tagged.txt.gz" % s)
    # drop the fastqs_to_sam comment tag (XO:Z:...) carried through
    gold_lines = sorted("\t".join(x for x in l.split("\t") if not x.startswith("XO:Z:"))
                        for l in gold_lines)
    reads = interleaved_reads(s)
    mapbin = tiny_ix.mappability()
    sizes = [int(x) for x in tiny_ix.sizes[0::2]]
    offsets = np.cumsum([0] + sizes[:-1]).astype(np.uint32)
    small = [1 if ("_gl000" in n or "chrM" in n) else 0 for n in tiny_ix.contigs]
    got = []
    for q in range(reads.shape[0] // 2):
        got += _expected_lines(tiny_ix, "r%09d" % q,
                               (reads[2 * q].tobytes(), reads[2 * q + 1].tobytes()),
                               mapbin, offsets, small)
    got.sort()
    assert len(got) == len(gold_lines)
    for a, b in zip(got, gold_lines):
        assert a == b


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_pipeline_positions_and_varbin(tiny_ix, s):
    """Whole oracle chain (orc_run_pairs) vs the REAL varbin.py output on the
    golden positions (whose smashMEM step is the oracle's; unpinned)."""
    reads = interleaved_reads(s)
    rows, starts = load_bins(gold("tiny_bins.txt"))
    cs = load_chrom_sizes(gold("tiny_chrom_sizes.txt"))
    pipe = O.Pipeline(tiny_ix, tiny_ix.mappability(), cs, starts)
    err = pipe.run(reads, threads=4)
    assert err == 0
    exp = [l.split("\t") for l in open(gold("%s_varbin.txt" % s))]
    assert [int(e[3]) for e in exp] == pipe.counts.tolist()
    st = open(gold("%s_varbin_stats_partial.txt" % s)).read().split("\n")[1].split("\t")
    assert int(st[0]) == pipe.state.total
    assert int(st[1]) == pipe.state.dups
    assert int(st[2]) == pipe.state.kept
    npos = sum(1 for _ in open(gold("%s_positions.txt" % s)))
    assert npos == pipe.n_pos.value


def test_varbin_edge_cases():
    """varbin.py quirks on hand-made positions with hg19 bins: adjacent de-dup
    ignores the chromosome (varbin.py:56-58), chrM/_/unknown skipped."""
    _, starts = load_bins(gold("../../data/bins/50000/bins.txt"))
    cs = load_chrom_sizes(gold("chrom_sizes_hg19.txt"))
    pos0, absp = [], []
    for l in open(gold("edge_positions.txt")):
        c, p = (l.rstrip("\n").split(" ") + [""])[:2]
        if "_" in c or c == "chrM" or c == "" or c not in cs:
            continue
        pos0.append(int(p))
        absp.append(int(p) + cs[c])
    counts, st = O.varbin(pos0, absp, starts)
    exp = [int(l.split("\t")[3]) for l in read_gz_lines("edge_varbin.txt.gz")]
    assert counts.tolist() == exp
    s = open(gold("edge_varbin_stats_partial.txt")).read().split("\n")[1].split("\t")
    assert (st.total, st.dups, st.kept) == (int(s[0]), int(s[1]), int(s[2]))


def test_varbin_before_first_bin_goes_to_last_bin():
    """bisect_right == 0 -> binCounts[-1] (varbin.py:89-92)."""
    counts, st = O.varbin([5, 6, 1000], [5, 6, 1000], [10, 20, 30])
    assert counts.tolist() == [0, 0, 3 - 0]
    assert (st.total, st.dups, st.kept) == (3, 0, 3)


# ---------------------------------------------------------------------------
# smashMEM.py: the reference script's own output (tools/make_golden_smashmem.sh
# ran it unmodified over tools/pysam_shim) against the oracle's restatement
# ---------------------------------------------------------------------------
_CIG = re.compile(r"(\d+)([MIDNSHP=X])")


def tagged_sam(s):
    """(@SQ names, body lines in samtools sort -n order) of the SAM the
    reference script ran on"""
    if s == "edge":
        lines = open(gold("smashmem_edge.sam")).read().splitlines()
        head = [l for l in lines if l.startswith("@")]
        body = [l for l in lines if l and not l.startswith("@")]
    else:
        head = open(gold("tiny_mapout_header.txt")).read().splitlines()
        body = read_gz_lines("%s_mapout_tagged_full.txt.gz" % s)
        body.sort(key=lambda l: (l.split("\t", 1)[0], 0 if int(l.split("\t")[1]) & 64 else 1))
    names = [x.split("SN:")[1].split("\t")[0] for x in head if x.startswith("@SQ")]
    return names, body


def orc_hit(f, tid_of):
    """pysam 0.8 fields of one mapped full SAM line"""
    h = O.OrcHit()
    h.tid = tid_of[f[2]]
    h.rc = 1 if int(f[1]) & 16 else 0
    h.pos = int(f[3]) - 1
    ops = _CIG.findall(f[5])
    rlen = len(f[9])
    lead = int(ops[0][0]) if ops[0][1] == "S" else 0
    trail = int(ops[-1][0]) if len(ops) > 1 and ops[-1][1] == "S" else 0
    h.qstart, h.qend = lead, rlen - trail
    tags = {t.split(":")[0]: t.split(":")[2] for t in f[11:]}
    h.hi, h.L0, h.R0 = int(tags["HI"]), int(tags["L0"]), int(tags["R0"])
    return h


@pytest.mark.parametrize("s", ["s100", "s150", "edge"])
def test_smashmem_restatement_equals_reference_script(s):
    """orc_smash_pair + the first-wins key set (smashMEM.py:154-228 restated)
    over the same name-sorted tagged SAM reproduce the script's output: the
    emitting pairs, each one's (chrom, pos) list in order (r1 by HI, then
    r2 by HI), and the dupe / non-dupe counts (smashMEM.py:230)."""
    names, body = tagged_sam(s)
    tid_of = {n: i for i, n in enumerate(names)}
    groups, order = {}, []
    for line in body:
        f = line.split("\t")
        if f[0] not in groups:
            groups[f[0]] = ([], [])
            order.append(f[0])
        if int(f[1]) & 4:
            continue
        groups[f[0]][0 if int(f[1]) & 64 else 1].append(orc_hit(f, tid_of))
    got, seen, dup = [], set(), 0
    for name in order:
        h1, h2 = groups[name]
        h1.sort(key=lambda h: h.hi)
        h2.sort(key=lambda h: h.hi)
        kept = O.smash_pair(h1, h2)
        if kept is None:
            continue
        if tuple(kept) in seen:
            dup += 1
            continue
        seen.add(tuple(kept))
        got += [(name, names[t], p) for t, p in kept]
    ref = read_gz_lines("%s_smashmem.txt.gz" % s)
    assert ref[0].startswith("read_id\t")
    exp = [(f[0], f[3], int(f[4])) for f in (l.split("\t") for l in ref[1:-1])]
    assert got == exp
    assert ref[-1] == "%d dupes\t%d non-dupes" % (dup, len(seen))


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_smashmem_reference_positions_are_the_golden_positions(s):
    """The awk/perl extraction (smash_mapping.sh:29) of the reference script's
    output is the positions file the varbin goldens were made from."""
    rx = re.compile(r"^chr(\d+|[XY]) \d+$")
    ref = read_gz_lines("%s_smashmem.txt.gz" % s)[1:-1]
    pos = [l for l in ("%s %s" % tuple(x.split("\t")[3:5]) for x in ref) if rx.match(l)]
    assert pos == open(gold("%s_positions.txt" % s)).read().splitlines()
