"""The command-line surface (smash-paper_amd/bin/fastqs_to_sam and
smash-paper_amd/smash_cli.py) against the reference's outputs.

CPU: fastqs_to_sam byte-identical to the reference binary's output on the
golden FASTQ pairs and on a parser edge-case pair; the CLI's FASTQ/SAM readers
and its `samtools sort -n` key.  GPU (`gpu` marker): `varbin`, `map` and
`count` on the tiny genome reproduce varbin.py's rows (the real varbin.py
output, tests/golden/*_varbin.txt) and the positions files.
"""
import gzip
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, gold

BIN = os.path.join(ROOT, "smash-paper_amd", "bin", "fastqs_to_sam")
sys.path.insert(0, os.path.join(ROOT, "smash-paper_amd"))
import smash_cli  # noqa: E402


def _fq(tmp_path, s, k):
    p = tmp_path / ("%s_r%d.fq" % (s, k))
    p.write_bytes(gzip.open(gold("%s_r%d.fq.gz" % (s, k))).read())
    return str(p)


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_fastqs_to_sam_matches_reference(tmp_path, s):
    out = subprocess.run([BIN, _fq(tmp_path, s, 1), _fq(tmp_path, s, 2), "1"],
                         capture_output=True, check=True).stdout
    assert out == gzip.open(gold("%s_fastqs_to_sam.sam.gz" % s)).read()


@pytest.mark.parametrize("replace", [False, True])
def test_fastqs_to_sam_edge_cases(replace):
    args = [BIN, gold("edge_r1.fq"), gold("edge_r2.fq")] + (["1"] if replace else [])
    out = subprocess.run(args, capture_output=True, check=True).stdout
    exp = open(gold("edge_fastqs_to_sam%s.sam" % ("_replaceN" if replace else "")), "rb").read()
    assert out == exp


def test_fastqs_to_sam_usage_error():
    r = subprocess.run([BIN, "only_one"], capture_output=True)
    assert r.returncode == 1 and b"usage" in r.stderr


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_cli_readers_agree_with_fastqs_to_sam(tmp_path, s):
    pairs = smash_cli.fastq_pairs([_fq(tmp_path, s, 1)], [_fq(tmp_path, s, 2)])
    sam = tmp_path / "x.sam"
    sam.write_bytes(gzip.open(gold("%s_fastqs_to_sam.sam.gz" % s)).read())
    spairs = smash_cli.sam_pairs(str(sam))
    assert [p[0] for p in pairs] == [p[0] for p in spairs]
    m = smash_cli.reads_matrix(pairs)
    assert np.array_equal(m, smash_cli.reads_matrix(spairs))   # replaceN before / after
    from conftest import interleaved_reads
    assert np.array_equal(m, interleaved_reads(s))


def test_strnum_key_orders_like_samtools_sort_n():
    names = [b"r10", b"r9", b"r009", b"a2b10", b"a2b9", b"r1", b"b"]
    got = sorted(names, key=smash_cli.strnum_key)
    assert got.index(b"r9") < got.index(b"r10")
    assert got.index(b"a2b9") < got.index(b"a2b10")
    assert got.index(b"r1") < got.index(b"r9")


# samtools 1.x strnum_cmp (bam_sort.c) worked by hand: a non-digit on either
# side compares the two bytes, so a byte below '0' sorts before a digit run
STRNUM_CASES = [
    (b"x-5", b"x5", -1),      # '-' (45) < '5'
    (b"a-", b"a1", -1),       # '-' < '1'
    (b"r.1", b"r1", -1),      # '.' (46) < '1'
    (b"r/2", b"r10", -1),     # '/' (47) < '1'
    (b"r 9", b"r1", -1),      # ' ' (32) < '1'
    (b"r9", b"r10", -1),      # longer digit run wins
    (b"r009", b"r10", -1),    # leading zeros skipped
    (b"r01", b"r1", 0),       # equal as numbers: samtools keeps input order
    (b"r1a", b"r01b", -1),    # then the bytes after the run
    (b"r1", b"r1a", -1),      # a prefix sorts first
    (b"a10b2", b"a10b10", -1),
    (b"ra", b"r5", 1),        # 'a' (97) > '5'
]


@pytest.mark.parametrize("a,b,sign", STRNUM_CASES)
def test_strnum_cmp_hand_cases(a, b, sign):
    c = smash_cli.strnum_cmp(a, b)
    assert (c > 0) - (c < 0) == sign
    c = smash_cli.strnum_cmp(b, a)
    assert (c > 0) - (c < 0) == -sign
    # the native port orders the pair the same way (stable on ties)
    got = S.strnum_order(np.array([a, b], "S16")).tolist()
    assert got == ([1, 0] if sign > 0 else [0, 1])


# ---------------------------------------------------------------------------
# GPU: the device-backed subcommands
# ---------------------------------------------------------------------------
def _ref_dir(tmp_path, tiny_fa):
    import shutil
    fa = tmp_path / "tiny.fa"
    shutil.copy(tiny_fa, fa)
    return str(fa)


@pytest.mark.gpu
def test_cli_index_varbin_map_count(tmp_path, tiny_fa, monkeypatch):
    pytest.importorskip("torch")
    fa = _ref_dir(tmp_path, tiny_fa)
    monkeypatch.chdir(tmp_path)
    smash_cli.main(["--ref", fa, "index"])
    cs = open(fa + ".bin/chrom_sizes.txt").read()
    assert cs == open(gold("tiny_chrom_sizes.txt")).read()
    assert open(fa + ".bin/sam_header.txt").read() == open(gold("tiny_sam_header.txt")).read()
    bindir = tmp_path / "bins"
    bindir.mkdir()
    (bindir / "bins.txt").write_text(open(gold("tiny_bins.txt")).read())
    for s in ("s100", "s150"):
        exp_rows = open(gold("%s_varbin.txt" % s)).read()
        part = open(gold("%s_varbin_stats_partial.txt" % s)).read()
        # varbin.py on the golden positions
        smash_cli.main(["varbin", gold("%s_positions.txt" % s), str(bindir / "bins.txt"),
                        "v.txt", "st.txt", fa + ".bin/chrom_sizes.txt"])
        assert open("v.txt").read() == exp_rows
        assert open("st.txt").read().startswith(part)
        # the whole chain from FASTQ
        r1, r2 = _fq(tmp_path, s, 1), _fq(tmp_path, s, 2)
        smash_cli.main(["--ref", fa, "map", s, r1, r2, "--batch", "97"])
        assert open(s + ".positions.txt").read() == open(gold("%s_positions.txt" % s)).read()
        smash_cli.main(["--ref", fa, "count", s, r1, r2, str(bindir), "--out", "c.txt"])
        assert open("c.txt").read() == exp_rows
        assert open(s + ".stats.txt").read().startswith(part)
        # from the unmapped SAM (mummer -samin)
        sam = tmp_path / "x.sam"
        sam.write_bytes(gzip.open(gold("%s_fastqs_to_sam.sam.gz" % s)).read())
        smash_cli.main(["--ref", fa, "count", s, "--sam", str(sam), str(bindir), "--out", "c2.txt"])
        assert open("c2.txt").read() == exp_rows


@pytest.mark.gpu
def test_cli_varbin_edge_positions_hg19_bins(tmp_path, monkeypatch):
    pytest.importorskip("torch")
    monkeypatch.chdir(tmp_path)
    bins = os.path.join(ROOT, "data", "bins", "50000", "bins.txt")
    smash_cli.main(["varbin", gold("edge_positions.txt"), bins, "v.txt", "st.txt",
                    gold("chrom_sizes_hg19.txt")])
    assert open("v.txt").read() == gzip.open(gold("edge_varbin.txt.gz"), "rt").read()
    assert open("st.txt").read().startswith(open(gold("edge_varbin_stats_partial.txt")).read())


@pytest.mark.gpu
@pytest.mark.parametrize("flag,mode", [([], "MAM"), (["-mum"], "MUM"), (["-maxmatch"], "MEM")])
def test_cli_search_triples(tmp_path, tiny_fa, capsys, flag, mode):
    pytest.importorskip("torch")
    fa = _ref_dir(tmp_path, tiny_fa)
    sam = tmp_path / "x.sam"
    sam.write_bytes(gzip.open(gold("s100_fastqs_to_sam.sam.gz")).read())
    smash_cli.main(["--ref", fa, "search"] + flag + [str(sam)])
    got = capsys.readouterr().out.splitlines()
    exp = gzip.open(gold("s100_%s.txt.gz" % mode), "rt").read().splitlines()
    for g, e in zip(got, exp):
        gt, et = g.split("\t"), e.split()
        assert gt[2:] == et[2:], (g[:80], e[:80])


@pytest.mark.gpu
@pytest.mark.parametrize("s", ["s100", "s150"])
def test_cli_memsam_mapout_tagged(tmp_path, tiny_fa, s):
    """`smash_cli memsam -nomap --tag` == `mummer -rcref -nomap -samin -samout`
    piped through mappability_tag (reduced as tools/make_golden.sh does)."""
    pytest.importorskip("torch")
    from test_samout import reduce_line
    fa = _ref_dir(tmp_path, tiny_fa)
    sam = tmp_path / "x.sam"
    sam.write_bytes(gzip.open(gold("%s_fastqs_to_sam.sam.gz" % s)).read())
    out = tmp_path / "mapout" / "mapout.1.txt"
    smash_cli.main(["--ref", fa, "memsam", "-nomap", "--tag", "--out", str(out),
                    "--batch", "97", str(sam)])
    lines = out.read_text().splitlines()
    head = [l for l in lines if l.startswith("@")]
    assert head[0] == "@HD\tVN:1.0\tSO:unsorted" and head[-1].startswith("@PG\tID:longMEM")
    got = sorted(reduce_line(l) for l in lines if not l.startswith("@"))
    exp = sorted(gzip.open(gold("%s_mapout_tagged.txt.gz" % s), "rt").read().splitlines())
    assert got == exp


# ---------------------------------------------------------------------------
# native ingest (smash_fastq_read / smash_strnum_order): host code, CPU tests
# ---------------------------------------------------------------------------
import smashgpu as S  # noqa: E402


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_native_fastq_reader_equals_fastqs_to_sam(tmp_path, s):
    """gzip and plain inputs, the read-1 list split over two files, small
    batches: same pairs, names and bytes as the fastqs_to_sam restatement."""
    pairs = smash_cli.fastq_pairs([_fq(tmp_path, s, 1)], [_fq(tmp_path, s, 2)])
    lines = open(_fq(tmp_path, s, 1), "rb").read().split(b"\n")
    cut = 4 * 37
    a, b = tmp_path / "a.fq.gz", tmp_path / "b.fq"
    with gzip.open(a, "wb") as f:
        f.write(b"\n".join(lines[:cut]) + b"\n")
    b.write_bytes(b"\n".join(lines[cut:]))
    names, reads = S.read_fastq_pairs([str(a), str(b)], [gold("%s_r2.fq.gz" % s)],
                                      batch_pairs=50)
    assert [n for n in names.tolist()] == [p[0] for p in pairs]
    assert np.array_equal(reads, smash_cli.reads_matrix(pairs))


def test_native_fastq_reader_edge_cases(tmp_path):
    """Blank lines, '+name' lines, '>' records, a pair whose mates both have
    no bases dropped (fastqs_to_sam.cpp:80 prints neither); N -> z; a mate of
    another length is an error (the device batches have one read length)."""
    a, b = tmp_path / "a.fq", tmp_path / "b.fq"
    a.write_bytes(b"@a1 1:N:0\nACGTNNAC\n+\nIIIIIIII\n\n@a3 x y\n\n+\n\n>f1 opt\nACGNTACG\n")
    b.write_bytes(b"@b1 2:N:0\r\nTTTTNNTT\r\n+b1\r\nIIIIIIII\r\n@b3 z\n\n+\n\n"
                  b">f2\nNNNNACGT")
    exp = smash_cli.fastq_pairs([str(a)], [str(b)])
    assert [p[0] for p in exp] == [b"a1", b"f1"]
    names, reads = S.read_fastq_pairs([str(a)], [str(b)], batch_pairs=1)
    assert names.tolist() == [b"a1", b"f1"]
    assert reads.tobytes() == b"acgtzzac" + b"ttttzztt" + b"acgztacg" + b"zzzzacgt"
    with pytest.raises(S.SmashError, match="same length"):
        S.read_fastq_pairs([gold("edge_r1.fq")], [gold("edge_r2.fq")], batch_pairs=8)
    with pytest.raises(S.SmashError, match="cannot open"):
        S.read_fastq_pairs(["/nonexistent.fq"], [gold("edge_r2.fq")])


def test_one_empty_mate_is_an_error(tmp_path):
    """fastqs_to_sam.cpp:80 drops only the empty record and prints its mate
    alone, which shifts memsam's read-1 / read-2 alternation (query.cpp:486-
    505) for every later pair; both readers reject such input instead."""
    a, b = tmp_path / "a.fq", tmp_path / "b.fq"
    a.write_bytes(b"@p1\nACGT\n+\nIIII\n@p2\n\n+\n\n")
    b.write_bytes(b"@p1\nTTTT\n+\nIIII\n@p2\nCCCC\n+\nJJJJ\n")
    with pytest.raises(SystemExit, match="no bases"):
        smash_cli.fastq_pairs([str(a)], [str(b)])
    with pytest.raises(S.SmashError, match="no bases"):
        S.read_fastq_pairs([str(a)], [str(b)])


def _strict_fq(path, recs, gz=False, crlf=False, final_nl=True):
    """write 4-line FASTQ records [(name_line, bases, plus_line, quals)]"""
    nl = b"\r\n" if crlf else b"\n"
    body = nl.join(b"\n".join([a, b, c, d]) if not crlf else nl.join([a, b, c, d])
                   for a, b, c, d in recs) + (nl if final_nl else b"")
    if gz:
        with gzip.open(path, "wb") as f:
            f.write(body)
    else:
        path.write_bytes(body)
    return str(path)


@pytest.mark.parametrize("s", ["s100", "s150"])
@pytest.mark.parametrize("threads", [1, 3, 16])
def test_parallel_reader_equals_streaming_reader(tmp_path, s, threads):
    """smash_fastq_read_parallel (csrc/fastq_par.hpp: files mapped / inflated,
    records found per byte range) == smash_fastq_read on the golden reads:
    gzip and plain, the read-1 list split over two files."""
    lines = open(_fq(tmp_path, s, 1), "rb").read().split(b"\n")
    cut = 4 * 37
    a, b = tmp_path / "a.fq.gz", tmp_path / "b.fq"
    with gzip.open(a, "wb") as f:
        f.write(b"\n".join(lines[:cut]) + b"\n")
    b.write_bytes(b"\n".join(lines[cut:]))
    l1, l2 = [str(a), str(b)], [gold("%s_r2.fq.gz" % s)]
    n0, r0 = S.read_fastq_pairs(l1, l2, batch_pairs=50)
    n1, r1 = S.read_fastq_pairs_parallel(l1, l2, threads=threads)
    assert n1.tolist() == n0.tolist() and np.array_equal(r1, r0)


def test_parallel_reader_record_boundaries(tmp_path):
    """Byte ranges that start inside any line: quality lines beginning with
    '@' (and '+'), '+name' lines, CRLF endings, Illumina comments, N -> z,
    a pair with both mates empty (dropped), a last line without '\\n', the
    two lists of different lengths (zip: the shorter ends the pairs);
    thousands of records so the 32 MB ranges of the index cut records."""
    rng = np.random.default_rng(7)
    recs1, recs2 = [], []
    for i in range(40000):
        L = 150
        pick = lambda al, **k: np.array(rng.choice(list(al), L, **k), np.uint8).tobytes()
        q1, q2 = pick(b"@+!#IJ"), pick(b"@+IJ")
        b1 = pick(b"ACGTN", p=[.24, .24, .24, .24, .04])
        b2 = pick(b"ACGTacgtN")
        if i == 777:
            b1, b2, q1, q2 = b"", b"", b"", b""
        recs1.append((b"@r%08d 1:N:0:AC" % i, b1, b"+" if i % 3 else b"+r%08d" % i, q1))
        recs2.append((b"@r%08d 2:N:0:AC" % i, b2, b"+", q2))
    recs2.append((b"@extra", b"A" * 150, b"+", b"I" * 150))
    a = _strict_fq(tmp_path / "a.fq", recs1, final_nl=False)
    b = _strict_fq(tmp_path / "b.fq.gz", recs2, gz=True)
    c = _strict_fq(tmp_path / "c.fq", recs1[:5], crlf=True)
    d = _strict_fq(tmp_path / "d.fq", recs2[:5], crlf=True)
    for l1, l2 in (([a], [b]), ([c], [d]), ([c, a], [d, b])):
        n0, r0 = S.read_fastq_pairs(l1, l2, batch_pairs=4096)
        for T in (1, 7):
            n1, r1 = S.read_fastq_pairs_parallel(l1, l2, threads=T)
            assert n1.tolist() == n0.tolist() and np.array_equal(r1, r0)
    assert len(n1) == 40000 + 4    # (c: 5, a: 40000) - the empty pair; zip drops "extra"


def test_parallel_reader_refuses_what_it_cannot_index(tmp_path):
    """Not strict 4-line FASTQ (blank lines, FASTA records, a '+' line with
    leading blanks, a truncated last record): SMASH_ERR_UNSUPPORTED, and the
    streaming reader reads them; errors are the streaming reader's."""
    bad = [b"@a\nACGT\n+\nIIII\n\n@b\nACGT\n+\nIIII\n",
           b">a\nACGT\n>b\nACGT\n",
           b"@a\nACGT\n +\nIIII\n",
           b"@a\nACGT\n+\nIIII\n@b\nACGT\n",
           # a name line and a bases line longer than the reader's 64 KB
           # line bound (fastq_par.hpp kMaxLine): refused, not parsed past
           b"@" + b"x" * (2 << 20) + b"\nACGT\n+\nIIII\n",
           b"@a\n" + b"A" * (1 << 17) + b"\n+\n" + b"I" * (1 << 17) + b"\n"]
    ok = tmp_path / "ok.fq"
    ok.write_bytes(b"@a\nACGT\n+\nIIII\n@b\nACGT\n+\nIIII\n")
    for k, body in enumerate(bad):
        f = tmp_path / ("bad%d.fq" % k)
        f.write_bytes(body)
        with pytest.raises(S.SmashError, match="not strict"):
            S.read_fastq_pairs_parallel([str(f)], [str(ok)])
    a, b = tmp_path / "a.fq", tmp_path / "b.fq"
    a.write_bytes(b"@p1\nACGT\n+\nIIII\n@p2\n\n+\n\n")
    b.write_bytes(b"@p1\nTTTT\n+\nIIII\n@p2\nCCCC\n+\nJJJJ\n")
    with pytest.raises(S.SmashError, match="no bases"):
        S.read_fastq_pairs_parallel([str(a)], [str(b)])
    b.write_bytes(b"@p1\nTTTT\n+\nIIII\n@p2\nCCCCC\n+\nJJJJJ\n")
    a.write_bytes(b"@p1\nACGT\n+\nIIII\n@p2\nACGT\n+\nIIII\n")
    with pytest.raises(S.SmashError, match="same length"):
        S.read_fastq_pairs_parallel([str(a)], [str(b)])
    with pytest.raises(S.SmashError, match="same length"):
        S.read_fastq_pairs([str(a)], [str(b)])
    with pytest.raises(S.SmashError, match="cannot open"):
        S.read_fastq_pairs_parallel(["/nonexistent.fq"], [str(ok)])


def test_native_strnum_order_equals_samtools_key():
    rng = np.random.default_rng(5)
    alpha = list("ab:_-./ ") + [str(d) for d in range(10)]
    names = [bytes("".join(rng.choice(alpha, rng.integers(1, 12))), "ascii") for _ in range(3000)]
    names += [b"r10", b"r9", b"r009", b"r1", b"", b"0", b"00", b"a2b10", b"a2b9"]
    arr = np.array(names, "S16")
    got = S.strnum_order(arr).tolist()
    exp = sorted(range(len(names)), key=lambda i: smash_cli.strnum_key(names[i]))
    assert got == exp


def _interleaved_fastq_from_sam(s, path):
    """The golden fastqs_to_sam SAM (replaceN applied) as one interleaved FASTQ
    with Illumina '1:N:0' / '2:N:0' comments."""
    out = []
    for line in gzip.open(gold("%s_fastqs_to_sam.sam.gz" % s)):
        f = line.rstrip(b"\n").split(b"\t")
        mate = b"1" if int(f[1]) & 64 else b"2"
        out.append(b"@%s %s:N:0\n%s\n+\n%s\n" % (f[0], mate, f[9], f[10]))
    path.write_bytes(b"".join(out))
    return out


def test_memsam_query_reader_fastq_and_fasta(tmp_path):
    """QueryReader::run's FASTA/FASTQ branch (query.cpp:648-676)."""
    fq = tmp_path / "q.fq"
    _interleaved_fastq_from_sam("s100", fq)
    recs = list(smash_cli.query_records_in(str(fq), True))
    sam = list(smash_cli.sam_records_in(gold("s100_fastqs_to_sam.sam.gz")))
    assert [(r[0], r[1], r[2]) for r in recs] == [(r[0], r[1], r[2]) for r in sam]
    fa = tmp_path / "q.fa"
    fa.write_bytes(b">  x1 2extra  \nAC GT \n\n>y\nAAAA\n>z 1\nC\n")
    recs = list(smash_cli.query_records_in(str(fa), False))
    assert recs == [(b"x1:1", b"ACGT", None, b""), (b"y", b"AAAA", None, b""),
                    (b"z:0", b"C", None, b"")]
    with pytest.raises(SystemExit):
        list(smash_cli.query_records_in(str(fa), True))


@pytest.mark.gpu
def test_cli_memsam_fastq_input(tmp_path, tiny_fa):
    """`mummer -rcref -fastq -nomap -samout` on the same reads as FASTQ: the
    lines equal the -samin golden without the SAM input's optional column."""
    pytest.importorskip("torch")
    from test_samout import reduce_line
    fa = _ref_dir(tmp_path, tiny_fa)
    fq = tmp_path / "q.fq"
    _interleaved_fastq_from_sam("s150", fq)
    out = tmp_path / "m.txt"
    smash_cli.main(["--ref", fa, "memsam", "-nomap", "-fastq", "--tag", "--out", str(out),
                    str(fq)])
    got = sorted(reduce_line(l) for l in out.read_text().splitlines() if not l.startswith("@"))
    exp = sorted("\t".join(x for x in l.split("\t") if not x.startswith("XO:Z:"))
                 for l in gzip.open(gold("s150_mapout_tagged.txt.gz"), "rt").read().splitlines())
    assert got == exp


def test_count_key_set_sizing_does_not_inflate_gzip(tmp_path, monkeypatch):
    """smash_cli count sizes the key set without inflating gzip input (the
    feed inflates each member once and grows the set itself): no FastqShards
    scan, the batch size as the start; plain files: the size bound."""
    import smashgpu as S

    def refuse(*a, **k):
        raise AssertionError("gzip input inflated to size the key set")
    monkeypatch.setattr(S, "FastqShards", refuse)
    monkeypatch.setattr(S, "FastqIndex", refuse)
    g1, g2 = gold("s150_r1.fq.gz"), gold("s150_r2.fq.gz")
    assert smash_cli.fastq_pairs_bound([g1], [g2], 150, 4096) == 4096
    p1, p2 = _fq(tmp_path, "s150", 1), _fq(tmp_path, "s150", 2)
    n = sum(1 for _ in open(p1)) // 4
    assert smash_cli.fastq_pairs_bound([p1], [p2], 150, 4096) >= n
