"""The mapout SAM writer (`mummer -rcref -qthreads 2 -nomap -samin -samout`,
query.cpp:231-415) + mappability_tag's L/R columns (mappability_tag.cpp:93-124).

Pinned to the reference's own output: tests/golden/s{100,150}_mapout_tagged.txt.gz
are the compiled reference's mapout lines after mappability_tag, reduced by
tools/make_golden.sh (fields 1-9 + the XM..XC/L0/R0 tags, SEQ/QUAL dropped as
they are the inputs themselves) and sorted.  Inputs: the reference's
fastqs_to_sam output (s*_fastqs_to_sam.sam.gz) and, for the CPU test, its own
MAM triples (s*_MAM.txt.gz).

CPU: the host formatter (smash_sam_format, pure host code in libsmashgpu) on
records restated here from the reference triples.  GPU (`-m gpu`): the whole
product path -- smash_map_batch -> smash_sam_records -> smash_sam_format --
against the same golden, and the device records against the restatement.
"""
import gzip
import re

import numpy as np
import pytest

from conftest import gold, read_gz_lines

import smashgpu as S

TAGS = re.compile(r"^(XM|XU|XE|XS|NH|HI|L0|R0|cc|cp|xo|xc|CC|CP|XO|XC):")


def load_sam_input(s):
    """QueryReader::run with -samin (query.cpp:638-646): name + ':0'/':1' by
    flag, SEQ, QUAL, optional columns each prefixed by a tab."""
    names, seqs, quals, opts = [], [], [], []
    with gzip.open(gold("%s_fastqs_to_sam.sam.gz" % s), "rb") as f:
        for line in f:
            if line.startswith(b"@"):
                continue
            c = line.rstrip(b"\n").split(b"\t")
            flag = int(c[1])
            names.append(c[0] + (b":0" if flag & 64 else b":1" if flag & 128 else b""))
            seqs.append(c[9])
            quals.append(c[10])
            opts.append(b"".join(b"\t" + x for x in c[11:]))
    L = len(seqs[0])
    assert all(len(x) == L for x in seqs)
    reads = np.frombuffer(b"".join(seqs), np.uint8).reshape(-1, L)
    return names, seqs, quals, opts, np.frombuffer(reads.tobytes().lower(), np.uint8).reshape(-1, L)


def reduce_line(line):
    """make_golden.sh's awk: fields 1-9, then the kept tags from field 12 on."""
    f = line.split("\t")
    return "\t".join(f[:9] + [x for x in f[11:] if TAGS.match(x)])


def py_records(ix, mapbin, offsets, reads, triples, cap):
    """Restatement of k_sam_recs: Alignment::resolve (query.cpp:68-97), XE of the
    diagonal (:270-274), mappability_tag L/R of the block (u32 arithmetic)."""
    n, L = reads.shape
    rec = np.zeros(n * cap, S.SAM_REC)
    cnt = np.zeros(n, np.uint32)
    sp = ix.startpos.astype(np.int64)
    T = ix.T
    N = ix.N
    for r in range(n):
        cnt[r] = len(triples[r])
        for k, (ref, q, ln) in enumerate(triples[r]):
            si = int(np.searchsorted(sp, ref, side="right")) - 1
            rcpos = ref - q
            pos = rcpos - int(sp[si])
            extra = L - ln - q
            o = rec[r * cap + k]
            if si & 1:
                si -= 1
                pos = int(ix.sizes[si]) - pos - L
                prefix, suffix, rc = extra, q, 1
            else:
                prefix, suffix, rc = q, extra, 0
            xe = 0
            for j in range(L):
                rp = rcpos + j
                xe += 0 <= rp < N and T[rp] == reads[r, j]
            left = right = 0
            if pos >= 0:
                ab = (int(offsets[si >> 1]) + pos + 1) & 0xFFFFFFFF
                li = (ab + prefix + ln - 1) & 0xFFFFFFFF
                ri = (ab + prefix - 1) & 0xFFFFFFFF
                la, ra = 2 + 2 * li, 2 + 2 * ri + 1
                lm = int(mapbin[la]) if la < len(mapbin) else 0
                rm = int(mapbin[ra]) if ra < len(mapbin) else 0
                left = lm - 1 if lm else 255
                right = rm if rm else 255
            rec[r * cap + k] = (pos, si >> 1, xe, prefix, ln, suffix, q, rc, 0, 0, left, right, 0)
    return rec, cnt


@pytest.fixture(scope="module")
def tables(tiny_ix):
    mapbin = tiny_ix.mappability()
    sizes = [int(x) for x in tiny_ix.sizes[0::2]]
    offsets = np.cumsum([0] + sizes[:-1]).astype(np.uint32)
    small = np.array([1 if ("_gl000" in c or "chrM" in c) else 0 for c in tiny_ix.contigs],
                     np.uint8)
    return mapbin, offsets, small


def _golden(s):
    return sorted(read_gz_lines("%s_mapout_tagged.txt.gz" % s))


def _check_full_columns(text, seqs, quals, names):
    """SEQ/QUAL (query.cpp:365-376): forward as read, reverse strand as the
    reverse complement with QUAL reversed."""
    by_name = {}
    for nm, sq, q in zip(names, seqs, quals):
        flag = 64 if nm.endswith(b":0") else 128
        by_name[(nm[:-2].decode(), flag)] = (sq.decode(), q.decode())
    comp = str.maketrans("acgtACGT", "tgcaTGCA")
    for line in text.decode().splitlines():
        f = line.split("\t")
        sq, q = by_name[(f[0], int(f[1]) & 192)]
        if int(f[1]) & 16:
            assert f[9] == sq[::-1].translate(comp) and f[10] == q[::-1]
        else:
            assert f[9] == sq and f[10] == q


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_formatter_on_reference_matches_equals_mapout(tiny_ix, tables, s):
    mapbin, offsets, small = tables
    names, seqs, quals, opts, reads = load_sam_input(s)
    triples = [[tuple(map(int, x.split(","))) for x in l.split()[2:]]
               for l in read_gz_lines("%s_MAM.txt.gz" % s)]
    assert len(triples) == len(names)
    cap = reads.shape[1] - 20 + 1
    rec, cnt = py_records(tiny_ix, mapbin, offsets, reads, triples, cap)
    text, terr = S.sam_format(tiny_ix.contigs, rec, cnt, cap, names, seqs, quals, opts,
                              nomap=True, tag=True, small_chr=small)
    assert terr == 0
    got = sorted(reduce_line(l) for l in text.decode().splitlines())
    assert got == _golden(s)
    _check_full_columns(text, seqs, quals, names)


def test_formatter_edge_cases(tiny_ix):
    """No -nomap: unmapped reads print nothing and their mate gets no mate
    columns (set_mate needs n_alignments on both sides, query.cpp:424-438);
    a record with pos < 0 is erased (query.cpp:243-250); an odd trailing read
    is printed alone (query.cpp:506-510); tag error surfaces."""
    cap = 4
    rec = np.zeros(3 * cap, S.SAM_REC)
    cnt = np.array([1, 1, 1], np.uint32)
    rec[0] = (99, 0, 30, 0, 30, 70, 0, 0, 0, 0, 200, 3, 0)   # left 200 > 30: tag error
    rec[cap] = (-5, 0, 30, 0, 30, 70, 0, 0, 0, 0, 0, 0, 0)   # erased
    rec[2 * cap] = (7, 1, 40, 60, 40, 0, 60, 1, 0, 0, 1, 1, 0)
    names = [b"a:0", b"a:1", b"b:0"]
    seqs = [b"A" * 100, b"C" * 100, b"ACGTN" * 20]
    text, terr = S.sam_format(tiny_ix.contigs, rec, cnt, cap, names, seqs, nomap=False,
                              tag=True)
    lines = text.decode().splitlines()
    assert terr == 1
    assert len(lines) == 2
    f0 = lines[0].split("\t")
    assert f0[:9] == ["a", "65", tiny_ix.contigs[0], "100", "50", "30=70S", "*", "0", "0"]
    assert f0[10] == "!" * 100 and "L0:i:200\tR0:i:3" in lines[0]
    f1 = lines[1].split("\t")
    assert f1[:6] == ["b", "81", tiny_ix.contigs[1], "8", "50", "60S40="]
    assert f1[9] == "NACGT" * 20
    # with -nomap the erased read prints as unmapped, mate columns set both ways
    text, _ = S.sam_format(tiny_ix.contigs, rec, cnt, cap, names, seqs, nomap=True)
    lines = text.decode().splitlines()
    assert len(lines) == 3
    f1 = lines[1].split("\t")
    assert f1[:9] == ["a", "133", tiny_ix.contigs[0], "100", "0", "*",
                      tiny_ix.contigs[0], "100", "0"]
    assert lines[1].endswith("XM:i:0\tNH:i:0")
    assert lines[0].split("\t")[1] == "73"   # mate unmapped: own best as mate
    assert lines[0].split("\t")[6:8] == [tiny_ix.contigs[0], "100"]


@pytest.mark.gpu
@pytest.mark.parametrize("s", ["s100", "s150"])
def test_device_mapout_equals_reference(tiny_fa, tiny_ix, tables, s):
    torch = pytest.importorskip("torch")
    mapbin, offsets, small = tables
    names, seqs, quals, opts, reads = load_sam_input(s)
    gix = S.Index.from_fasta(tiny_fa)
    d = torch.from_numpy(np.ascontiguousarray(reads)).cuda()
    text, terr = S.sam_lines(gix, d, reads.shape[1], names, seqs, quals, opts, nomap=True,
                             tag_offsets=offsets, small_chr=small)
    assert terr == 0
    got = sorted(reduce_line(l) for l in text.decode().splitlines())
    assert got == _golden(s)
    _check_full_columns(text, seqs, quals, names)


@pytest.mark.gpu
@pytest.mark.parametrize("s", ["s100", "s150"])
def test_device_records_equal_restatement(tiny_fa, tiny_ix, tables, s):
    torch = pytest.importorskip("torch")
    mapbin, offsets, small = tables
    names, seqs, quals, opts, reads = load_sam_input(s)
    triples = [[tuple(map(int, x.split(","))) for x in l.split()[2:]]
               for l in read_gz_lines("%s_MAM.txt.gz" % s)]
    cap = reads.shape[1] - 20 + 1
    exp, ecnt = py_records(tiny_ix, mapbin, offsets, reads, triples, cap)
    gix = S.Index.from_fasta(tiny_fa)
    d = torch.from_numpy(np.ascontiguousarray(reads)).cuda()
    got, cnt = S.sam_records(gix, d, reads.shape[0], reads.shape[1], cap, tag_offsets=offsets)
    assert cnt.tolist() == ecnt.tolist()
    off = np.concatenate([[0], np.cumsum(cnt.astype(np.int64))])   # packed, read after read
    assert len(got) == off[-1]
    for r in range(reads.shape[0]):
        a, b = got[off[r]:off[r + 1]], exp[r * cap:r * cap + cnt[r]]
        assert a.tobytes() == b.tobytes(), (r, a, b)


def _golden_full(s, tagged):
    return sorted(read_gz_lines("%s_mapout%s_full.txt.gz" % (s, "_tagged" if tagged else "")))


@pytest.mark.parametrize("tagged", [False, True])
@pytest.mark.parametrize("s", ["s100", "s150"])
def test_formatter_full_lines_equal_reference(tiny_ix, tables, s, tagged):
    """Every column (SEQ reverse-complemented on '-' hits, QUAL reversed, the
    XO:Z comment from fastqs_to_sam) against the reference's own mapout of
    smash_mapping.sh:19 as written (-verbose -rcref -qthreads 12 -nomap
    -samin -samout) and, tagged, after mappability_tag (:23)."""
    mapbin, offsets, small = tables
    names, seqs, quals, opts, reads = load_sam_input(s)
    triples = [[tuple(map(int, x.split(","))) for x in l.split()[2:]]
               for l in read_gz_lines("%s_MAM.txt.gz" % s)]
    cap = reads.shape[1] - 20 + 1
    rec, cnt = py_records(tiny_ix, mapbin, offsets, reads, triples, cap)
    text, terr = S.sam_format(tiny_ix.contigs, rec, cnt, cap, names, seqs, quals, opts,
                              nomap=True, tag=tagged, small_chr=small)
    assert terr == 0
    assert sorted(text.decode().splitlines()) == _golden_full(s, tagged)
    # the packed layout (cap 0, smash_sam_records_packed) formats identically
    packed = np.concatenate([rec[r * cap:r * cap + cnt[r]] for r in range(len(cnt))])
    text0, terr0 = S.sam_format(tiny_ix.contigs, packed, cnt, 0, names, seqs, quals, opts,
                                nomap=True, tag=tagged, small_chr=small)
    assert (text0, terr0) == (text, terr)


@pytest.mark.parametrize("mode,n,golden,nomap", [("MEM", 60, "s100_60_mapout_MEM_full", True),
                                                 ("MUM", 300, "s100_300_mapout_MUM_full", False)])
def test_formatter_other_modes_equal_reference(tiny_ix, tables, mode, n, golden, nomap):
    """-maxmatch / -mum through -samout: the reference's own triples (in the
    order longSA::MEM / MUM emit them) formatted on the host == the
    reference's full mapout lines.  Under -maxmatch many alignments tie in
    to_print order (qpos, rc); the order of the tie is std::sort's over the
    to_merge order, as in query.cpp:292."""
    mapbin, offsets, small = tables
    names, seqs, quals, opts, reads = load_sam_input("s100")
    names, seqs, quals, opts, reads = names[:n], seqs[:n], quals[:n], opts[:n], reads[:n]
    triples = [[tuple(map(int, x.split(","))) for x in l.split()[2:]]
               for l in read_gz_lines("s100_%s.txt.gz" % mode)][:n]
    cap = max(1, max(len(t) for t in triples))
    rec, cnt = py_records(tiny_ix, mapbin, offsets, reads, triples, cap)
    text, terr = S.sam_format(tiny_ix.contigs, rec, cnt, cap, names, seqs, quals, opts,
                              nomap=nomap, tag=False, small_chr=small)
    assert sorted(text.decode().splitlines()) == sorted(read_gz_lines(golden + ".txt.gz"))
