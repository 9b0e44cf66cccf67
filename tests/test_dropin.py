"""The drop-in command-line surface: the reference scripts' $SMASH_CODE
tools (smash-paper_amd/bin: mummer, fastqs_to_sam, mappability_tag,
varbin.py) run with the reference's own command lines.

CPU: mappability_tag (host code) on the reference's own full mapout lines
against the reference's own tagged output; mummer's argument checks.
GPU (`-m gpu`): index_setup.sh:19-22 and smash_mapping.sh:19-23 as written
(samtools absent: everything up to the BAM conversion), the other query
formats / search modes through `-samout`, binning.sh:36's varbin.py call.
Pinned to tests/golden/*_full.txt.gz (tools/make_golden_r02.sh: the compiled
reference's own output, sorted full lines).
"""
import gzip
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT, gold, read_gz_lines

BIN = os.path.join(ROOT, "smash-paper_amd", "bin")


def _tool(name):
    p = os.path.join(BIN, name)
    if not os.path.exists(p):
        pytest.fail("%s not built (make -C smash-paper_amd)" % p)
    return p


def _ref_dir(tmp_path, tiny_fa, with_map=None):
    """REF.fa plus the side files index_setup.sh:24-31 writes with samtools
    (absent here): chrom_sizes.txt and sam_header.txt."""
    fa = str(tmp_path / "tiny.fa")
    shutil.copy(tiny_fa, fa)
    os.makedirs(fa + ".bin", exist_ok=True)
    shutil.copy(gold("tiny_sam_header.txt"), fa + ".bin/sam_header.txt")
    shutil.copy(gold("tiny_chrom_sizes.txt"), fa + ".bin/chrom_sizes.txt")
    if with_map is not None:
        with open(fa + ".bin/map.bin", "wb") as f:
            f.write(with_map.tobytes())
    return fa


def _body(path_glob_dir):
    lines = []
    for f in sorted(os.listdir(path_glob_dir)):
        for l in open(os.path.join(path_glob_dir, f)):
            if not l.startswith("@"):
                lines.append(l.rstrip("\n"))
    return sorted(lines)


# ---------------------------------------------------------------------------
# CPU
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def mapbin(tiny_ix):
    return tiny_ix.mappability()   # the oracle's map.bin (pinned to the reference's)


@pytest.mark.parametrize("s", ["s100", "s150"])
def test_mappability_tag_cli_equals_reference(tmp_path, tiny_fa, mapbin, s):
    """smash_mapping.sh:23 up to samtools: the header (head -n 100 | grep ^@)
    and the perl-munged body of the reference's own mapout, tagged."""
    fa = _ref_dir(tmp_path, tiny_fa, mapbin)
    sam = tmp_path / "in.sam"
    hdr = open(gold("tiny_mapout_header.txt")).read()
    sam.write_text(hdr + "\n".join(read_gz_lines("%s_mapout_full.txt.gz" % s)) + "\n")
    r = subprocess.run([_tool("mappability_tag"), fa, str(sam)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    out = r.stdout.splitlines()
    assert [l for l in out if l.startswith("@")] == hdr.splitlines()
    got = sorted(l for l in out if not l.startswith("@"))
    assert got == sorted(read_gz_lines("%s_mapout_tagged_full.txt.gz" % s))


def test_mappability_tag_cli_errors(tmp_path, tiny_fa, mapbin):
    """mappability_tag.cpp:55,107-117: usage, unknown contig, a block whose
    left mappability exceeds its length (non-small contig), unexpected CIGAR
    op: message, exit 1, output written up to the failing line."""
    fa = _ref_dir(tmp_path, tiny_fa, mapbin)
    tool = _tool("mappability_tag")
    r = subprocess.run([tool, fa], capture_output=True, text=True)
    assert r.returncode == 1 and "usage" in r.stderr
    line = read_gz_lines("s100_mapout_full.txt.gz")[0]
    f = line.split("\t")
    cases = {
        "Unknown chromosome": f[:2] + ["chrNope"] + f[3:],
        "unexpected cigar": f[:5] + ["10S5I85="] + f[6:],
        # one base blocks: mappability is >= 1 base longer than that
        "mappability too big": f[:2] + ["chr1", "70000", f[4], "1=99S"] + f[6:],
    }
    for msg, fields in cases.items():
        sam = tmp_path / "e.sam"
        sam.write_text(line + "\n" + "\t".join(fields) + "\n")
        r = subprocess.run([tool, fa, str(sam)], capture_output=True, text=True)
        assert r.returncode == 1 and msg in r.stderr, (msg, r.stderr)
        assert r.stdout.startswith(line)


def test_mummer_cli_argument_errors(tmp_path):
    """mummer.cpp:136-147: too few arguments -> usage; -nomap without
    -samout, -fastq with -samin, -mappability without -rcref -> Error, 1.
    No device is touched before these checks."""
    tool = _tool("mummer")
    r = subprocess.run([tool, "-rcref", "x.fa"], capture_output=True, text=True)
    assert r.returncode == 1 and "too few arguments" in r.stderr and "Usage" in r.stderr
    for flags, msg in ((["-rcref", "-nomap"], "-nomap can only be used with -sam_out"),
                       (["-rcref", "-fastq", "-samin"], "-fastq cannot be used with -samin"),
                       (["-mappability"], "-mappability requires -rcref")):
        r = subprocess.run([tool] + flags + ["x.fa", "q"], capture_output=True, text=True)
        assert r.returncode == 1 and r.stderr.startswith("Error") and msg in r.stderr, r.stderr


# ---------------------------------------------------------------------------
# GPU: the scripts' lines as written
# ---------------------------------------------------------------------------
def _bash(script, cwd, env):
    e = dict(os.environ)
    e.update(env)
    r = subprocess.run(["bash", "-c", script], cwd=cwd, env=e, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, (script, r.stdout[-2000:], r.stderr[-2000:])
    return r


@pytest.mark.gpu
def test_index_setup_and_smash_mapping_lines_as_written(tmp_path, tiny_fa):
    """index_setup.sh:19,22 then smash_mapping.sh:19-23 (up to samtools) with
    $SMASH_CODE = smash-paper_amd/bin: the mapout and its tagged form equal
    the reference's own, full lines, sorted."""
    fa = str(tmp_path / "tiny.fa")
    shutil.copy(tiny_fa, fa)
    env = {"SMASH_REF": fa, "SMASH_CODE": BIN}
    # index_setup.sh:19,22 (the first fails on the 'dummy' query, as the
    # reference's does after writing the cache)
    r = subprocess.run(["bash", "-c", "$SMASH_CODE/mummer -verbose -rcref $SMASH_REF dummy"],
                       cwd=tmp_path, env=dict(os.environ, **env), capture_output=True, text=True)
    assert r.returncode == 1 and "unable to open dummy" in r.stderr
    assert os.path.exists(fa + ".bin/rc1.i4.index.sa.bin")
    _bash("$SMASH_CODE/mummer -verbose -rcref -mappability $SMASH_REF $SMASH_REF.bin/map.bin",
          tmp_path, env)
    shutil.copy(gold("tiny_sam_header.txt"), fa + ".bin/sam_header.txt")   # samtools faidx
    shutil.copy(gold("tiny_chrom_sizes.txt"), fa + ".bin/chrom_sizes.txt")
    for s in ("s100", "s150"):
        id_ = "id_" + s
        env2 = dict(env, R1=gold(s + "_r1.fq.gz"), R2=gold(s + "_r2.fq.gz"), ID=id_)
        _bash('$SMASH_CODE/mummer -verbose -rcref -qthreads 12 -nomap -samin -samout $SMASH_REF '
              '<($SMASH_CODE/fastqs_to_sam <(zcat $R1) <(zcat $R2) 1)\n'
              'mv mapout $ID.mapout\n'
              '$SMASH_CODE/mappability_tag $SMASH_REF <(cat $ID.mapout/*.txt | head -n 100 | '
              'grep ^@ ; cat $ID.mapout/*.txt | grep -v ^@ | perl -pe '
              "'s/^(\\S+?)\\/\\S+\\/\\d+/\\1/' ) > $ID.tagged.sam", tmp_path, env2)
        assert _body(str(tmp_path / (id_ + ".mapout"))) == \
            sorted(read_gz_lines("%s_mapout_full.txt.gz" % s))
        tagged = [l.rstrip("\n") for l in open(tmp_path / (id_ + ".tagged.sam"))]
        assert sorted(l for l in tagged if not l.startswith("@")) == \
            sorted(read_gz_lines("%s_mapout_tagged_full.txt.gz" % s))
        hdr = open(gold("tiny_mapout_header.txt")).read().splitlines()
        for f in os.listdir(tmp_path / (id_ + ".mapout")):
            lines = open(tmp_path / (id_ + ".mapout") / f).read().splitlines()
            assert sorted(l for l in lines if l.startswith("@")) == hdr


@pytest.mark.gpu
@pytest.mark.parametrize("kind,args,golden,n", [
    ("fastq", ["-rcref", "-qthreads", "2", "-fastq", "-nomap", "-samout"],
     "s150_mapout_fastq_full", None),
    ("fasta", ["-rcref", "-qthreads", "2", "-nomap", "-samout"], "s150_mapout_fasta_full", None),
    ("sam", ["-rcref", "-qthreads", "2", "-maxmatch", "-nomap", "-samin", "-samout"],
     "s100_60_mapout_MEM_full", 60),
    ("sam", ["-rcref", "-qthreads", "2", "-mum", "-samin", "-samout"],
     "s100_300_mapout_MUM_full", 300),
])
def test_mummer_cli_formats_and_modes(tmp_path, tiny_fa, kind, args, golden, n):
    import golden_queries
    fa = str(tmp_path / "tiny.fa")
    shutil.copy(tiny_fa, fa)
    src = gold(("s150" if golden.startswith("s150") else "s100") + "_fastqs_to_sam.sam.gz")
    q = str(tmp_path / ("q." + kind))
    golden_queries.write(src, kind, q, n)
    r = subprocess.run([_tool("mummer")] + args + [fa, q], cwd=tmp_path, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert _body(str(tmp_path / "mapout")) == sorted(read_gz_lines(golden + ".txt.gz"))


@pytest.mark.gpu
def test_mummer_cli_without_samout_writes_the_header_only(tmp_path, tiny_fa):
    """query.cpp:404-412 never ends its non-SAM lines: the reference's
    mapout file holds the header alone, and so does ours."""
    fa = str(tmp_path / "tiny.fa")
    shutil.copy(tiny_fa, fa)
    q = str(tmp_path / "q.fa")
    import golden_queries
    golden_queries.write(gold("s100_fastqs_to_sam.sam.gz"), "fasta", q, 20)
    r = subprocess.run([_tool("mummer"), "-rcref", "-l", "20", fa, q], cwd=tmp_path,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    files = os.listdir(tmp_path / "mapout")
    assert len(files) == 1
    assert open(tmp_path / "mapout" / files[0]).read() == open(gold("tiny_mapout_header.txt")).read() \
        or sorted(open(tmp_path / "mapout" / files[0]).read().splitlines()) == \
        sorted(open(gold("tiny_mapout_header.txt")).read().splitlines())


@pytest.mark.gpu
@pytest.mark.parametrize("s", ["s100", "s150"])
def test_binning_varbin_line_as_written(tmp_path, s):
    """binning.sh:36: `$SMASH_CODE/varbin.py $id.positions.txt $bins varbin.txt
    $id.stats.txt $SMASH_REF.bin/chrom_sizes.txt`: bin rows equal the real
    varbin.py's (tests/golden/s*_varbin.txt), stats its first three columns."""
    fa = str(tmp_path / "tiny.fa")
    open(fa, "w").close()
    os.makedirs(fa + ".bin")
    shutil.copy(gold("tiny_chrom_sizes.txt"), fa + ".bin/chrom_sizes.txt")
    shutil.copy(gold("%s_positions.txt" % s), tmp_path / "id.positions.txt")
    bindir = tmp_path / "bins"
    os.makedirs(bindir)
    shutil.copy(gold("tiny_bins.txt"), bindir / "bins.txt")
    _bash("$SMASH_CODE/varbin.py $id.positions.txt $bins varbin.txt $id.stats.txt "
          "$SMASH_REF.bin/chrom_sizes.txt > $id.varbin.out.txt".replace("$id", "id")
          .replace("$bins", str(bindir / "bins.txt")), tmp_path,
          {"SMASH_REF": fa, "SMASH_CODE": BIN})
    got = [l.split("\t")[:4] for l in open(tmp_path / "varbin.txt").read().splitlines()]
    exp = [l.split("\t")[:4] for l in open(gold("%s_varbin.txt" % s)).read().splitlines()]
    assert got == exp
    st = open(tmp_path / "id.stats.txt").read().splitlines()[1].split("\t")
    g = open(gold("%s_varbin_stats_partial.txt" % s)).read().splitlines()[1].split("\t")
    assert st[:3] == g[:3]


# ---------------------------------------------------------------------------
# GPU: mummer without -rcref (the forward-only text, fasta.cpp:160-169),
# pinned to tools/make_golden_r03.sh's reference output
# ---------------------------------------------------------------------------
def _chr1_fa(tmp_path, tiny_fa):
    """tiny.fa up to its second '>' line (awk '/^>/{n++} n<2')."""
    out, n = [], 0
    for l in open(tiny_fa):
        if l.startswith(">"):
            n += 1
        if n < 2:
            out.append(l)
    fa = str(tmp_path / "chr1.fa")
    open(fa, "w").write("".join(out))
    return fa


@pytest.mark.gpu
def test_mummer_without_rcref_writes_the_reference_rc0_cache(tmp_path, tiny_fa):
    """`mummer tiny.fa dummy`: the rc0.* cache (text, contig table, SA, ISA,
    LCP) built on the device equals the reference's byte for byte (lcp.m.bin
    with its uninitialised padding masked); no map.bin (-mappability requires
    -rcref); the cache loads back through smash_index_load_layout."""
    import hashlib
    fa = str(tmp_path / "tiny.fa")
    shutil.copy(tiny_fa, fa)
    r = subprocess.run([_tool("mummer"), fa, "dummy"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 1 and "unable to open dummy" in r.stderr, r.stderr
    sums = {l.split()[0]: (l.split()[1], int(l.split()[2]))
            for l in open(gold("tiny_index_rc0.sha256"))}
    for name, (h, size) in sums.items():
        if name.endswith(":masked") or name == "rc0.i4.index.lcp.m.bin":
            continue
        b = open(fa + ".bin/" + name, "rb").read()
        assert (hashlib.sha256(b).hexdigest(), len(b)) == (h, size), name
    m = np.fromfile(fa + ".bin/rc0.i4.index.lcp.m.bin", np.uint64).reshape(-1, 2).copy()
    m[:, 1] &= 0xFFFFFFFF
    assert hashlib.sha256(m.tobytes()).hexdigest() == sums["rc0.i4.index.lcp.m.bin:masked"][0]
    assert not os.path.exists(fa + ".bin/map.bin")
    assert not os.path.exists(fa + ".bin/rc1.ref.bin")
    import smashgpu as S
    ix = S.Index.load(fa, rcref=False)
    assert not ix.rcref and ix.info.map_bytes == 0 and ix.contigs == S.Index.from_fasta(
        fa, rcref=False).contigs
    with pytest.raises(S.SmashError, match="-mappability requires -rcref"):
        S.check(S.lib().smash_mappability_scan(ix.h, 0, 10, 36, None, None, None, 0, None, None,
                                               None), "smash_mappability_scan")


@pytest.mark.gpu
@pytest.mark.parametrize("kind,args,golden,n", [
    ("sam", ["-qthreads", "2", "-nomap", "-samin", "-samout"], "s150_chr1_mapout_fwd_full", None),
    ("sam", ["-qthreads", "2", "-maxmatch", "-nomap", "-samin", "-samout"],
     "s100_60_chr1_mapout_MEM_fwd_full", 60),
    ("sam", ["-qthreads", "2", "-mum", "-samin", "-samout"],
     "s100_300_chr1_mapout_MUM_fwd_full", 300),
])
def test_mummer_without_rcref_modes(tmp_path, tiny_fa, kind, args, golden, n):
    """MAM / MEM / MUM on the forward-only text of one contig: the reference's
    own -samout lines (forward hits only, every record's XS '+'), full lines,
    and its header (one @SQ per contig, fasta.cpp:247)."""
    import golden_queries
    fa = _chr1_fa(tmp_path, tiny_fa)
    src = gold(("s150" if golden.startswith("s150") else "s100") + "_fastqs_to_sam.sam.gz")
    q = str(tmp_path / ("q." + kind))
    golden_queries.write(src, kind, q, n)
    r = subprocess.run([_tool("mummer")] + args + [fa, q], cwd=tmp_path, capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert _body(str(tmp_path / "mapout")) == sorted(read_gz_lines(golden + ".txt.gz"))
    hdr = sorted(open(gold("tiny_chr1_fwd_mapout_header.txt")).read().splitlines())
    for f in os.listdir(tmp_path / "mapout"):
        lines = open(tmp_path / "mapout" / f).read().splitlines()
        assert sorted(l for l in lines if l.startswith("@")) == hdr


@pytest.mark.gpu
def test_mummer_without_rcref_samout_on_every_second_contig_fails_as_the_reference(
        tmp_path, tiny_fa):
    """The reference's absolute-position map steps over the contigs by 2
    without -rcref too (query.cpp:547-551), so a -samout line on chr2 / chrM
    ends its run: the worker thread prints "map::at" and exits 1
    (query.cpp:522-535).  Recorded in tests/golden/tiny_fwd_samout_error.txt."""
    fa = str(tmp_path / "tiny.fa")
    shutil.copy(tiny_fa, fa)
    q = str(tmp_path / "s150.sam")
    with open(q, "wb") as f:
        f.write(gzip.open(gold("s150_fastqs_to_sam.sam.gz")).read())
    r = subprocess.run([_tool("mummer"), "-qthreads", "2", "-nomap", "-samin", "-samout", fa, q],
                       cwd=tmp_path, capture_output=True, text=True, timeout=600)
    want = open(gold("tiny_fwd_samout_error.txt")).read().splitlines()
    assert want[0] == "exit 1"
    assert r.returncode == 1 and r.stderr.splitlines() == want[1:], r.stderr
