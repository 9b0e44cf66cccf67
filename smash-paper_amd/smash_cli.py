"""smash_cli -- the reference's command-line surface over the MI355X path.

The reference is driven by three shell scripts around its binaries; each
subcommand below takes the same inputs and writes the same files:

  index REF.fa                  index_setup.sh: REF.fa.bin/ cache (rc1.*,
                                `mummer -rcref`), map.bin (`mummer -rcref
                                -mappability`), chrom_sizes.txt, sam_header.txt
  map ID "R1.gz.." "R2.gz.."    smash_mapping.sh: fastqs_to_sam | mummer -samin |
                                mappability_tag | samtools sort -n | smashMEM.py
                                0 0 10000 4 | awk/perl -> ID.positions.txt
  varbin POS BINS OUT STATS CS  varbin.py's five arguments (binning.sh:36)
  count ID "R1.gz.." "R2.gz.." BINDIR
                                map + varbin fused on the device, no positions
                                file: ID.varbin.txt and ID.stats.txt
  memsam [-nomap] [--tag] QUERY.sam
                                `mummer -rcref -samin -samout [-nomap]`: the
                                mapout SAM file; --tag adds mappability_tag's
                                L/R columns (the next smash_mapping.sh stage)
  search [-mum|-maxmatch] [-l N] REF.fa QUERY
                                mummer's match triples for FASTA/FASTQ/SAM queries
                                (one line per read: name, then ref,query,len)

REF.fa comes from --ref or $SMASH_REF as in the scripts.  Every computation
runs in libsmashgpu.so (include/smash_gpu.h); without it the commands fail.
Pairs are processed in `samtools sort -n` order (strnum_cmp,
smash_mapping.sh:23), read 1 before read 2.
"""
from __future__ import annotations

import argparse
import functools
import gzip
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)
import smashgpu as S  # noqa: E402


# ---------------------------------------------------------------------------
# inputs
# ---------------------------------------------------------------------------
def _open(path):
    if path == "-":
        return sys.stdin.buffer
    with open(path, "rb") as f:
        magic = f.read(2)
    return gzip.open(path, "rb") if magic == b"\x1f\x8b" else open(path, "rb")


def fastq_records(path):
    """(name, optional, bases) per record, parsed as fastqs_to_sam does
    (fastqs_to_sam.cpp:48-76): '@' or '>' records, name = first token after
    the marker, `optional` = the second token, FASTQ: '+' line and qualities."""
    f = _open(path)
    lines = iter(f)
    for line in lines:
        line = line.strip()
        if not line:
            continue
        mark, rest = line[:1], line[1:]
        if mark not in (b"@", b">"):
            raise SystemExit("Fastq @ parse error: %r" % line[:40])
        tok = rest.split()
        if not tok:
            raise SystemExit("Problem reading read name")
        bases = next(lines, b"").rstrip(b"\r\n")
        if mark == b"@":
            plus = next(lines, b"").strip()
            if plus[:1] != b"+":
                raise SystemExit("Fastq + parse error")
            next(lines, None)
        yield tok[0], (tok[1] if len(tok) > 1 else b""), bases


def fastq_pairs(r1s, r2s):
    """Interleaved mates of the FASTQ lists (zcat r1s / zcat r2s, as
    smash_mapping.sh:19 feeds fastqs_to_sam); a pair whose mates both have no
    bases is dropped (fastqs_to_sam.cpp:80 prints neither); a pair with ONE
    empty mate is an error (fastqs_to_sam would print the other mate alone,
    misaligning memsam's mate alternation, query.cpp:486-505)."""
    def chain(paths):
        for p in paths:
            yield from fastq_records(p)
    out = []
    for a, b in zip(chain(r1s), chain(r2s)):
        if a[2] and b[2]:
            out.append((a[0], a[2], b[2]))
        elif a[2] or b[2]:
            raise SystemExit("one mate of pair %s has no bases" % a[0].decode(errors="replace"))
    return out


def sam_pairs(path):
    """Mate pairs of an unmapped SAM (fastqs_to_sam output, mummer -samin):
    consecutive lines, flag 64 = read 1 (query.cpp:614-687)."""
    out, pend = [], None
    for line in _open(path):
        if line.startswith(b"@"):
            continue
        f = line.rstrip(b"\r\n").split(b"\t")
        if len(f) < 10:
            continue
        flag = int(f[1])
        if flag & 64:
            pend = (f[0], f[9])
        elif flag & 128 and pend is not None:
            out.append((pend[0], pend[1], f[9]))
            pend = None
    return out


def strnum_cmp(a: bytes, b: bytes) -> int:
    """samtools sort -n's strnum_cmp (bam_sort.c, samtools 1.x; samtools is
    absent here, so the version is unpinned): bytes compare one by one; where
    both sides are at a digit, leading zeros are skipped, matching digits
    walked, the longer digit run wins, else the first differing digit."""
    i = j = 0
    na, nb = len(a), len(b)

    def at(s, n, k):
        return s[k] if k < n else 0

    def isd(c):
        return 48 <= c <= 57
    while at(a, na, i) and at(b, nb, j):
        ca, cb = at(a, na, i), at(b, nb, j)
        if not isd(ca) or not isd(cb):
            if ca != cb:
                return ca - cb
            i += 1
            j += 1
        else:
            while at(a, na, i) == 48:
                i += 1
            while at(b, nb, j) == 48:
                j += 1
            while isd(at(a, na, i)) and at(a, na, i) == at(b, nb, j):
                i += 1
                j += 1
            diff = at(a, na, i) - at(b, nb, j)
            while isd(at(a, na, i)) and isd(at(b, nb, j)):
                i += 1
                j += 1
            if isd(at(a, na, i)):
                return 1
            if isd(at(b, nb, j)):
                return -1
            if diff:
                return diff
    return 1 if at(a, na, i) else -1 if at(b, nb, j) else 0


strnum_key = functools.cmp_to_key(strnum_cmp)


def reads_matrix(pairs):
    """[2n, L] uint8 mates (read 1, read 2, ...) after replaceN + lowercasing
    (fastqs_to_sam.cpp:74 with argc == 4, query.cpp:125-144)."""
    if not pairs:
        return np.zeros((0, 0), np.uint8)
    L = len(pairs[0][1])
    if any(len(a) != L or len(b) != L for _, a, b in pairs):
        raise SystemExit("all mates must have the same length (the device batches are "
                         "fixed-length); split the input by read length")
    raw = np.frombuffer(b"".join(a + b for _, a, b in pairs), np.uint8).reshape(-1, L)
    return S.prepare_reads(raw)


def contig_offsets(ix, chrom_sizes):
    return {off: name for name, off in chrom_sizes.items()}


# ---------------------------------------------------------------------------
# outputs (varbin.py:95-114)
# ---------------------------------------------------------------------------
def write_varbin(bins_rows, counts, total, dups, kept, out_path, stats_path):
    nb = len(bins_rows)
    print(nb)
    print(nb)
    if kept == 0:
        raise SystemExit("ZeroDivisionError: no read kept (varbin.py:96)")
    with open(out_path, "w") as o:
        for row, c in zip(bins_rows, counts):
            ratio = float(int(c)) / (float(kept) / float(nb))
            o.write("\t".join(row[0:3]) + "\t" + str(int(c)) + "\t" + repr(ratio) + "\n")
    with open(stats_path, "w") as o:
        med = sorted(int(c) for c in counts)[nb // 2]
        o.write("TotalReads\tDupsRemoved\tReadsKept\tMedianBinCount\n")
        o.write("%d\t%d\t%d\t%d\n" % (total, dups, kept, med))


# ---------------------------------------------------------------------------
# commands
# ---------------------------------------------------------------------------
def _ref(args):
    ref = args.ref or os.environ.get("SMASH_REF", "")
    if not ref or not os.path.isfile(ref):
        raise SystemExit("export SMASH_REF variable as fasta file path")
    return ref


def load_index(ref, device=0):
    if os.path.isdir(ref + ".bin") and any(
            os.path.exists(ref + ".bin/rc1.i%d.index.bin" % w) for w in (4, 8)):
        return S.Index.load(ref, device=device)
    return S.Index.from_fasta(ref, device=device)


def cmd_index(args):
    ref = _ref(args)
    if os.path.exists(ref + ".bin") and not args.force:
        raise SystemExit("binary index directory %s.bin already exists - quitting" % ref)
    ix = S.Index.from_fasta(ref, device=args.device)
    ix.save(ref)
    d = ref + ".bin"
    n = 0
    with open(os.path.join(d, "chrom_sizes.txt"), "w") as cs, \
            open(os.path.join(d, "sam_header.txt"), "w") as sh:
        for name, size in zip(ix.contigs, ix.contig_sizes):
            if "_" not in name:
                cs.write("%s\t%d\t%d\n" % (name, size, n))
                n += size
            sh.write("@SQ\tSN:%s\tLN:%d\n" % (name, size))
    print("index: N=%d, %.1f GB in HBM, %.1f s" % (ix.N, ix.info.device_bytes / 1e9,
                                                  ix.info.build_seconds), file=sys.stderr)


class _Run:
    """Index + pipeline + batches over pairs in name order."""

    def __init__(self, args, bins_path=None):
        import torch
        self.torch = torch
        self.ref = _ref(args)
        self.ix = load_index(self.ref, args.device)
        cs_path = args.chrom_sizes or self.ref + ".bin/chrom_sizes.txt"
        self.cs = S.read_chrom_sizes(cs_path)
        if bins_path:
            self.bins_rows, self.starts = S.read_bins(bins_path)
        else:
            self.bins_rows, self.starts = [], np.zeros(1, np.int64)
        if args.sam:
            pairs = sam_pairs(args.sam)
            pairs.sort(key=lambda p: strnum_key(p[0]))
            self.reads = reads_matrix(pairs)
            self.n = len(pairs)
        else:   # native ingest (smash_fastq_read) + samtools sort -n order
            names, reads = S.read_fastq_pairs(args.reads1.split(), args.reads2.split())
            order = S.strnum_order(names)
            n = len(names)
            self.reads = reads.reshape(n, -1)[order].reshape(2 * n, -1) if n else reads
            self.n = n
        self.batch = min(args.batch, max(self.n, 1))
        self.dev = torch.device("cuda", args.device)

    def run(self, on_batch):
        torch = self.torch
        L = self.reads.shape[1] if self.n else 150
        pipe = S.Pipeline(self.ix, self.cs, self.starts, L, self.batch,
                          dedup_capacity=max(self.n, 1))
        counts = torch.zeros(len(self.starts), dtype=torch.int64, device=self.dev)
        pipe.reset()
        for b0 in range(0, self.n, self.batch):
            b1 = min(self.n, b0 + self.batch)
            d = torch.from_numpy(np.ascontiguousarray(self.reads[2 * b0:2 * b1])).to(self.dev)
            pipe.count_batch(d, b1 - b0, counts)
            on_batch(pipe)
        st = pipe.stats(raise_on_error=False)
        if st.error:
            raise SystemExit("%s: %s" % (_err_label(st.error), S.ERRORS.get(st.error, st.error)))
        return counts.cpu().numpy(), st


def cmd_map(args):
    run = _Run(args)
    names = contig_offsets(run.ix, run.cs)
    with open(args.id + ".positions.txt", "w") as out:
        def emit(pipe):
            pos0, absp = pipe.positions()
            for p, a in zip(pos0.tolist(), absp.tolist()):
                out.write("%s %d\n" % (names[a - p], p))
        _, st = run.run(emit)
    with open(args.id + ".smash.summary.txt", "w") as o:   # smashMEM.py:230
        o.write("%d dupes\t%d non-dupes\n" % (st.dupe_pairs, st.key_pairs - st.dupe_pairs))


def _is_gzip(path):
    with open(path, "rb") as f:
        return f.read(2) == b"\x1f\x8b"


def fastq_pairs_bound(r1, r2, L, batch=1 << 20):
    """The starting key-set capacity of a file-fed run.  Plain files: a
    record is at least 2 L + 6 bytes ("@x", seq, "+", qual), so the sizes
    bound the pairs.  Gzip files are not inflated to count them (that would
    inflate every member twice, once here and once in the feed): the set
    starts at one batch and smash_count_fastq grows it, doubling, before a
    batch could overflow it (smash_pipeline_reserve_keys moves the held keys).
    A set HBM cannot grow fails the run (SMASH_ERR_NOMEM), never cuts it."""
    if any(_is_gzip(p) for p in r1 + r2):
        return max(int(batch), 1)
    n = 0
    for p in r1:
        n += os.path.getsize(p) // (2 * L + 6) + 1
    return max(n, 1)


def _err_label(code):
    """the stage a pipeline data error belongs to: the tag throws are
    mappability_tag's (mappability_tag.cpp:107-113), the rest the count's"""
    return "mappability_tag" if code in (1, 2) else "count"


def _count_files(args, bins):
    """count from the FASTQ lists through the file-fed pipeline
    (smash_count_fastq: parse / H2D / compute overlapped, pairs ordered by
    name first unless --presorted)"""
    import torch
    ref = _ref(args)
    ix = load_index(ref, args.device)
    cs = S.read_chrom_sizes(args.chrom_sizes or ref + ".bin/chrom_sizes.txt")
    rows, starts = S.read_bins(bins)
    r1, r2 = args.reads1.split(), args.reads2.split()
    L = S.first_read_length(r1)
    cap = args.dedup_capacity or fastq_pairs_bound(r1, r2, L, args.batch)
    pipe = S.Pipeline(ix, cs, starts, L, args.batch, dedup_capacity=cap)
    counts = torch.zeros(len(starts), dtype=torch.int64, device=torch.device("cuda", args.device))
    pipe.reset()
    pipe.count_fastq(r1, r2, counts, sort_names=not args.presorted)
    st = pipe.stats(raise_on_error=False)
    if st.error:
        raise SystemExit("%s: %s" % (_err_label(st.error), S.ERRORS.get(st.error, st.error)))
    return rows, counts.cpu().numpy(), st


class _NoPipe:
    max_pairs = 0


def _count_files_dist(args, bins, world):
    """count over `world` ranks (one process per GPU, torch.distributed over
    RCCL: torchrun sets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*): every rank
    indexes the FASTQ lists (smashgpu.FastqIndex, strict 4-line FASTQ) and
    counts its (step, rank) batches (dist.count_fastq); counts and statistics
    are summed over the ranks; rank 0 writes the output."""
    import torch
    import torch.distributed as tdist
    from dist import ShardedCounter, count_fastq, open_fastq
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    tdist.init_process_group("nccl", device_id=dev)
    cpu = tdist.new_group(backend="gloo")
    ref = _ref(args)
    ix = load_index(ref, local)
    cs = S.read_chrom_sizes(args.chrom_sizes or ref + ".bin/chrom_sizes.txt")
    rows, starts = S.read_bins(bins)
    r1, r2 = args.reads1.split(), args.reads2.split()
    # the pipeline is made once the plan (pairs, read length) is known: a
    # placeholder counter carries the communicator for the scan exchange
    sc = ShardedCounter(_NoPipe(), rank, world, dev, count_group=cpu)
    fq = open_fastq(sc, r1, r2, sort_names=not args.presorted)
    # an owner keeps the keys it owns for the whole run: ~pairs / world to
    # start with; unless --dedup-capacity fixes it, ShardedCounter grows each
    # owner's set after the first batch's export to the run's pairs x that
    # owner's measured share (a skewed owner is sized, not overflowed), and a
    # set that still overflows stops every rank at the next batch
    cap = args.dedup_capacity or (fq.n // world + fq.n // (8 * world) + (1 << 20))
    pipe = S.Pipeline(ix, cs, starts, fq.L, args.batch, dedup_capacity=cap)
    counts = torch.zeros(len(starts), dtype=torch.int64, device=dev)
    sc = ShardedCounter(pipe, rank, world, dev, count_group=cpu,
                        plan_pairs=0 if args.dedup_capacity else fq.n)
    sc.reset()
    count_fastq(sc, fq, args.batch, counts)
    st = pipe.stats(raise_on_error=False)
    v = torch.tensor([st.positions, st.dups, st.kept, st.key_pairs, st.dupe_pairs,
                      1 if st.error else 0], dtype=torch.int64, device=dev)
    tdist.all_reduce(counts)
    tdist.all_reduce(v)
    tdist.barrier()
    tdist.destroy_process_group()
    if int(v[5]):
        raise SystemExit("count: a rank recorded a pipeline data error (%s)"
                         % S.ERRORS.get(st.error, st.error))
    pos, dups, kept, kp, dp, _ = [int(x) for x in v.tolist()]
    return rank, rows, counts.cpu().numpy(), (pos, dups, kept, kp, dp)


def cmd_count(args):
    bins = os.path.join(args.bindir, "bins.txt")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if not args.sam and args.reads1 and world > 1:
        rank, rows, counts, (pos, dups, kept, _, _) = _count_files_dist(args, bins, world)
        if rank == 0:
            write_varbin(rows, counts, pos, dups, kept, args.out or args.id + ".varbin.txt",
                         args.id + ".stats.txt")
        return
    if not args.sam and args.reads1:
        rows, counts, st = _count_files(args, bins)
        write_varbin(rows, counts, st.positions, st.dups, st.kept,
                     args.out or args.id + ".varbin.txt", args.id + ".stats.txt")
        return
    run = _Run(args, bins)
    counts, st = run.run(lambda pipe: None)
    write_varbin(run.bins_rows, counts, st.positions, st.dups, st.kept,
                 args.out or args.id + ".varbin.txt", args.id + ".stats.txt")


def cmd_varbin(args):
    import torch
    chrominfo = S.read_chrom_sizes(args.chrom_sizes)
    rows, starts = S.read_bins(args.bins)
    pos0, absp = [], []
    with open(args.positions) as f:
        for x in f:
            arow = x.rstrip().split(" ")                   # varbin.py:38-49
            chrom = arow[0]
            if chrom.find("_") > -1 or chrom == "chrM" or chrom == "" or chrom not in chrominfo:
                continue
            s = arow[1]
            p = int(s)
            if str(p) != s:
                raise SystemExit("position %r is not a canonical integer: varbin.py compares "
                                 "the strings" % s)
            pos0.append(p)
            absp.append(p + chrominfo[chrom])
    dev = torch.device("cuda", args.device)
    d_pos = torch.tensor(pos0, dtype=torch.int64, device=dev)
    d_abs = torch.tensor(absp, dtype=torch.int64, device=dev)
    d_bins = torch.from_numpy(starts).to(dev)
    counts = torch.zeros(len(starts), dtype=torch.int64, device=dev)
    total, dups, kept = S.bin_positions(d_pos, d_abs, len(pos0), -1, d_bins, len(starts), counts)
    write_varbin(rows, counts.cpu().numpy(), total, dups, kept, args.out, args.stats)


def cmd_search(args):
    """mummer's match triples per read, in --batch chunks of one read length:
    MAM / MUM emit at most L - l + 1 matches per read; MEM (-maxmatch) starts
    at --cap records per read and re-runs a chunk with the largest count when
    any read has more (smash_match_batch counts past the capacity)."""
    import torch
    ref = _ref(args)
    ix = load_index(ref, args.device)
    mode = "MUM" if args.mum else "MEM" if args.maxmatch else "MAM"
    q = args.query
    if q.endswith((".sam", ".sam.gz")):
        recs = []
        for a, s1, s2 in sam_pairs(q):
            recs += [(a + b":0", s1), (a + b":1", s2)]
    else:
        recs = [(r[0], r[2]) for r in fastq_records(q)]
    dev = torch.device("cuda", args.device)
    out = sys.stdout
    for L in sorted({len(s) for _, s in recs}):
        sel_all = [(n, s) for n, s in recs if len(s) == L and L > 0]
        for c0 in range(0, len(sel_all), args.batch):
            sel = sel_all[c0:c0 + args.batch]
            reads = S.prepare_reads(np.frombuffer(b"".join(s for _, s in sel),
                                                  np.uint8).reshape(-1, L))
            d = torch.from_numpy(np.ascontiguousarray(reads)).to(dev)
            cap = max(1, L - args.l + 1) if mode != "MEM" else args.cap
            while True:
                o = torch.zeros(len(sel) * cap * 2, dtype=torch.int64, device=dev)
                nn = torch.zeros(len(sel), dtype=torch.int32, device=dev)
                S.match_batch(ix, d, len(sel), L, o, cap, nn, mode=mode, min_len=args.l)
                k = nn.cpu().numpy()
                if int(k.max()) <= cap:
                    break
                cap = int(k.max())           # MEM: every occurrence is a record
            w = o.cpu().numpy().view(np.uint64).reshape(len(sel), 2 * cap)
            for i, (name, _) in enumerate(sel):
                ms = S.unpack_records(w[i], k[i], cap)
                out.write(name.decode() + "\t" + str(int(k[i])) + "".join(
                    "\t%d,%d,%d" % m for m in ms) + "\n")


def sam_records_in(path):
    """QueryReader::run with -samin (query.cpp:638-646): per record the name with
    the ':0'/':1' mate suffix by flag, SEQ, QUAL and the optional columns, each
    prefixed by a tab."""
    for line in _open(path):
        if line.startswith(b"@"):
            continue
        f = line.rstrip(b"\r\n").split(b"\t")
        if len(f) < 11:
            continue
        flag = int(f[1])
        name = f[0] + (b":0" if flag & 64 else b":1" if flag & 128 else b"")
        yield name, f[9], f[10], b"".join(b"\t" + x for x in f[11:])


def query_records_in(path, fastq):
    """QueryReader::run without -samin (query.cpp:648-676): '>' (or '@' with
    -fastq) records; the name runs to the first space after trimming spaces, and
    a '1' / '2' right after that space adds ':0' / ':1'; one sequence line
    (spaces dropped, NewQuery::extend); with -fastq a '+' line and one QUAL
    line, else QUAL is '!' per base (Aligner::run, query.cpp:323)."""
    mark = b"@" if fastq else b">"
    it = iter(_open(path))
    for raw in it:
        line = raw.rstrip(b"\n")
        if not line:
            continue
        if line[:1] != mark:
            raise SystemExit("missing query start character %sin input line%s"
                             % (mark.decode(), line.decode(errors="replace")))
        body = line[1:].strip(b" ")
        sp = body.find(b" ")
        name = body if sp < 0 else body[:sp]
        if 0 <= sp < len(body) - 1:
            name += {b"1": b":0", b"2": b":1"}.get(body[sp + 1:sp + 2], b"")
        seq = next(it, b"").rstrip(b"\n")
        if not seq:
            raise SystemExit("empty sequence")
        seq = seq.rstrip(b" ").replace(b" ", b"")
        qual = None
        if fastq:
            next(it, None)
            qual = next(it, b"").rstrip(b"\n")
            if not qual:
                raise SystemExit("empty errors")
        yield name, seq, qual, b""


def cmd_memsam(args):
    """`mummer -rcref -samin -samout [-nomap] ref.fa query.sam` (mummer.cpp:77-96):
    mapout SAM text (header fasta.cpp:243-252, lines query.cpp:331-415); with
    --tag the mappability_tag L/R columns are appended (mappability_tag.cpp:
    93-124) and a tag error exits 1 as the reference throws."""
    import torch
    if args.fastq and args.samin:
        raise SystemExit("-fastq cannot be used with -samin")   # mummer.cpp:143
    ref = _ref(args)
    ix = load_index(ref, args.device)
    dev = torch.device("cuda", args.device)
    sizes = ix.contig_sizes
    offsets = np.cumsum([0] + sizes[:-1]).astype(np.uint32) if args.tag else None
    small = np.array([1 if ("_gl000" in c or "chrM" in c) else 0 for c in ix.contigs], np.uint8)
    out_path = args.out or os.path.join("mapout", "mapout.1.txt")
    os.makedirs(os.path.dirname(out_path) or ".", exist_ok=True)
    with open(out_path, "wb") as out:
        out.write(b"@HD\tVN:1.0\tSO:unsorted\n")
        for name, size in zip(ix.contigs, sizes):
            out.write(b"@SQ\tSN:%s\tLN:%d\n" % (name.encode(), size))
        out.write(b"@PG\tID:longMEM\tPN:longMEM\tVN:0.5\n")
        recs = sam_records_in(args.query) if args.samin or args.query.endswith(
            (".sam", ".sam.gz")) else query_records_in(args.query, args.fastq)
        while True:
            batch = [r for _, r in zip(range(2 * args.batch), recs)]
            if not batch:
                break
            L = len(batch[0][1])
            if any(len(r[1]) != L for r in batch) or L == 0 or L > 255:
                raise SystemExit("all reads must have one length in 1..255 (device batches)")
            # NewQuery::extend lowercases only (replaceN is fastqs_to_sam's, upstream)
            reads = S._LOWER[np.frombuffer(b"".join(r[1] for r in batch),
                                           np.uint8).reshape(-1, L)]
            d = torch.from_numpy(np.ascontiguousarray(reads)).to(dev)
            text, terr = S.sam_lines(ix, d, L, [r[0] for r in batch], [r[1] for r in batch],
                                     [r[2] for r in batch], [r[3] for r in batch],
                                     nomap=args.nomap, tag_offsets=offsets, small_chr=small,
                                     min_len=args.l)
            out.write(text)
            if terr:
                raise SystemExit(S.ERRORS.get(terr, terr))


def main(argv=None):
    ap = argparse.ArgumentParser(prog="smash_cli", description=__doc__.split("\n\n")[0])
    ap.add_argument("--ref", default=None, help="reference FASTA (default $SMASH_REF)")
    ap.add_argument("--device", type=int, default=0)
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("index")
    p.add_argument("--force", action="store_true")
    p.set_defaults(fn=cmd_index)
    for name, fn in (("map", cmd_map), ("count", cmd_count)):
        p = sub.add_parser(name)
        p.add_argument("id")
        p.add_argument("reads1", nargs="?", default="", help="space-separated r1 fastq(.gz) list")
        p.add_argument("reads2", nargs="?", default="", help="space-separated r2 fastq(.gz) list")
        if name == "count":
            p.add_argument("bindir")
            p.add_argument("--out", default=None)
        p.add_argument("--sam", default=None, help="unmapped SAM input instead (mummer -samin)")
        p.add_argument("--chrom-sizes", default=None)
        p.add_argument("--batch", type=int, default=2_000_000, help="pairs per device batch")
        if name == "count":
            p.add_argument("--presorted", action="store_true",
                           help="FASTQ pairs already in samtools sort -n order: stream them")
            p.add_argument("--dedup-capacity", type=int, default=0,
                           help="distinct pair keys the de-dup set holds (0: sized from "
                                "the input files)")
        p.set_defaults(fn=fn)
    p = sub.add_parser("varbin")
    for a in ("positions", "bins", "out", "stats", "chrom_sizes"):
        p.add_argument(a)
    p.set_defaults(fn=cmd_varbin)
    p = sub.add_parser("memsam")
    p.add_argument("-nomap", action="store_true", help="print unmapped reads (query.cpp:308)")
    p.add_argument("-samin", action="store_true", help="SAM input (default for *.sam[.gz])")
    p.add_argument("-fastq", action="store_true", help="FASTQ input (else FASTA)")
    p.add_argument("-l", type=int, default=20, help="minimum match length (query.h:129)")
    p.add_argument("--tag", action="store_true", help="append mappability_tag L/R columns")
    p.add_argument("--out", default=None, help="default mapout/mapout.1.txt")
    p.add_argument("--batch", type=int, default=250_000,
                   help="pairs per device batch (device memory ~ batch x 2 x (L - l + 1) x 48 B)")
    p.add_argument("query", help="unmapped SAM (fastqs_to_sam output), FASTA or FASTQ")
    p.set_defaults(fn=cmd_memsam)
    p = sub.add_parser("search")
    p.add_argument("-mum", action="store_true")
    p.add_argument("-maxmatch", action="store_true")
    p.add_argument("-l", type=int, default=20, help="minimum match length (query.h:129)")
    p.add_argument("--cap", type=int, default=256,
                   help="-maxmatch: initial records per read (grown when exceeded)")
    p.add_argument("--batch", type=int, default=200_000, help="reads per device batch")
    p.add_argument("query")
    p.set_defaults(fn=cmd_search)
    args = ap.parse_args(argv)
    args.fn(args)


if __name__ == "__main__":
    main()
