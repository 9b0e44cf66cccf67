"""The rank-local reader of the multi-GPU driver (csrc/fastq_shard.cpp,
smashgpu.FastqShards) against the whole-input index (smashgpu.FastqIndex,
itself pinned to the streaming reader and fastqs_to_sam): W ranks as threads,
each scanning only its segments, must plan the same pairs and pack the same
bytes for any range -- over plain and gzip lane files, single- and
multi-member gzip, many segments and restart points (small
SMASH_SHARD_SEG_BYTES / SMASH_SHARD_AP_SPAN), dropped empty pairs, a
shorter mate list, and the reference reader's error cases.  CPU only."""
import gzip
import threading

import numpy as np
import pytest

from conftest import gold

import smashgpu as S


def _records(prefix, mate):
    lines = gzip.open(gold("%s_r%d.fq.gz" % (prefix, mate)), "rb").read().split(b"\n")
    return [b"\n".join(lines[i:i + 4]) + b"\n" for i in range(0, len(lines) - 3, 4)]


def _shards(paths, world, **kw):
    """W FastqShards of the same lists, built concurrently (the blob
    all-gather needs every rank)"""
    bar = threading.Barrier(world, timeout=120)
    slot = [None] * world
    out, errs = [None] * world, [None] * world

    def allgather_for(r):
        def ag(b):
            slot[r] = b
            bar.wait()
            got = list(slot)
            bar.wait()
            return got
        return ag

    def run(r):
        try:
            out[r] = S.FastqShards(*paths, rank=r, world=world, allgather=allgather_for(r),
                                   threads=3, **kw)
        except BaseException as e:   # noqa: BLE001
            errs[r] = e
    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for e in errs:
        if e is not None:
            raise e
    return out


def _pack(reader, k0, k1):
    a = np.zeros((2 * (k1 - k0), reader.L), np.uint8)
    reader.pack(k0, k1, a)
    return a


def _gz_members(data, parts):
    """`data` as `parts` concatenated gzip members (BGZF-like)"""
    cuts = [len(data) * k // parts for k in range(parts + 1)]
    return b"".join(gzip.compress(data[cuts[k]:cuts[k + 1]]) for k in range(parts))


@pytest.fixture
def lanes(tmp_path):
    """s150 as lane files per mate: plain, single-member gzip, multi-member
    gzip (record boundaries and member boundaries unrelated), plain"""
    paths = [[], []]
    for m in (1, 2):
        recs = _records("s150", m)
        cuts = [0, 300, 900, 1400, len(recs)]
        for k in range(4):
            body = b"".join(recs[cuts[k]:cuts[k + 1]])
            f = tmp_path / ("m%d_L%d.fq%s" % (m, k, ".gz" if k in (1, 2) else ""))
            if k == 1:
                f.write_bytes(gzip.compress(body, compresslevel=6))
            elif k == 2:
                f.write_bytes(_gz_members(body, 7))
            else:
                f.write_bytes(body)
            paths[m - 1].append(str(f))
    return paths


@pytest.mark.parametrize("world", [1, 2, 3, 5])
@pytest.mark.parametrize("seg,span", [(0, 0), (4096, 20000)])
def test_shards_equal_index(lanes, world, seg, span, monkeypatch):
    if seg:
        monkeypatch.setenv("SMASH_SHARD_SEG_BYTES", str(seg))
        monkeypatch.setenv("SMASH_SHARD_AP_SPAN", str(span))
    ix = S.FastqIndex(*lanes)
    ref = _pack(ix, 0, ix.n)
    sh = _shards(lanes, world)
    for r in sh:
        assert (r.n, r.L) == (ix.n, ix.L)
    rng = np.random.default_rng(world * 7 + seg)
    for r, x in enumerate(sh):
        assert np.array_equal(_pack(x, 0, x.n), ref)
        for _ in range(6):
            a = int(rng.integers(0, ix.n))
            b = int(rng.integers(a, ix.n + 1))
            assert np.array_equal(_pack(x, a, b), ref[2 * a:2 * b]), (r, a, b)
    # each rank scanned its own segments only: together every byte once
    # (plus, per plain segment, the tail of its last record past its end)
    st = [x.stats() for x in sh]
    total = sum(len(gzip.decompress(open(p, "rb").read())) if p.endswith(".gz")
                else len(open(p, "rb").read()) for p in lanes[0] + lanes[1])
    segs = sum(s["scan_segments"] for s in st)
    assert total <= sum(s["scan_bytes"] for s in st) <= total + segs * 400
    assert all(s["scan_bytes"] < total for s in st) or world == 1


def test_shards_pack_reads_only_its_share(tmp_path, monkeypatch):
    """W = 4 ranks each packing their (step, rank) batches parse about 1/W
    of the FASTQ bytes in the packs (plus a segment or restart span per
    cursor), not the whole input."""
    monkeypatch.setenv("SMASH_SHARD_SEG_BYTES", str(1 << 16))
    monkeypatch.setenv("SMASH_SHARD_AP_SPAN", str(1 << 16))
    recs = [_records("s150", 1), _records("s150", 2)]
    paths = [[], []]
    W, B = 4, 250
    for m in (0, 1):
        # 4 renamed copies (8 000 pairs, names in sort -n order); mate 2 gzip
        out = []
        for c in range(4):
            for k, r in enumerate(recs[m]):
                out.append(b"@c%d_%06d\n" % (c, k) + r.split(b"\n", 1)[1])
        body = b"".join(out)
        f = tmp_path / ("m%d.fq%s" % (m, ".gz" if m else ""))
        f.write_bytes(gzip.compress(body) if m else body)
        paths[m].append(str(f))
    sh = _shards(paths, W)
    n = sh[0].n
    total = sum(len(gzip.decompress(open(p, "rb").read())) if p.endswith(".gz")
                else len(open(p, "rb").read()) for p in paths[0] + paths[1])
    ix = S.FastqIndex(*paths)
    ref = _pack(ix, 0, ix.n)
    for r, x in enumerate(sh):
        steps = (n + W * B - 1) // (W * B)
        for s in range(steps):
            lo = min(n, s * W * B + r * B)
            hi = min(n, lo + B)
            if hi > lo:
                assert np.array_equal(_pack(x, lo, hi), ref[2 * lo:2 * hi])
        st = x.stats()
        assert st["pack_pairs"] <= n // W + B
        # its pairs' bytes plus the skips before each pack's cursors
        assert st["pack_bytes"] < total / W * 1.6 + steps * 2 * (1 << 16) * 2, (st, total)


def _write(tmp_path, name, recs):
    f = tmp_path / name
    f.write_bytes(b"".join(recs))
    return str(f)


def test_shards_drop_empty_pairs_and_zip(tmp_path):
    """pairs whose two mates are empty are dropped (fastqs_to_sam.cpp:80);
    the shorter list ends the pairs; a pair with one empty mate is an error"""
    r = lambda n, s: b"@%s\n%s\n+\n%s\n" % (n, s, b"I" * len(s))
    a = [r(b"p%03d" % i, b"ACGT" if i not in (3, 7) else b"") for i in range(12)]
    b = [r(b"p%03d" % i, b"TTGA" if i not in (3, 7) else b"") for i in range(10)]
    p = [[_write(tmp_path, "a.fq", a)], [_write(tmp_path, "b.fq", b)]]
    ix = S.FastqIndex(*p)
    for W in (1, 2):
        sh = _shards(p, W)
        assert sh[0].n == ix.n == 8
        assert np.array_equal(_pack(sh[-1], 0, 8), _pack(ix, 0, 8))
    b[5] = r(b"p005", b"")
    p2 = [[p[0][0]], [_write(tmp_path, "b2.fq", b)]]
    sh = _shards(p2, 2)
    with pytest.raises(S.SmashError, match="no bases"):
        _pack(sh[0], 0, sh[0].n)


def test_shards_order_and_strictness(tmp_path):
    r = lambda n, s: b"@%s\n%s\n+\n%s\n" % (n, s, b"I" * len(s))
    a = [r(b"q%d" % i, b"ACGT") for i in (1, 2, 10, 3)]
    b = [r(b"q%d" % i, b"ACGT") for i in (1, 2, 10, 3)]
    p = [[_write(tmp_path, "a.fq", a)], [_write(tmp_path, "b.fq", b)]]
    with pytest.raises(S.SmashError, match="sort -n order at read q3"):
        _shards(p, 2)
    with pytest.raises(S.SmashError) as e:
        _shards(p, 2, sort_names=True)
    assert e.value.code == S.SMASH_ERR_UNSUPPORTED
    bad = [[_write(tmp_path, "c.fq", [b">x\nACGT\n"])], [p[1][0]]]
    with pytest.raises(S.SmashError) as e:
        _shards(bad, 2)
    assert e.value.code == S.SMASH_ERR_UNSUPPORTED
    nonl = tmp_path / "d.fq"
    nonl.write_bytes(b"@x\nACGT\n+\nIIII")
    with pytest.raises(S.SmashError) as e:
        _shards([[str(nonl)], [p[1][0]]], 1)
    assert e.value.code == S.SMASH_ERR_UNSUPPORTED


def test_shards_blob_mismatch_is_refused(lanes):
    """a rank whose files differ (here: a scan of other files) is refused"""
    other = [lanes[0][:2], lanes[1][:2]]
    import ctypes as C
    L = S.lib()
    blobs = []
    for r, ps in enumerate((lanes, other)):
        a1 = S._cstrs([p.encode() for p in ps[0]])
        a2 = S._cstrs([p.encode() for p in ps[1]])
        blob, nb = S.vp(), C.c_uint64()
        assert L.smash_fastq_shard_scan(a1, len(ps[0]), a2, len(ps[1]), 2, r, 2, C.byref(blob),
                                        C.byref(nb)) == 0
        blobs.append(C.string_at(blob.value, nb.value))
        L.smash_fastq_shard_free_blob(blob)
    it = iter([blobs])
    with pytest.raises(S.SmashError, match="not a scan of these files"):
        S.FastqShards(*lanes, rank=0, world=2, allgather=lambda b: next(it))


_RSS_SCRIPT = r"""
import gzip, os, resource, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import smashgpu as S
paths = [[sys.argv[2]], [sys.argv[3]]]
S.lib()
base = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
x = S.FastqShards(*paths, rank=0, world=1, allgather=lambda b: [b], threads=4)
out = np.zeros((2 * 20000, x.L), np.uint8)
for k0 in range(0, x.n, 20000):
    k1 = min(x.n, k0 + 20000)
    x.pack(k0, k1, out)
print(x.n, (resource.getrusage(resource.RUSAGE_SELF).ru_maxrss - base) * 1024)
"""


def test_shards_host_memory_is_bounded(tmp_path):
    """A rank's host memory does not grow with the input: ~400 MB of FASTQ
    text (gzip, one file per mate) scanned and packed in batches of 20 000
    pairs raises the process's peak RSS by far less than the text (the
    readers keep bounded buffers: restart windows, 8 MB cursors, 4 MB input
    chunks; no whole file)."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    recs = [_records("s150", 1), _records("s150", 2)]
    paths = []
    for m in (0, 1):
        f = tmp_path / ("m%d.fq.gz" % m)
        with gzip.open(f, "wb", compresslevel=1) as g:
            for c in range(1000):
                g.write(b"".join(b"@c%04d_%06d\n" % (c, k) + r.split(b"\n", 1)[1]
                                 for k, r in enumerate(recs[m])))
        paths.append(str(f))
    text = 2 * 1000 * sum(len(r) for r in recs[0])
    res = subprocess.run([sys.executable, "-c", _RSS_SCRIPT,
                          os.path.join(ROOT, "smash-paper_amd"), *paths],
                         capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr
    n, grew = (int(v) for v in res.stdout.split())
    assert n == 1000 * len(recs[0])
    assert grew < 96 << 20 and grew < text / 3, (grew, text)
