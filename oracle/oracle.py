"""ctypes front-end of the C oracle (oracle/smash_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the product (smash-paper_amd/).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
u8p = C.POINTER(C.c_uint8)
i64p = C.POINTER(C.c_int64)


class OrcText(C.Structure):
    _fields_ = [("N", C.c_uint64), ("T", u8p), ("n_seq", C.c_uint32),
                ("startpos", u64p), ("sizes", u64p),
                ("names", C.POINTER(C.c_char_p))]


class OrcIndex(C.Structure):
    _fields_ = [("N", C.c_uint64), ("logN", C.c_uint64), ("T", u8p),
                ("SA", C.c_void_p), ("ISA", C.c_void_p), ("idx_bytes", C.c_uint32),
                ("L8", u8p), ("ovf", u64p), ("n_ovf", C.c_uint64),
                ("n_seq", C.c_uint32), ("startpos", u64p), ("sizes", u64p),
                ("pos_mask", C.c_uint64)]


class OrcCounters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "sa_loads", "isa_loads", "ref_loads", "lcp_loads",
        "sa_lines", "isa_lines", "ref_lines", "lcp_lines",
        "last_sa", "last_isa", "last_ref", "last_lcp", "ovf_lookups",
        "kt_lines", "u_lines", "last_kt", "last_u", "bm_lines", "last_bm")]

    def lines(self):
        return (self.sa_lines + self.isa_lines + self.ref_lines + self.lcp_lines
                + self.kt_lines + self.u_lines + self.bm_lines)


class OrcAccel(C.Structure):
    _fields_ = [("U", u8p), ("KT", u64p), ("K", C.c_uint32), ("BM", u64p),
                ("B", C.c_uint32), ("in_text", C.c_uint8 * 256)]


class OrcMatch(C.Structure):
    _fields_ = [("ref", C.c_uint64), ("query", C.c_uint64), ("len", C.c_uint64)]


CIGAR_MAX = 1024   # smash_oracle.h ORC_CIGAR_MAX


class OrcHit(C.Structure):
    _fields_ = [("tid", C.c_uint32), ("rc", C.c_uint32), ("pos", C.c_int64),
                ("qpos", C.c_int64), ("n_matches", C.c_uint32),
                ("n_unique", C.c_uint32), ("n_matched", C.c_uint32),
                ("hi", C.c_uint32), ("nh", C.c_uint32), ("qstart", C.c_uint32),
                ("qend", C.c_uint32), ("first_off", C.c_uint32),
                ("first_len", C.c_uint32), ("L0", C.c_int32), ("R0", C.c_int32),
                ("cigar", C.c_char * CIGAR_MAX)]


class OrcVarbinState(C.Structure):
    _fields_ = [("total", C.c_uint64), ("dups", C.c_uint64),
                ("kept", C.c_uint64), ("prev_pos", C.c_int64)]


class OrcPipeline(C.Structure):
    _fields_ = [("ix", C.POINTER(OrcIndex)), ("min_len", C.c_uint32),
                ("tag_offsets", u32p), ("small_chr", u8p), ("major", u8p),
                ("chrom_off", i64p), ("map", u8p), ("map_size", C.c_uint64),
                ("bin_starts", i64p), ("nbins", C.c_uint32)]


def build():
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.orc_text_from_fasta.argtypes = [C.c_char_p, C.POINTER(OrcText)]
        L.orc_text_free.argtypes = [C.POINTER(OrcText)]
        L.orc_build_sa.argtypes = [u8p, C.c_uint64, u64p]
        L.orc_build_isa.argtypes = [u64p, C.c_uint64, u64p]
        L.orc_build_lcp.argtypes = [u8p, C.c_uint64, u64p, u64p, u64p]
        L.orc_logN.argtypes = [C.c_uint64]
        L.orc_logN.restype = C.c_uint64
        for fn in ("orc_mam", "orc_mem", "orc_mum"):
            getattr(L, fn).argtypes = [C.POINTER(OrcIndex), u8p, C.c_uint32,
                                       C.c_uint32, C.POINTER(OrcMatch),
                                       C.c_uint32, C.POINTER(OrcCounters)]
        L.orc_mem_dev.argtypes = [C.POINTER(OrcIndex), C.POINTER(OrcAccel), u8p, C.c_uint32,
                                  C.c_uint32, C.POINTER(OrcMatch), C.c_uint32,
                                  C.POINTER(OrcCounters)]
        L.orc_mem_batch.argtypes = [C.POINTER(OrcIndex), C.POINTER(OrcAccel), u8p, C.c_uint32,
                                    C.c_uint64, C.c_uint64, C.c_uint32, C.c_int, u32p,
                                    C.POINTER(OrcCounters)]
        L.orc_mem_batch.restype = C.c_uint64
        L.orc_resolve.argtypes = [C.POINTER(OrcIndex), u8p, C.c_uint32,
                                  C.POINTER(OrcMatch), C.c_uint32,
                                  C.POINTER(OrcHit), C.c_uint32, u32p, i64p]
        L.orc_mappability.argtypes = [C.POINTER(OrcIndex), u8p]
        L.orc_mappability_range.argtypes = [C.POINTER(OrcIndex), C.c_uint64, C.c_uint64,
                                            C.c_uint32, u8p]
        L.orc_mappability_range.restype = C.c_uint64
        L.orc_tag.argtypes = [C.POINTER(OrcHit), u32p, u8p, C.c_uint64, C.c_int]
        L.orc_smash_pair.argtypes = [C.POINTER(OrcHit), C.c_uint32,
                                     C.POINTER(OrcHit), C.c_uint32, C.c_int,
                                     C.c_int64, u32p, i64p]
        L.orc_varbin.argtypes = [i64p, i64p, C.c_uint64, i64p, C.c_uint32,
                                 u64p, C.POINTER(OrcVarbinState)]
        L.orc_dedup_new.restype = C.c_void_p
        L.orc_dedup_free.argtypes = [C.c_void_p]
        L.orc_run_pairs.argtypes = [C.POINTER(OrcPipeline), u8p, C.c_uint32,
                                    C.c_uint64, C.c_uint64, C.c_int, C.c_void_p,
                                    u64p, C.POINTER(OrcVarbinState), u64p, u64p]
        L.orc_map_only.argtypes = [C.POINTER(OrcIndex), u8p, C.c_uint32,
                                   C.c_uint64, C.c_uint64, C.c_uint32, C.c_int,
                                   C.POINTER(OrcCounters)]
        L.orc_map_only.restype = C.c_uint64
        L.orc_accel_k.argtypes = [C.c_uint64]
        L.orc_accel_k.restype = C.c_uint32
        L.orc_build_accel.argtypes = [C.POINTER(OrcIndex), C.c_uint32, u8p, u64p]
        L.orc_build_ktf.argtypes = [C.POINTER(OrcIndex), C.c_uint32, u64p, u64p]
        L.orc_mam_fast.argtypes = [C.POINTER(OrcIndex), C.POINTER(OrcAccel), u8p,
                                   C.c_uint32, C.c_uint32, C.POINTER(OrcMatch),
                                   C.c_uint32, C.POINTER(OrcCounters)]
        L.orc_map_only_fast.argtypes = [C.POINTER(OrcIndex), C.POINTER(OrcAccel), u8p,
                                        C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint32,
                                        C.c_int, C.POINTER(OrcCounters)]
        L.orc_map_only_fast.restype = C.c_uint64
        L.orc_accel_b.argtypes = [C.c_uint64]
        L.orc_accel_b.restype = C.c_uint32
        L.orc_build_bitmap.argtypes = [C.POINTER(OrcIndex), C.c_uint32, u64p, u8p]
        L.orc_mam_v3.argtypes = L.orc_mam_fast.argtypes
        L.orc_map_only_v3.argtypes = L.orc_map_only_fast.argtypes
        L.orc_map_only_v3.restype = C.c_uint64
        _LIB = L
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


def text_from_fasta(path):
    """(T uint8 incl. '$', startpos u64[n_seq], sizes u64[n_seq], names)."""
    t = OrcText()
    rc = lib().orc_text_from_fasta(path.encode(), C.byref(t))
    if rc:
        raise OSError("cannot read " + path)
    T = np.ctypeslib.as_array(t.T, shape=(t.N,)).copy()
    sp = np.ctypeslib.as_array(t.startpos, shape=(t.n_seq,)).copy()
    sz = np.ctypeslib.as_array(t.sizes, shape=(t.n_seq,)).copy()
    names = [t.names[i].decode() for i in range(t.n_seq)]
    lib().orc_text_free(C.byref(t))
    return T, sp, sz, names


def text_from_contigs(contigs):
    """Same layout as text_from_fasta, from [(name, ASCII uint8)] (no file)."""
    lower = np.arange(256, dtype=np.uint8)
    lower[ord("A"):ord("Z") + 1] += 32
    comp = np.arange(256, dtype=np.uint8)
    for a, b in zip(b"acgtrymkbdhvACGTRYMKBDHV", b"tgcayrkmvhdbTGCAYRKMVHDB"):
        comp[a] = b
    parts, sp, sz, names = [], [], [], []
    pos = 0
    for k, (name, s) in enumerate(contigs):
        f = lower[s]
        sp.append(pos); sz.append(len(f)); names.append(name)
        parts.append(f); parts.append(np.array([ord("`")], np.uint8))
        pos += len(f) + 1
        sp.append(pos); sz.append(len(f)); names.append(name)
        parts.append(comp[f[::-1]])
        pos += len(f)
        if k + 1 < len(contigs):
            parts.append(np.array([ord("`")], np.uint8))
            pos += 1
    parts.append(np.array([ord("$")], np.uint8))
    T = np.concatenate(parts)
    return T, np.array(sp, np.uint64), np.array(sz, np.uint64), names


def build_index(T):
    N = len(T)
    Tp = np.zeros(N + 64, np.uint8)
    Tp[:N] = T
    SA = np.empty(N, np.uint64)
    ISA = np.empty(N, np.uint64)
    LCP = np.empty(N, np.uint64)
    L = lib()
    if L.orc_build_sa(_p(Tp, u8p), N, _p(SA, u64p)):
        raise MemoryError
    L.orc_build_isa(_p(SA, u64p), N, _p(ISA, u64p))
    L.orc_build_lcp(_p(Tp, u8p), N, _p(SA, u64p), _p(ISA, u64p), _p(LCP, u64p))
    return SA, ISA, LCP


class Index:
    """Host index wrapped for the C oracle: text, SA/ISA (u32 when N < 2^32,
    else u64, like the reference's ANINT) and the vec_uchar LCP (u8 + sorted
    {idx,val} overflow, longSA.h:18-61).  Built by the oracle's own builder
    unless arrays are given (e.g. downloaded from the device)."""

    def __init__(self, T, startpos, sizes, names, SA=None, ISA=None, LCP=None,
                 L8=None, ovf=None, padded_text=False, pos_mask=None):
        N = len(T) - (64 if padded_text else 0)
        if padded_text:
            self.T = T
        else:
            self.T = np.zeros(N + 64, np.uint8)
            self.T[:N] = T
        self.N = N
        if SA is None:
            SA, ISA, LCP = build_index(self.T[:N])
        it = np.uint32 if N <= 0xFFFFFFFF and not pos_mask else np.uint64   # (packed: u64 words)
        self.SA = np.ascontiguousarray(SA, dtype=it)
        self.ISA = np.ascontiguousarray(ISA, dtype=it)
        if L8 is None:
            LCP = np.asarray(LCP, np.uint64)
            L8 = np.minimum(LCP, 255).astype(np.uint8)
            big = np.nonzero(LCP >= 255)[0]
            ovf = np.empty((len(big), 2), np.uint64)
            ovf[:, 0] = big
            ovf[:, 1] = LCP[big]
        self.L8 = np.ascontiguousarray(L8, np.uint8)
        self.ovf = np.ascontiguousarray(np.asarray(ovf, np.uint64).reshape(-1, 2))
        self.startpos = np.ascontiguousarray(startpos, dtype=np.uint64)
        self.sizes = np.ascontiguousarray(sizes, dtype=np.uint64)
        self.names = list(names)
        self.contigs = [names[i] for i in range(0, len(names), 2)]
        self.c = OrcIndex(N, lib().orc_logN(N), _p(self.T, u8p),
                          self.SA.ctypes.data, self.ISA.ctypes.data,
                          self.SA.itemsize, _p(self.L8, u8p),
                          _p(self.ovf, u64p) if len(self.ovf) else None,
                          len(self.ovf), len(self.startpos),
                          _p(self.startpos, u64p), _p(self.sizes, u64p), pos_mask or 0)
        # SA / ISA as given may be the device's packed words: the oracle reads
        # their element bits only (pos_mask), the emulator their hints too
        self.pos_mask = pos_mask

    @property
    def LCP(self):
        """Exact LCP (u64) rebuilt from the vec_uchar layout (tests)."""
        out = self.L8.astype(np.uint64)
        if len(self.ovf):
            out[self.ovf[:, 0].astype(np.int64)] = self.ovf[:, 1]
        return out

    @classmethod
    def from_fasta(cls, path):
        T, sp, sz, names = text_from_fasta(path)
        return cls(T, sp, sz, names)

    def search(self, read: bytes, mode="MAM", min_len=20, counters=None):
        P = np.frombuffer(read, np.uint8)
        fn = {"MAM": lib().orc_mam, "MEM": lib().orc_mem, "MUM": lib().orc_mum,
              "MEM_DEV": lib().orc_mem_dev}[mode]
        cap = 512
        while True:
            out = (OrcMatch * cap)()
            extra = (C.byref(self.acc),) if mode == "MEM_DEV" else ()
            n = fn(C.byref(self.c), *extra, _p(P, u8p), len(P), min_len, out, cap,
                   C.byref(counters) if counters is not None else None)
            if n <= cap:
                break
            cap = n
        return [(out[i].ref, out[i].query, out[i].len) for i in range(n)]

    def accel(self, U=None, KT=None, K=None, BM=None, B=None, in_text=None, KTF=None):
        """Search accelerators (built here, or given, e.g. from the device).
        KT: {lo, hi} per K-mer (the oracle's own accelerated searches); KTF:
        the device layout with the (K+2)-mer presence bits (orc_build_ktf;
        tools/sm_emu runs the device kernel over it)."""
        if U is None:
            K = lib().orc_accel_k(self.N)
            U = np.zeros(self.N + 64, np.uint8)
            KT = np.zeros(2 << (2 * K), np.uint64)
            lib().orc_build_accel(C.byref(self.c), K, _p(U, u8p), _p(KT, u64p))
        if KTF is None:
            KTF = np.zeros(2 << (2 * K), np.uint64)
            lib().orc_build_ktf(C.byref(self.c), K, _p(np.ascontiguousarray(KT, np.uint64), u64p),
                                _p(KTF, u64p))
        self._KTF = np.ascontiguousarray(KTF, np.uint64)
        if BM is None:
            B = lib().orc_accel_b(self.N)
            BM = np.zeros((1 << (2 * B)) // 64 + 1, np.uint64)
            in_text = np.zeros(256, np.uint8)
            lib().orc_build_bitmap(C.byref(self.c), B, _p(BM, u64p), _p(in_text, u8p))
        self._U = np.ascontiguousarray(U, np.uint8)
        self._KT = np.ascontiguousarray(KT, np.uint64)
        self._BM = np.ascontiguousarray(BM, np.uint64)
        self.acc = OrcAccel(_p(self._U, u8p), _p(self._KT, u64p), int(K),
                            _p(self._BM, u64p), int(B),
                            (C.c_uint8 * 256)(*[int(v) for v in in_text]))
        return self._U, self._KT, int(K)

    def search_v3(self, read: bytes, min_len=20, counters=None):
        P = np.frombuffer(read, np.uint8)
        out = (OrcMatch * 512)()
        n = lib().orc_mam_v3(C.byref(self.c), C.byref(self.acc), _p(P, u8p), len(P),
                             min_len, out, 512,
                             C.byref(counters) if counters is not None else None)
        return [(out[i].ref, out[i].query, out[i].len) for i in range(min(n, 512))]

    def search_fast(self, read: bytes, min_len=20, counters=None):
        P = np.frombuffer(read, np.uint8)
        out = (OrcMatch * 512)()
        n = lib().orc_mam_fast(C.byref(self.c), C.byref(self.acc), _p(P, u8p), len(P),
                               min_len, out, 512,
                               C.byref(counters) if counters is not None else None)
        return [(out[i].ref, out[i].query, out[i].len) for i in range(min(n, 512))]

    def resolve(self, read: bytes, matches):
        P = np.frombuffer(read, np.uint8)
        m = (OrcMatch * max(1, len(matches)))()
        for i, (r, q, l) in enumerate(matches):
            m[i].ref, m[i].query, m[i].len = r, q, l
        cap = max(1, len(matches))              # hits <= matches: never truncated
        hits = (OrcHit * cap)()
        bt = C.c_uint32()
        bp = C.c_int64()
        n = lib().orc_resolve(C.byref(self.c), _p(P, u8p), len(P), m, len(matches),
                              hits, cap, C.byref(bt), C.byref(bp))
        if n < 0:
            raise RuntimeError("orc_resolve: capacity exceeded (%d matches)" % len(matches))
        best = None if bt.value == 0xFFFFFFFF else (bt.value, bp.value)
        return [hits[i] for i in range(n)], best

    def mappability(self):
        total = int(sum(self.sizes[0::2]))
        out = np.zeros(2 + 2 * total, np.uint8)
        if lib().orc_mappability(C.byref(self.c), _p(out, u8p)):
            raise MemoryError
        return out

    def mappability_range(self, g0, g1, k=36):
        """(map.bin bytes of forward bases [g0, g1), unique k-mer count)"""
        out = np.zeros(2 * (g1 - g0), np.uint8)
        n = lib().orc_mappability_range(C.byref(self.c), g0, g1, k, _p(out, u8p))
        return out, int(n)


def lower_read(seq: bytes) -> bytes:
    """NewQuery::extend (query.cpp:125-144): drop spaces, lowercase; the
    fastqs_to_sam replaceN step (fastqs_to_sam.cpp:289) turns N into Z
    first, so reads' Ns become 'z'."""
    return seq.replace(b" ", b"").replace(b"N", b"Z").lower()


def tag(hit, offsets, mapbin, small):
    off = np.ascontiguousarray(offsets, dtype=np.uint32)
    return lib().orc_tag(C.byref(hit), _p(off, u32p), _p(mapbin, u8p),
                         len(mapbin), int(small))


def smash_pair(h1, h2, min_excess=4, window=10000):
    a = (OrcHit * max(1, len(h1)))(*h1)
    b = (OrcHit * max(1, len(h2)))(*h2)
    tid = np.zeros(len(h1) + len(h2) + 1, np.uint32)   # kept <= hits: never truncated
    pos = np.zeros(len(h1) + len(h2) + 1, np.int64)
    n = lib().orc_smash_pair(a, len(h1), b, len(h2), min_excess, window,
                             _p(tid, u32p), _p(pos, i64p))
    if n < -1:
        raise RuntimeError("orc_smash_pair: capacity exceeded")
    if n < 0:
        return None
    return list(zip(tid[:n].tolist(), pos[:n].tolist()))


def varbin(pos0, abspos, bin_starts, state=None, counts=None):
    pos0 = np.ascontiguousarray(pos0, np.int64)
    abspos = np.ascontiguousarray(abspos, np.int64)
    bs = np.ascontiguousarray(bin_starts, np.int64)
    if counts is None:
        counts = np.zeros(len(bs), np.uint64)
    if state is None:
        state = OrcVarbinState(0, 0, 0, -1)
    lib().orc_varbin(_p(pos0, i64p), _p(abspos, i64p), len(pos0), _p(bs, i64p),
                     len(bs), _p(counts, u64p), C.byref(state))
    return counts, state


MAJOR_RE = None


def major_flags(names, chrom_sizes_names):
    """perl filter ^chr(\\d+|[XY]) \\d+$ (smash_mapping.sh:29) and varbin's
    chromosome filter (varbin.py:38-49)."""
    import re
    rx = re.compile(r"^chr(\d+|[XY])$")
    return np.array([1 if (rx.match(n) and "_" not in n and n != "chrM"
                           and n in chrom_sizes_names) else 0 for n in names],
                    np.uint8)


class Pipeline:
    """Whole-chain oracle: map -> resolve -> tag -> smash -> dedup -> varbin."""

    def __init__(self, ix: Index, mapbin, chrom_sizes, bin_starts, min_len=20):
        self.ix = ix
        names = ix.contigs
        sizes = [int(s) for s in ix.sizes[0::2]]
        self.tag_off = np.array(np.cumsum([0] + sizes[:-1]), dtype=np.uint32)
        self.small = np.array([1 if ("_gl000" in n or "chrM" in n) else 0
                               for n in names], np.uint8)
        self.major = major_flags(names, chrom_sizes)
        self.chrom_off = np.array([chrom_sizes.get(n, 0) for n in names], np.int64)
        self.mapbin = np.ascontiguousarray(mapbin, np.uint8)
        self.bin_starts = np.ascontiguousarray(bin_starts, np.int64)
        self.c = OrcPipeline(C.pointer(ix.c), min_len, _p(self.tag_off, u32p),
                             _p(self.small, u8p), _p(self.major, u8p),
                             _p(self.chrom_off, i64p), _p(self.mapbin, u8p),
                             len(self.mapbin), _p(self.bin_starts, i64p),
                             len(self.bin_starts))
        self.dedup = lib().orc_dedup_new()
        self.counts = np.zeros(len(self.bin_starts), np.uint64)
        self.state = OrcVarbinState(0, 0, 0, -1)
        self.n_dupe = C.c_uint64(0)
        self.n_pos = C.c_uint64(0)

    def run(self, reads: np.ndarray, threads=1):
        """reads: uint8 [2*n_pairs, L] lowercased (N->z), mates interleaved."""
        reads = np.ascontiguousarray(reads, np.uint8)
        n_pairs = reads.shape[0] // 2
        err = lib().orc_run_pairs(C.byref(self.c), _p(reads, u8p), reads.shape[1],
                                  reads.shape[1], n_pairs, threads, self.dedup,
                                  _p(self.counts, u64p), C.byref(self.state),
                                  C.byref(self.n_dupe), C.byref(self.n_pos))
        return err

    def __del__(self):
        try:
            lib().orc_dedup_free(self.dedup)
        except Exception:
            pass


def map_only(ix: Index, reads: np.ndarray, min_len=20, threads=1):
    """longSA::MAM over every read (the reference's own probe sequence), on
    `threads` host threads; returns the number of matches."""
    reads = np.ascontiguousarray(reads, np.uint8)
    return int(lib().orc_map_only(C.byref(ix.c), _p(reads, u8p), reads.shape[1],
                                  reads.shape[1], reads.shape[0], min_len, threads, None))


def mem_batch(ix: Index, reads: np.ndarray, min_len=20, threads=1, device_probes=False,
              count=False):
    """longSA::findMEM (-maxmatch) over every read on `threads` host threads:
    the reference's probe sequence, or (device_probes) smash-paper_amd/csrc/
    mem.hip's (k-mer table from the root, 8-byte singleton compares; needs
    ix.accel()) -- the same matches.  Returns (total, per-read counts,
    counters or None)."""
    reads = np.ascontiguousarray(reads, np.uint8)
    n, L = reads.shape
    ctr = OrcCounters() if count else None
    per = np.zeros(n, np.uint32)
    tot = lib().orc_mem_batch(C.byref(ix.c), C.byref(ix.acc) if device_probes else None,
                              _p(reads, u8p), L, L, n, min_len, threads, _p(per, u32p),
                              C.byref(ctr) if ctr is not None else None)
    return int(tot), per, ctr


def map_only_fast(ix: Index, reads: np.ndarray, min_len=20, threads=1, count=False):
    """Accelerated search (device algorithm) on the CPU; counters = its lines."""
    reads = np.ascontiguousarray(reads, np.uint8)
    ctr = OrcCounters() if count else None
    n = lib().orc_map_only_fast(C.byref(ix.c), C.byref(ix.acc), _p(reads, u8p),
                                reads.shape[1], reads.shape[1], reads.shape[0], min_len,
                                threads, C.byref(ctr) if ctr is not None else None)
    return n, ctr


def map_only_v3(ix: Index, reads: np.ndarray, min_len=20, threads=1, count=False):
    reads = np.ascontiguousarray(reads, np.uint8)
    ctr = OrcCounters() if count else None
    n = lib().orc_map_only_v3(C.byref(ix.c), C.byref(ix.acc), _p(reads, u8p),
                              reads.shape[1], reads.shape[1], reads.shape[0], min_len,
                              threads, C.byref(ctr) if ctr is not None else None)
    return n, ctr


def map_only(ix: Index, reads: np.ndarray, min_len=20, threads=1, count=False):
    reads = np.ascontiguousarray(reads, np.uint8)
    ctr = OrcCounters() if count else None
    n = lib().orc_map_only(C.byref(ix.c), _p(reads, u8p), reads.shape[1],
                           reads.shape[1], reads.shape[0], min_len, threads,
                           C.byref(ctr) if ctr is not None else None)
    return n, ctr
