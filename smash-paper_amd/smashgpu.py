"""smashgpu -- Python host side of the MI355X SMASH read -> bin-count path.

Mirrors the reference's driver layer (index_setup.sh / smash_mapping.sh /
binning.sh glue around mummer, mappability_tag, smashMEM.py and varbin.py)
over the C ABI of libsmashgpu.so (include/smash_gpu.h).  PyTorch is used only
for device memory, streams and torch.distributed; every computation runs in
the HIP kernels of smash-paper_amd/csrc.  There is no CPU fallback: if the
library is missing this module raises on import of the library.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libsmashgpu.so")
# A/B measurement of library builds (tools/ab.sh): SMASH_LIB names another build
LIB_PATH = os.environ.get("SMASH_LIB", LIB_PATH)

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
u8p = C.POINTER(C.c_uint8)
i64p = C.POINTER(C.c_int64)
i32p = C.POINTER(C.c_int32)
vp = C.c_void_p

SMASH_MODE_MAM = 1
SMASH_MODE_MAM_PLAIN = 2
SMASH_MODE_MUM = 3
SMASH_MODE_MEM = 4
MODES = {"MAM": SMASH_MODE_MAM, "MUM": SMASH_MODE_MUM, "MEM": SMASH_MODE_MEM}
SAM_PACKED = 0x80000000   # smash_sam_format: records packed read after read (| cap)

ERRORS = {1: "left mappability too big (mappability_tag.cpp:110)",
          2: "right mappability too big (mappability_tag.cpp:113)",
          -4: "out of device memory / key set full",
          -5: "unsupported (more matches per read than on-chip slots)"}

EXPORTS = [
    "smash_last_error", "smash_text_from_fasta", "smash_text_free",
    "smash_index_create", "smash_index_load", "smash_index_save",
    "smash_index_free", "smash_index_query", "smash_map_batch", "smash_match_batch",
    "smash_pipeline_create", "smash_pipeline_free", "smash_count_batch",
    "smash_phase_map", "smash_phase_export", "smash_dedup_owner",
    "smash_phase_import", "smash_phase_positions", "smash_phase_bin",
    "smash_pipeline_stats", "smash_pipeline_reset", "smash_pipeline_reset_ex", "smash_pipeline_reads_resident", "smash_pipeline_peek",
    "smash_pipeline_profile", "smash_pipeline_profile_read",
    "smash_pipeline_positions", "smash_bin_positions", "smash_mappability_scan",
    "smash_sam_records", "smash_sam_format", "smash_sam_free",
    "smash_fastq_open", "smash_fastq_read", "smash_fastq_close", "smash_strnum_order",
    "smash_count_fastq", "smash_count_batches", "smash_count_batches_ready",
    "smash_pipeline_profile_active",
    "smash_pipeline_profile_intervals", "smash_fastq_read_parallel",
    "smash_fastq_index_open", "smash_fastq_index_pack", "smash_fastq_index_close",
    "smash_phase_map_ahead", "smash_sam_records_packed",
    "smash_text_from_fasta_layout", "smash_index_create_layout", "smash_index_load_layout",
    "smash_phase_search_ahead",
    "smash_fastq_shard_scan", "smash_fastq_shard_free_blob", "smash_fastq_shard_open",
    "smash_fastq_shard_pack", "smash_fastq_shard_stats", "smash_fastq_shard_close",
    "smash_read_stride", "smash_pipeline_max_batch",
    "smash_mappability_prepare", "smash_mappability_window", "smash_index_pack",
    "smash_pipeline_reserve_keys", "smash_pipeline_key_capacity", "smash_pipeline_error",
    "smash_mappability_release", "smash_pipeline_map_hints",
]


class IndexInfo(C.Structure):
    _fields_ = [("N", C.c_uint64), ("logN", C.c_uint64), ("idx_bytes", C.c_uint32),
                ("n_seq", C.c_uint32), ("n_lcp_overflow", C.c_uint64),
                ("map_bytes", C.c_uint64), ("d_text", vp), ("d_sa", vp),
                ("d_isa", vp), ("d_lcp8", vp), ("d_lcp_ovf", vp), ("d_map", vp),
                ("device_bytes", C.c_uint64), ("build_seconds", C.c_double),
                ("kmer_k", C.c_uint32), ("d_uniq", vp), ("d_kmer", vp),
                ("bitmap_b", C.c_uint32), ("d_bitmap", vp), ("in_text", C.c_uint64 * 4),
                ("rcref", C.c_uint32), ("pos_bits", C.c_uint32)]


class PipelineCfg(C.Structure):
    _fields_ = [("min_len", C.c_uint32), ("read_len", C.c_uint32),
                ("max_pairs", C.c_uint64), ("n_contig", C.c_uint32),
                ("h_tag_offsets", u32p), ("h_small_chr", u8p),
                ("h_chrom_off", i64p), ("nbins", C.c_uint32),
                ("h_bin_starts", i64p), ("min_excess", C.c_int32),
                ("hit_window", C.c_int64), ("dedup_capacity", C.c_uint64),
                ("read_stride", C.c_uint32)]


class FeedStats(C.Structure):
    _fields_ = [("pairs", C.c_uint64), ("batches", C.c_uint64), ("wall_s", C.c_double),
                ("ingest_s", C.c_double), ("wait_s", C.c_double), ("read_len", C.c_uint32),
                ("parallel", C.c_uint32), ("index_s", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class ShardStats(C.Structure):
    _fields_ = [("input_bytes", C.c_uint64), ("scan_segments", C.c_uint64),
                ("scan_bytes", C.c_uint64), ("scan_bytes_in", C.c_uint64), ("scan_s", C.c_double),
                ("pack_pairs", C.c_uint64), ("pack_bytes", C.c_uint64),
                ("pack_bytes_in", C.c_uint64), ("pack_s", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Stats(C.Structure):
    _fields_ = [("pairs", C.c_uint64), ("key_pairs", C.c_uint64),
                ("dupe_pairs", C.c_uint64), ("positions", C.c_uint64),
                ("dups", C.c_uint64), ("kept", C.c_uint64),
                ("matches", C.c_uint64), ("error", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class SmashError(RuntimeError):
    pass


_LIB = None


def lib():
    """Load libsmashgpu.so (raises if it was not built: no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise SmashError("libsmashgpu.so not built (run `make -C smash-paper_amd` "
                         "or __graft_entry__.build()); there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    L.smash_last_error.restype = C.c_char_p
    L.smash_text_from_fasta.argtypes = [C.c_char_p, C.POINTER(u8p), u64p, u32p,
                                        C.POINTER(u64p), C.POINTER(u64p),
                                        C.POINTER(C.POINTER(C.c_char_p))]
    L.smash_text_from_fasta_layout.argtypes = [C.c_char_p, C.c_int, C.POINTER(u8p), u64p, u32p,
                                               C.POINTER(u64p), C.POINTER(u64p),
                                               C.POINTER(C.POINTER(C.c_char_p))]
    L.smash_text_free.argtypes = [u8p, C.c_uint32, u64p, u64p, C.POINTER(C.c_char_p)]
    L.smash_text_free.restype = None
    L.smash_index_create.argtypes = [u8p, C.c_uint64, C.c_uint32, u64p, u64p,
                                     C.POINTER(C.c_char_p), C.c_int, C.POINTER(vp)]
    L.smash_index_create_layout.argtypes = [u8p, C.c_uint64, C.c_uint32, u64p, u64p,
                                            C.POINTER(C.c_char_p), C.c_int, C.c_int,
                                            C.POINTER(vp)]
    L.smash_index_load.argtypes = [C.c_char_p, C.c_int, C.POINTER(vp)]
    L.smash_index_load_layout.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(vp)]
    L.smash_index_save.argtypes = [vp, C.c_char_p, C.c_uint64]
    L.smash_index_free.argtypes = [vp]
    L.smash_index_free.restype = None
    L.smash_index_query.argtypes = [vp, C.POINTER(IndexInfo)]
    L.smash_map_batch.argtypes = [vp, C.c_int, C.c_uint32, vp, C.c_uint64, vp,
                                  C.c_uint32, C.c_uint64, vp, C.c_uint32, vp, vp]
    L.smash_match_batch.argtypes = [vp, C.c_int, C.c_uint32, vp, C.c_uint64, vp,
                                    C.c_uint32, C.c_uint64, vp, C.c_uint32, vp, vp]
    L.smash_pipeline_create.argtypes = [vp, C.POINTER(PipelineCfg), C.POINTER(vp)]
    L.smash_pipeline_free.argtypes = [vp]
    L.smash_pipeline_free.restype = None
    L.smash_count_batch.argtypes = [vp, vp, C.c_uint64, vp, vp]
    L.smash_count_batches.argtypes = [vp, vp, C.c_uint64, C.c_uint64, vp, vp]
    L.smash_count_batches_ready.argtypes = [vp, vp, C.c_uint64, C.c_uint64, vp, vp, vp]
    L.smash_phase_map_ahead.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, vp]
    L.smash_phase_search_ahead.argtypes = [vp, vp, C.c_uint64, vp]
    L.smash_pipeline_profile_active.argtypes = [vp, C.POINTER(C.c_double)]
    L.smash_pipeline_profile_intervals.argtypes = [vp, C.POINTER(C.c_double), C.c_uint64, u64p]
    L.smash_phase_map.argtypes = [vp, vp, C.c_uint64, vp]
    L.smash_phase_export.argtypes = [vp, C.c_int, C.c_uint64, i64p, i64p, C.POINTER(vp),
                                     C.POINTER(vp), vp]
    L.smash_dedup_owner.argtypes = [vp, vp, C.c_uint64, vp, i64p, i64p, C.c_int, vp, vp]
    L.smash_phase_import.argtypes = [vp, vp, vp]
    L.smash_phase_positions.argtypes = [vp, vp, vp]
    L.smash_phase_bin.argtypes = [vp, vp, vp, vp]
    L.smash_pipeline_stats.argtypes = [vp, C.POINTER(Stats)]
    L.smash_pipeline_reset.argtypes = [vp, vp]
    L.smash_pipeline_reset_ex.argtypes = [vp, C.c_uint32, vp]
    L.smash_pipeline_reads_resident.argtypes = [vp, C.c_int]
    L.smash_pipeline_peek.argtypes = [vp, i32p, u8p, u64p, u64p]
    L.smash_pipeline_profile.argtypes = [vp, C.c_int]
    L.smash_pipeline_profile_read.argtypes = [vp, C.POINTER(C.c_double), u64p, u64p]
    L.smash_pipeline_positions.argtypes = [vp, i64p, i64p, C.c_uint64, u64p]
    L.smash_bin_positions.argtypes = [vp, vp, C.c_uint64, C.c_int64, vp, C.c_uint32, vp, u64p,
                                      vp]
    L.smash_mappability_scan.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_uint32, vp, i64p, vp,
                                         C.c_uint32, vp, vp, vp]
    L.smash_sam_records.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint32, C.c_uint64, vp,
                                    C.c_uint32, vp, vp, vp, vp]
    L.smash_sam_records_packed.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint32, C.c_uint64, vp,
                                           C.c_uint32, vp, vp, vp, vp, vp]
    L.smash_sam_format.argtypes = [C.POINTER(C.c_char_p), C.c_uint32, vp, u32p, C.c_uint32, C.c_uint64,
                                   C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                   C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.c_int, C.c_int,
                                   u8p, C.POINTER(C.c_void_p), u64p, i32p]
    L.smash_sam_free.argtypes = [C.c_void_p]
    L.smash_sam_free.restype = None
    L.smash_fastq_open.argtypes = [C.POINTER(C.c_char_p), C.c_uint32, C.POINTER(C.c_char_p),
                                   C.c_uint32, C.POINTER(vp)]
    L.smash_fastq_read.argtypes = [vp, C.c_uint64, u32p, vp, vp, C.c_uint32, u64p]
    L.smash_fastq_close.argtypes = [vp]
    L.smash_fastq_close.restype = None
    L.smash_strnum_order.argtypes = [vp, C.c_uint32, C.c_uint64, u64p]
    L.smash_fastq_index_open.argtypes = [C.POINTER(C.c_char_p), C.c_uint32,
                                         C.POINTER(C.c_char_p), C.c_uint32, C.c_uint32, u32p,
                                         C.c_int, C.POINTER(vp), u64p]
    L.smash_fastq_index_pack.argtypes = [vp, C.c_uint64, C.c_uint64, vp, vp, C.c_uint32]
    L.smash_fastq_index_close.argtypes = [vp]
    L.smash_fastq_index_close.restype = None
    L.smash_fastq_read_parallel.argtypes = [C.POINTER(C.c_char_p), C.c_uint32,
                                            C.POINTER(C.c_char_p), C.c_uint32, C.c_uint32,
                                            u32p, C.c_uint64, vp, vp, C.c_uint32, u64p]
    L.smash_fastq_shard_scan.argtypes = [C.POINTER(C.c_char_p), C.c_uint32,
                                         C.POINTER(C.c_char_p), C.c_uint32, C.c_uint32,
                                         C.c_uint32, C.c_uint32, C.POINTER(vp), u64p]
    L.smash_fastq_shard_free_blob.argtypes = [vp]
    L.smash_fastq_shard_free_blob.restype = None
    L.smash_fastq_shard_open.argtypes = [C.POINTER(C.c_char_p), C.c_uint32,
                                         C.POINTER(C.c_char_p), C.c_uint32, C.c_uint32,
                                         C.c_uint32, C.POINTER(vp), u64p, C.c_uint32, u32p,
                                         C.c_int, C.POINTER(vp), u64p]
    L.smash_fastq_shard_pack.argtypes = [vp, C.c_uint64, C.c_uint64, vp]
    L.smash_fastq_shard_stats.argtypes = [vp, C.POINTER(ShardStats)]
    L.smash_fastq_shard_close.argtypes = [vp]
    L.smash_fastq_shard_close.restype = None
    L.smash_read_stride.argtypes = [C.c_uint32]
    L.smash_read_stride.restype = C.c_uint32
    L.smash_mappability_prepare.argtypes = [vp, C.c_uint64, C.c_uint64, vp]
    L.smash_index_pack.argtypes = [vp, C.c_int, vp]
    L.smash_mappability_release.argtypes = [vp]
    L.smash_pipeline_reserve_keys.argtypes = [vp, C.c_uint64, vp]
    L.smash_pipeline_key_capacity.argtypes = [vp]
    L.smash_pipeline_key_capacity.restype = C.c_uint64
    L.smash_pipeline_map_hints.argtypes = [vp]
    L.smash_pipeline_map_hints.restype = C.c_int
    L.smash_pipeline_error.argtypes = [vp, vp, C.POINTER(C.c_int32)]
    L.smash_mappability_window.argtypes = [vp, C.c_uint64, C.c_uint64, u64p, u64p]
    L.smash_pipeline_max_batch.argtypes = [C.c_uint32, C.c_uint32]
    L.smash_pipeline_max_batch.restype = C.c_uint64
    L.smash_count_fastq.argtypes = [vp, C.POINTER(C.c_char_p), C.c_uint32,
                                    C.POINTER(C.c_char_p), C.c_uint32, C.c_int, C.c_uint32, vp,
                                    C.POINTER(FeedStats), vp]
    _LIB = L
    return L


def check(rc, what=""):
    if rc != 0:
        msg = lib().smash_last_error().decode(errors="replace")
        raise SmashError("%s failed (%d): %s" % (what, rc, msg))


def _p(a, t):
    return a.ctypes.data_as(t)


def _stream(stream):
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return int(stream)


# ---------------------------------------------------------------------------
# reference text
# ---------------------------------------------------------------------------
_LOWER = np.arange(256, dtype=np.uint8)
_LOWER[ord("A"):ord("Z") + 1] += 32
_COMP = np.arange(256, dtype=np.uint8)
for _a, _b in zip(b"acgtrymkbdhvACGTRYMKBDHV", b"tgcayrkmvhdbTGCAYRKMVHDB"):
    _COMP[_a] = _b


def text_from_fasta(path, rcref=True):
    """Sequence::Sequence (fasta.cpp:133-285), in the library: with -rcref
    (default) or the forward-only layout of `mummer` without it."""
    L = lib()
    t = u8p()
    N = C.c_uint64()
    ns = C.c_uint32()
    sp = u64p()
    sz = u64p()
    nm = C.POINTER(C.c_char_p)()
    check(L.smash_text_from_fasta_layout(path.encode(), 1 if rcref else 0, C.byref(t),
                                         C.byref(N), C.byref(ns), C.byref(sp), C.byref(sz),
                                         C.byref(nm)),
          "smash_text_from_fasta")
    T = np.ctypeslib.as_array(t, shape=(N.value,)).copy()
    startpos = np.ctypeslib.as_array(sp, shape=(ns.value,)).copy()
    sizes = np.ctypeslib.as_array(sz, shape=(ns.value,)).copy()
    names = [nm[i].decode() for i in range(ns.value)]
    L.smash_text_free(t, ns, sp, sz, nm)
    return T, startpos, sizes, names


def text_from_contigs(contigs):
    """The same text layout from in-memory contigs [(name, ASCII uint8)]."""
    parts, sp, sz, names = [], [], [], []
    pos = 0
    for k, (name, s) in enumerate(contigs):
        f = _LOWER[s]
        sp.append(pos); sz.append(len(f)); names.append(name)
        parts.append(f)
        parts.append(np.array([ord("`")], np.uint8))
        pos += len(f) + 1
        sp.append(pos); sz.append(len(f)); names.append(name)
        parts.append(_COMP[f[::-1]])
        pos += len(f)
        if k + 1 < len(contigs):
            parts.append(np.array([ord("`")], np.uint8))
            pos += 1
    parts.append(np.array([ord("$")], np.uint8))
    return (np.concatenate(parts), np.array(sp, np.uint64), np.array(sz, np.uint64),
            names)


def prepare_reads(seqs) -> np.ndarray:
    """fastqs_to_sam replaceN (N->Z, fastqs_to_sam.cpp:289) + NewQuery::extend
    lowercasing (query.cpp:125-144).  seqs: uint8 [n, L] ASCII."""
    a = np.asarray(seqs, np.uint8).copy()
    a[a == ord("N")] = ord("Z")
    return _LOWER[a]


# ---------------------------------------------------------------------------
# index
# ---------------------------------------------------------------------------
class Index:
    """HBM-resident SA/ISA/LCP/text/map.bin (replaces longSA, longSA.cpp:94)."""

    def __init__(self, handle, names, sizes):
        self.h = vp(handle)
        self.info = IndexInfo()
        check(lib().smash_index_query(self.h, C.byref(self.info)), "smash_index_query")
        self.rcref = bool(self.info.rcref)
        self.names = list(names)
        self.sizes = [int(x) for x in sizes]
        step = 2 if self.rcref else 1
        self.contigs = [self.names[i] for i in range(0, len(self.names), step)]
        self.contig_sizes = self.sizes[0::step]

    @classmethod
    def create(cls, T, startpos, sizes, names, device=0, rcref=True):
        T = np.ascontiguousarray(T, np.uint8)
        sp = np.ascontiguousarray(startpos, np.uint64)
        sz = np.ascontiguousarray(sizes, np.uint64)
        arr = (C.c_char_p * len(names))(*[n.encode() for n in names])
        h = vp()
        check(lib().smash_index_create_layout(_p(T, u8p), len(T), len(sp), _p(sp, u64p),
                                              _p(sz, u64p), arr, 1 if rcref else 0, device,
                                              C.byref(h)),
              "smash_index_create")
        return cls(h.value, names, sz)

    @classmethod
    def from_fasta(cls, path, device=0, rcref=True):
        return cls.create(*text_from_fasta(path, rcref), device=device, rcref=rcref)

    @classmethod
    def from_contigs(cls, contigs, device=0):
        return cls.create(*text_from_contigs(contigs), device=device)

    @classmethod
    def load(cls, fasta_path, device=0, rcref=True):
        """Load the reference's <fasta>.bin/ cache (longSA.cpp:100-136)."""
        h = vp()
        check(lib().smash_index_load_layout(fasta_path.encode(), 1 if rcref else 0, device,
                                            C.byref(h)),
              "smash_index_load")
        names, sizes = [], []
        with open(fasta_path + ".bin/rc%d.ref.bin" % (1 if rcref else 0), "rb") as f:
            b = f.read()
        n = int.from_bytes(b[16:24], "little")
        off = 24
        for _ in range(n):
            sizes.append(int.from_bytes(b[off + 8:off + 16], "little"))
            L = int.from_bytes(b[off + 16:off + 24], "little")
            names.append(b[off + 24:off + 24 + L].decode())
            off += 24 + L
        return cls(h.value, names, sizes)

    def save(self, fasta_path, fasta_size=None):
        if fasta_size is None:
            fasta_size = os.path.getsize(fasta_path)
        check(lib().smash_index_save(self.h, fasta_path.encode(), fasta_size),
              "smash_index_save")

    @property
    def N(self):
        return self.info.N

    @property
    def pos_mask(self):
        """the element bits of an SA / ISA word (packed index words keep the
        search's hints above them, smash_index_info.pos_bits)"""
        b = self.info.pos_bits
        return (1 << b) - 1 if b else (1 << (8 * self.info.idx_bytes)) - 1

    def pack(self, on=True):
        """smash_index_pack: put the search's hints into the SA / ISA words
        (on) or strip them (results are the same either way)"""
        check(lib().smash_index_pack(self.h, 1 if on else 0, None), "smash_index_pack")
        check(lib().smash_index_query(self.h, C.byref(self.info)), "smash_index_query")

    def download_sa_isa(self, plain=True):
        """host copies of SA and ISA (u32 / u64 as in HBM); plain: the
        elements alone (the packed hints masked off)"""
        i = self.info
        dt = np.uint32 if i.idx_bytes == 4 else np.uint64
        SA = download(i.d_sa, i.N * i.idx_bytes, dt)
        ISA = download(i.d_isa, i.N * i.idx_bytes, dt)
        if plain and i.pos_bits:
            m = dt(self.pos_mask)
            np.bitwise_and(SA, m, out=SA)
            np.bitwise_and(ISA, m, out=ISA)
        return SA, ISA

    def __del__(self):
        try:
            if self.h:
                lib().smash_index_free(self.h)
                self.h = None
        except Exception:
            pass


# ---------------------------------------------------------------------------
# read -> bin-count pipeline
# ---------------------------------------------------------------------------
MAJOR = re.compile(r"^chr(\d+|[XY])$")


def contig_tables(contigs, sizes, chrom_sizes):
    """Host-side per-contig tables of the reference glue:
    tag offsets = cumulative sam_header.txt lengths (chromosomes.h:169-196,
    index_setup.sh:31); small = '_gl000'/'chrM' (mappability_tag.cpp:82);
    chrom_off = chrom_sizes.txt offset when the perl filter
    ^chr(\\d+|[XY]) \\d+$ (smash_mapping.sh:29) and varbin's filters
    (varbin.py:38-49) keep the contig, else -1."""
    tag = np.cumsum([0] + [int(s) for s in sizes[:-1]]).astype(np.uint32)
    small = np.array([1 if ("_gl000" in c or "chrM" in c) else 0 for c in contigs], np.uint8)
    off = np.array([chrom_sizes[c] if (MAJOR.match(c) and "_" not in c and c != "chrM"
                                       and c in chrom_sizes) else -1 for c in contigs],
                   np.int64)
    return tag, small, off


def read_chrom_sizes(path):
    out = {}
    for line in open(path):
        c = line.rstrip("\n").split("\t")
        if c[0] in out:
            continue    # fileToDictionary keeps the first (varbin.py:131-146)
        out[c[0]] = int(c[2])
    return out


def read_bins(path):
    rows = [line.rstrip("\n").split("\t") for line in open(path)]
    return rows, np.array([int(r[2]) for r in rows], np.int64)


def read_stride(read_len):
    """bytes of the device's native row for a mate of read_len bases
    (smash_read_stride): batches laid out in such rows (16-byte aligned, zero
    padded) are searched without a record build"""
    return int(lib().smash_read_stride(read_len))


def pipeline_max_batch(read_len, min_len=20):
    """The largest batch (pairs) a Pipeline of read_len-base mates accepts:
    max_pairs * 2 * (read_len - min_len + 1) < 2^32 (include/smash_gpu.h)."""
    return int(lib().smash_pipeline_max_batch(read_len, min_len))


def to_rows(d_reads, read_len=None):
    """a [2n, L] uint8 device tensor of mates as the native rows [2n, stride]
    (zero padded)"""
    import torch
    L = read_len or d_reads.shape[1]
    rows = torch.zeros((d_reads.shape[0], read_stride(L)), dtype=torch.uint8, device=d_reads.device)
    rows[:, :L] = d_reads[:, :L]
    return rows


class Pipeline:
    """prepare_matches + mappability_tag + smashMEM + varbin on the device.
    read_stride: the bytes from one mate to the next in the batches (0:
    read_len, dense; read_stride(read_len): native rows, see to_rows)."""

    # u64 words per key in phase_export's headers (SMASH_EXPORT_HDR_WORDS)
    hdr_words = 1

    def __init__(self, index: Index, chrom_sizes: dict, bin_starts, read_len,
                 max_pairs, min_len=20, min_excess=4, hit_window=10000,
                 dedup_capacity=None, read_stride=0):
        self.index = index
        sizes = index.contig_sizes
        self.tag, self.small, self.off = contig_tables(index.contigs, sizes, chrom_sizes)
        self.bins = np.ascontiguousarray(bin_starts, np.int64)
        self.cfg = PipelineCfg(min_len, read_len, max_pairs, len(index.contigs),
                               _p(self.tag, u32p), _p(self.small, u8p),
                               _p(self.off, i64p), len(self.bins), _p(self.bins, i64p),
                               min_excess, hit_window,
                               dedup_capacity or max_pairs, read_stride)
        h = vp()
        check(lib().smash_pipeline_create(index.h, C.byref(self.cfg), C.byref(h)),
              "smash_pipeline_create")
        self.h = h
        self.read_len = read_len
        self.stride = read_stride or read_len
        self.max_pairs = max_pairs
        self.slots = read_len - min_len + 1

    def count_batch(self, d_reads, n_pairs, d_counts, stream=None):
        """d_reads: device uint8 [2*n_pairs, read_len] (torch tensor or ptr)."""
        check(lib().smash_count_batch(self.h, _reads(d_reads, n_pairs, self.stride), n_pairs,
                                      _ptr(d_counts),
                                      vp(_stream(stream))), "smash_count_batch")

    def count_fastq(self, r1_paths, r2_paths, d_counts, sort_names=True, threads=0,
                    stream=None):
        """File-fed counting (smash_count_fastq): the two mate lists parsed,
        batched in pinned memory, copied and counted with overlap.
        sort_names=False: the input is in samtools sort -n order already.
        Returns the feed statistics (pairs, batches, wall_s, ingest_s, wait_s)."""
        arr1 = _cstrs([os.fsencode(x) for x in r1_paths])
        arr2 = _cstrs([os.fsencode(x) for x in r2_paths])
        st = FeedStats()
        T = threads or min(16, os.cpu_count() or 1)
        check(lib().smash_count_fastq(self.h, arr1, len(r1_paths), arr2, len(r2_paths),
                                      int(bool(sort_names)), T, _ptr(d_counts), C.byref(st),
                                      vp(_stream(stream))), "smash_count_fastq")
        return st.as_dict()

    def count_batches(self, d_reads, n_pairs, batch_pairs, d_counts, stream=None,
                      resident=False):
        """n_pairs resident pairs in batches (smash_count_batches): one batch's
        search overlaps the previous one's tail.  resident=True: the reads are
        complete already (smash_count_batches_ready, no input event), so the
        searches need not wait for the work queued on the stream before this
        call -- consecutive runs over the same reads overlap."""
        if resident:
            check(lib().smash_count_batches_ready(self.h, _reads(d_reads, n_pairs, self.stride),
                                                  n_pairs, batch_pairs,
                                                  _ptr(d_counts), vp(_stream(stream)), None),
                  "smash_count_batches_ready")
            return
        check(lib().smash_count_batches(self.h, _reads(d_reads, n_pairs, self.stride), n_pairs,
                                        batch_pairs,
                                        _ptr(d_counts), vp(_stream(stream))),
              "smash_count_batches")

    def phase_map(self, d_reads, n_pairs, stream=None):
        check(lib().smash_phase_map(self.h, _reads(d_reads, n_pairs, self.stride), n_pairs,
                                    vp(_stream(stream))),
              "smash_phase_map")

    def phase_map_ahead(self, d_reads, n_pairs, d_next, n_next, stream=None):
        """phase_map, and the next batch's search issued at once on the
        pipeline's other search stream (smash_phase_map_ahead)."""
        check(lib().smash_phase_map_ahead(self.h, _reads(d_reads, n_pairs, self.stride), n_pairs,
                                          _reads(d_next, n_next, self.stride) if n_next else None,
                                          n_next,
                                          vp(_stream(stream))), "smash_phase_map_ahead")

    def phase_search_ahead(self, d_reads, n_pairs, stream=None):
        """after phase_export of batch b: batch b + 2's search into the set
        b used (smash_phase_search_ahead)."""
        check(lib().smash_phase_search_ahead(self.h, _reads(d_reads, n_pairs, self.stride), n_pairs,
                                             vp(_stream(stream))), "smash_phase_search_ahead")

    def phase_export(self, world, global_base, stream=None):
        """(headers [n, hdr_words] int64, words [w] int64, per-owner key counts,
        per-owner word counts) -- the tensors alias pipeline-owned device
        memory, valid until the next export."""
        import torch
        counts = np.zeros(world, np.int64)
        wcounts = np.zeros(world, np.int64)
        ds, dw = vp(), vp()
        check(lib().smash_phase_export(self.h, world, global_base, _p(counts, i64p),
                                       _p(wcounts, i64p), C.byref(ds), C.byref(dw),
                                       vp(_stream(stream))), "smash_phase_export")
        n, w = int(counts.sum()), int(wcounts.sum())
        H = self.hdr_words
        hdr = device_view(ds.value, 8 * H * n, torch.int64).view(n, H) if n else \
            torch.zeros((0, H), dtype=torch.int64, device="cuda")
        words = device_view(dw.value, 8 * w, torch.int64) if w else \
            torch.zeros(0, dtype=torch.int64, device="cuda")
        return hdr, words, counts, wcounts

    def dedup_owner(self, d_recv, n_recv, d_recv_words, recv_counts, recv_words, d_flags,
                    stream=None):
        rc = np.ascontiguousarray(recv_counts, np.int64)
        rw = np.ascontiguousarray(recv_words, np.int64)
        check(lib().smash_dedup_owner(self.h, _ptr(d_recv), n_recv, _ptr(d_recv_words),
                                      _p(rc, i64p), _p(rw, i64p), len(rc), _ptr(d_flags),
                                      vp(_stream(stream))), "smash_dedup_owner")

    def phase_import(self, d_flags_back, stream=None):
        check(lib().smash_phase_import(self.h, _ptr(d_flags_back), vp(_stream(stream))),
              "smash_phase_import")

    def phase_positions(self, d_tail, stream=None):
        check(lib().smash_phase_positions(self.h, _ptr(d_tail), vp(_stream(stream))),
              "smash_phase_positions")

    def phase_bin(self, d_prev, d_counts, stream=None):
        check(lib().smash_phase_bin(self.h, _ptr(d_prev), _ptr(d_counts),
                                    vp(_stream(stream))), "smash_phase_bin")

    def reset(self, stream=None, keep_search=False):
        """a new run (smash_pipeline_reset); keep_search: look-ahead searches
        already issued stay valid for it (smash_pipeline_reset_ex,
        SMASH_RESET_KEEP_SEARCH)"""
        if keep_search:
            check(lib().smash_pipeline_reset_ex(self.h, 1, vp(_stream(stream))),
                  "smash_pipeline_reset_ex")
        else:
            check(lib().smash_pipeline_reset(self.h, vp(_stream(stream))), "smash_pipeline_reset")

    def reads_resident(self, on=True):
        """the reads later given to the phase calls are resident and complete:
        their searches wait on no input event (smash_pipeline_reads_resident)"""
        check(lib().smash_pipeline_reads_resident(self.h, 1 if on else 0),
              "smash_pipeline_reads_resident")

    @property
    def map_hints(self):
        """the searches hand forward matches' right map.bin bytes to the post
        stage (smash_pipeline_map_hints)"""
        return bool(lib().smash_pipeline_map_hints(self.h))

    @property
    def key_capacity(self):
        """keys the persistent pair-key set takes for sure"""
        return int(lib().smash_pipeline_key_capacity(self.h))

    def reserve_keys(self, keys, stream=None):
        """grow the key set to `keys` keys; held keys move into the larger set
        (smash_pipeline_reserve_keys)"""
        check(lib().smash_pipeline_reserve_keys(self.h, int(keys), vp(_stream(stream))),
              "smash_pipeline_reserve_keys")

    def data_error(self, stream=None):
        """the data error recorded by the work queued on `stream` (0: none);
        waits for that stream only (smash_pipeline_error)"""
        e = C.c_int32()
        check(lib().smash_pipeline_error(self.h, vp(_stream(stream)), C.byref(e)),
              "smash_pipeline_error")
        return int(e.value)

    def stats(self, raise_on_error=True):
        """Counters of the run so far.  A data error the device recorded (the
        mappability_tag throw, a full key set) raises SmashError unless
        raise_on_error=False, so no caller can read counts of a failed run."""
        s = Stats()
        check(lib().smash_pipeline_stats(self.h, C.byref(s)), "smash_pipeline_stats")
        if s.error and raise_on_error:
            raise SmashError("pipeline data error %d: %s" % (s.error, ERRORS.get(s.error, "?")))
        return s

    def profile(self, enable=True):
        check(lib().smash_pipeline_profile(self.h, int(enable)), "smash_pipeline_profile")

    def profile_read(self):
        """(summed k_mam milliseconds, launches, reads searched)"""
        ms = C.c_double()
        n = C.c_uint64()
        r = C.c_uint64()
        check(lib().smash_pipeline_profile_read(self.h, C.byref(ms), C.byref(n), C.byref(r)),
              "smash_pipeline_profile_read")
        return ms.value, n.value, r.value

    def profile_active(self):
        """milliseconds during which at least one profiled search launch ran"""
        ms = C.c_double()
        check(lib().smash_pipeline_profile_active(self.h, C.byref(ms)),
              "smash_pipeline_profile_active")
        return ms.value

    def profile_intervals(self):
        """[(start, end)] ms of every profiled search launch, from the first start"""
        n = C.c_uint64()
        check(lib().smash_pipeline_profile_intervals(self.h, None, 0, C.byref(n)),
              "smash_pipeline_profile_intervals")
        out = (C.c_double * (2 * max(n.value, 1)))()
        check(lib().smash_pipeline_profile_intervals(self.h, out, n.value, C.byref(n)),
              "smash_pipeline_profile_intervals")
        return [(out[2 * i], out[2 * i + 1]) for i in range(n.value)]

    def positions(self):
        """(pos0, abspos) int64 arrays of the positions the last batch emitted
        (smash_pipeline_positions), in emission order."""
        n = C.c_uint64()
        check(lib().smash_pipeline_positions(self.h, None, None, 0, C.byref(n)),
              "smash_pipeline_positions")
        pos0 = np.zeros(n.value, np.int64)
        absp = np.zeros(n.value, np.int64)
        check(lib().smash_pipeline_positions(self.h, _p(pos0, i64p), _p(absp, i64p), n.value,
                                             C.byref(n)), "smash_pipeline_positions")
        return pos0, absp

    def peek(self, n_pairs):
        nk = np.zeros(n_pairs, np.int32)
        keep = np.zeros(n_pairs, np.uint8)
        hits = np.zeros(n_pairs * 2 * self.slots, np.uint64)
        check(lib().smash_pipeline_peek(self.h, _p(nk, i32p), _p(keep, u8p),
                                        _p(hits, u64p), None), "smash_pipeline_peek")
        return nk, keep, hits.reshape(n_pairs, 2 * self.slots)

    def close(self):
        """free the pipeline's device buffers now (its streams are
        synchronised first); the object is unusable afterwards"""
        if self.h:
            lib().smash_pipeline_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _reads(x, n_pairs, read_len):
    """the pointer of a batch of n_pairs pairs: a torch tensor must hold
    2 * n_pairs * read_len bytes (the kernels read that many; a short tensor
    would be an out-of-bounds device read), a raw pointer is the caller's
    responsibility"""
    if x is not None and not isinstance(x, int) and n_pairs:
        have = x.numel() * x.element_size()
        if have < 2 * n_pairs * read_len:
            raise SmashError("reads tensor holds %d bytes, %d pairs x %d bp need %d"
                             % (have, n_pairs, read_len, 2 * n_pairs * read_len))
    return _ptr(x)


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return vp(x)
    return vp(x.data_ptr())


def map_batch(index: Index, d_reads, n_reads, read_len, d_out, cap, d_n, min_len=20,
              stream=None, mode=SMASH_MODE_MAM):
    """longSA::MAM over a batch (smash_map_batch)."""
    check(lib().smash_map_batch(index.h, mode, min_len, _ptr(d_reads),
                                read_len, None, read_len, n_reads, _ptr(d_out), cap,
                                _ptr(d_n), vp(_stream(stream))), "smash_map_batch")


def match_batch(index: Index, d_reads, n_reads, read_len, d_out, cap, d_n, mode="MAM",
                min_len=20, stream=None):
    """longSA::MAM / MUM / MEM over a batch (smash_match_batch, memsam's default /
    -mum / -maxmatch).  d_out: int64 tensor of 2*cap*n_reads words (smash_match
    {u64 ref; u32 query; u32 len})."""
    check(lib().smash_match_batch(index.h, MODES.get(mode, mode), min_len, _ptr(d_reads),
                                  read_len, None, read_len, n_reads, _ptr(d_out), cap,
                                  _ptr(d_n), vp(_stream(stream))), "smash_match_batch")


def bin_positions(d_pos0, d_abspos, n, prev_pos0, d_bin_starts, nbins, d_counts, stream=None):
    """varbin.py's counting loop on the device (smash_bin_positions); returns
    [TotalReads, DupsRemoved, ReadsKept] of this call."""
    st = np.zeros(3, np.uint64)
    check(lib().smash_bin_positions(_ptr(d_pos0), _ptr(d_abspos), n, prev_pos0,
                                    _ptr(d_bin_starts), nbins, _ptr(d_counts), _p(st, u64p),
                                    vp(_stream(stream))), "smash_bin_positions")
    return [int(x) for x in st]


def mappability_scan(index: Index, begin, end, k=36, d_map_out=None, chrom_off=None,
                     d_bin_starts=None, nbins=0, d_bin_counts=None, d_contig_counts=None,
                     stream=None):
    """map.bin bytes of forward bases [begin, end) and unique-k-mer counts
    (smash_mappability_scan).  chrom_off: host int64 per contig or None."""
    off = None if chrom_off is None else np.ascontiguousarray(chrom_off, np.int64)
    check(lib().smash_mappability_scan(index.h, begin, end, k, _ptr(d_map_out),
                                       None if off is None else _p(off, i64p),
                                       _ptr(d_bin_starts), nbins, _ptr(d_bin_counts),
                                       _ptr(d_contig_counts), vp(_stream(stream))),
          "smash_mappability_scan")


def mappability_prepare(index: Index, begin, end, stream=None):
    """C5's preparation from the index arrays (smash_mappability_prepare):
    U and its directory for the scan of forward bases [begin, end), rebuilt
    from SA + the LCP bytes, in place."""
    check(lib().smash_mappability_prepare(index.h, begin, end, vp(_stream(stream))),
          "smash_mappability_prepare")


def mappability_release(index: Index):
    """free mappability_prepare's scratch HBM (smash_mappability_release)"""
    check(lib().smash_mappability_release(index.h), "smash_mappability_release")


def mappability_window(index: Index, begin, end):
    """the text window [lo, hi) mappability_prepare(begin, end) rebuilds"""
    lo, hi = C.c_uint64(), C.c_uint64()
    check(lib().smash_mappability_window(index.h, begin, end, C.byref(lo), C.byref(hi)),
          "smash_mappability_window")
    return int(lo.value), int(hi.value)


def unpack_records(words, n, cap):
    """smash_match records (2 u64 words each) -> [(ref, query, len)] (first min(n, cap))"""
    w = np.asarray(words, np.uint64).reshape(-1, 2)[:min(int(n), cap)]
    return [(int(a), int(b & 0xFFFFFFFF), int(b >> 32)) for a, b in w]


def unpack_matches(words, n):
    """packed u64 (ref 48 | qoff 8 | len 8) -> [(ref, qoff, len)]"""
    w = np.asarray(words[:n], np.uint64)
    return [(int(x & 0xFFFFFFFFFFFF), int((x >> 48) & 0xFF), int(x >> 56)) for x in w]


_HIP = None


class _DeviceArray:
    """__cuda_array_interface__ view of raw device memory (torch.as_tensor)."""

    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr,
                                         "data": (int(ptr), False), "version": 3,
                                         "strides": None}


def device_view(dptr, nbytes, torch_dtype):
    """A torch tensor aliasing nbytes of device memory at dptr (no copy)."""
    import torch
    size = torch.tensor([], dtype=torch_dtype).element_size()
    ts = {1: "|u1", 4: "<i4", 8: "<i8"}[size]
    return torch.as_tensor(_DeviceArray(dptr, nbytes // size, ts), device="cuda")


def download(dptr, nbytes, dtype=np.uint8):
    """Device -> host copy of raw device memory (tests / index export)."""
    global _HIP
    if _HIP is None:
        _HIP = C.CDLL("libamdhip64.so")
        _HIP.hipMemcpy.argtypes = [vp, vp, C.c_size_t, C.c_int]
        _HIP.hipDeviceSynchronize.argtypes = []
    out = np.empty(nbytes, np.uint8)
    _HIP.hipDeviceSynchronize()
    rc = _HIP.hipMemcpy(out.ctypes.data_as(vp), vp(dptr), nbytes, 2)
    if rc != 0:
        raise SmashError("hipMemcpy D2H failed (%d)" % rc)
    return out.view(dtype)


SAM_REC = np.dtype([("pos", "<i8"), ("tid", "<u4"), ("xe", "<u4"), ("prefix", "<u2"),
                    ("len", "<u2"), ("suffix", "<u2"), ("qpos", "<u2"), ("rc", "u1"),
                    ("pad", "u1"), ("spare", "<u2"), ("left", "<i4"), ("right", "<i4"),
                    ("reserved", "<u4")])


def _cstrs(xs):
    if xs is None:
        return None
    return (C.c_char_p * len(xs))(*[None if x is None else bytes(x) for x in xs])


def sam_format(contigs, h_rec, h_n, cap, names, seqs, quals=None, optionals=None, nomap=True,
               tag=False, small_chr=None):
    """Host half of the mapout writer (smash_sam_format, query.cpp:231-415):
    SAM lines from the per-match records (read r's at r * cap, or packed read
    after read when cap is 0, as sam_records returns them); returns
    (bytes, tag_error)."""
    h_rec = np.ascontiguousarray(h_rec)
    h_n = np.ascontiguousarray(h_n, np.uint32)
    packed = cap == 0 or bool(cap & SAM_PACKED)
    need = int(h_n.astype(np.int64).sum()) if packed else len(names) * cap
    assert h_rec.nbytes >= need * SAM_REC.itemsize and len(h_n) == len(names)
    sm = None if small_chr is None else np.ascontiguousarray(small_chr, np.uint8)
    out = C.c_void_p()
    olen = C.c_uint64()
    terr = C.c_int32()
    check(lib().smash_sam_format(_cstrs([c.encode() for c in contigs]), len(contigs),
                                 _p(h_rec, vp), _p(h_n, u32p), cap, len(names), _cstrs(names),
                                 _cstrs(seqs), _cstrs(quals), _cstrs(optionals), int(nomap),
                                 int(tag), None if sm is None else _p(sm, u8p), C.byref(out),
                                 C.byref(olen), C.byref(terr)), "smash_sam_format")
    try:
        text = C.string_at(out.value, olen.value)
    finally:
        lib().smash_sam_free(out)
    return text, terr.value


def sam_records(index: Index, d_reads, n, read_len, cap, tag_offsets=None, min_len=20,
                stream=None):
    """MAM search + per-match records on the device (smash_map_batch ->
    smash_sam_records_packed); returns host copies (SAM_REC[sum(counts)] packed
    read after read, counts[n]).  The record table is sized by the matches
    found (an exclusive scan of the counts), not by n * cap."""
    import torch
    dev = d_reads.device
    d_m = torch.empty(n * cap, dtype=torch.int64, device=dev)
    d_n = torch.empty(n, dtype=torch.int32, device=dev)
    map_batch(index, d_reads, n, read_len, d_m, cap, d_n, min_len=min_len, stream=stream)
    cnt = d_n.to(torch.int64).clamp_(max=cap)
    d_off = torch.cumsum(cnt, 0) - cnt
    total = int(cnt.sum().item()) if n else 0
    d_rec = torch.empty(max(total, 1) * SAM_REC.itemsize, dtype=torch.uint8, device=dev)
    d_tag = None
    if tag_offsets is not None:
        d_tag = torch.from_numpy(np.ascontiguousarray(tag_offsets, np.uint32).view(np.int32)).to(dev)
    check(lib().smash_sam_records_packed(index.h, _ptr(d_reads), read_len, None, read_len, n, _ptr(d_m),
                                         cap, _ptr(d_n), _ptr(d_off), _ptr(d_tag), _ptr(d_rec),
                                         vp(_stream(stream))),
          "smash_sam_records_packed")
    torch.cuda.synchronize(dev)
    h_n = d_n.cpu().numpy().view(np.uint32).copy()
    if (h_n > cap).any():
        raise SmashError("sam_records: a read has more matches than cap")
    return d_rec[:total * SAM_REC.itemsize].cpu().numpy().view(SAM_REC), h_n


def sam_lines(index: Index, d_reads, read_len, names, seqs, quals=None, optionals=None,
              nomap=True, tag_offsets=None, small_chr=None, cap=None, min_len=20, stream=None):
    """memsam `-rcref -samin -samout [-nomap]` lines for 2n mates (read 1, read 2 of
    each pair, names with the ':0'/':1' suffix of query.cpp:641-642): the MAM search
    (smash_map_batch), the per-match records on the device (smash_sam_records) and
    the host formatting of print_matches (query.cpp:331-415).  With tag_offsets
    (u32 sam_header offsets per forward contig) the mappability_tag L/R columns
    are appended (mappability_tag.cpp:93-124).  Returns (bytes, tag_error)."""
    n = len(names)
    if cap is None:
        cap = read_len - min_len + 1
    h_rec, h_n = sam_records(index, d_reads, n, read_len, cap, tag_offsets, min_len, stream)
    return sam_format(index.contigs, h_rec, h_n, SAM_PACKED | cap, names, seqs, quals, optionals,
                      nomap, tag_offsets is not None, small_chr)


def read_fastq_pairs(r1_paths, r2_paths, batch_pairs=1 << 20, name_stride=64):
    """All pairs of the two FASTQ lists through the native reader
    (smash_fastq_*): (names[n] as a fixed-width bytes array, reads[2n, L] u8
    after replaceN + lowercasing), in file order."""
    arr1 = _cstrs([p.encode() for p in r1_paths])
    arr2 = _cstrs([p.encode() for p in r2_paths])
    h = vp()
    check(lib().smash_fastq_open(arr1, len(r1_paths), arr2, len(r2_paths), C.byref(h)),
          "smash_fastq_open")
    try:
        L = C.c_uint32(0)
        reads, names = [], []
        while True:
            cap_len = L.value or 255
            rb = np.empty(2 * batch_pairs * cap_len, np.uint8)
            nb = np.zeros(batch_pairs, "S%d" % name_stride)
            n = C.c_uint64()
            check(lib().smash_fastq_read(h, batch_pairs, C.byref(L), _p(rb, vp), _p(nb, vp),
                                         name_stride, C.byref(n)), "smash_fastq_read")
            k = n.value
            if k:
                reads.append(rb[:2 * k * L.value].reshape(2 * k, L.value).copy())
                names.append(nb[:k].copy())
            if k < batch_pairs:
                break
    finally:
        lib().smash_fastq_close(h)
    if not reads:
        return np.zeros(0, "S%d" % name_stride), np.zeros((0, 0), np.uint8)
    return np.concatenate(names), np.concatenate(reads)


def read_fastq_pairs_parallel(r1_paths, r2_paths, threads=0, name_stride=64, read_len=0):
    """read_fastq_pairs through the parallel reader (smash_fastq_read_parallel):
    strict 4-line FASTQ only (SmashError SMASH_ERR_UNSUPPORTED otherwise)."""
    arr1 = _cstrs([os.fsencode(p) for p in r1_paths])
    arr2 = _cstrs([os.fsencode(p) for p in r2_paths])
    T = threads or min(16, os.cpu_count() or 1)
    L = C.c_uint32(read_len)
    n = C.c_uint64()
    check(lib().smash_fastq_read_parallel(arr1, len(r1_paths), arr2, len(r2_paths), T, C.byref(L),
                                          0, None, None, name_stride, C.byref(n)),
          "smash_fastq_read_parallel")
    k = n.value
    rb = np.empty((2 * max(k, 1), max(L.value, 1)), np.uint8)
    nb = np.zeros(max(k, 1), "S%d" % name_stride)
    check(lib().smash_fastq_read_parallel(arr1, len(r1_paths), arr2, len(r2_paths), T, C.byref(L),
                                          k, _p(rb, vp), _p(nb, vp), name_stride, C.byref(n)),
          "smash_fastq_read_parallel")
    if not k:
        return np.zeros(0, "S%d" % name_stride), np.zeros((0, 0), np.uint8)
    return nb[:k], rb[:2 * k, :L.value]


class FastqIndex:
    """Both FASTQ lists indexed once by the parallel reader
    (smash_fastq_index_*): .n pairs of .L bases in samtools sort -n order;
    pack(k0, k1, out) fills a [2 (k1 - k0), L] uint8 array (or a pinned CPU
    tensor) with planned pairs [k0, k1).  Strict 4-line FASTQ only."""

    def __init__(self, r1_paths, r2_paths, threads=0, read_len=0, sort_names=False):
        a1 = _cstrs([os.fsencode(p) for p in r1_paths])
        a2 = _cstrs([os.fsencode(p) for p in r2_paths])
        T = threads or min(16, os.cpu_count() or 1)
        L = C.c_uint32(read_len)
        n = C.c_uint64()
        h = vp()
        check(lib().smash_fastq_index_open(a1, len(r1_paths), a2, len(r2_paths), T, C.byref(L),
                                           int(bool(sort_names)), C.byref(h), C.byref(n)),
              "smash_fastq_index_open")
        self.h, self.n, self.L = h, n.value, L.value

    def pack(self, k0, k1, out):
        ptr = out.data_ptr() if hasattr(out, "data_ptr") else out.ctypes.data
        check(lib().smash_fastq_index_pack(self.h, k0, k1, vp(ptr), None, 0),
              "smash_fastq_index_pack")
        return out

    def close(self):
        if self.h:
            lib().smash_fastq_index_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


SMASH_ERR_NOMEM = -4
SMASH_ERR_UNSUPPORTED = -5


class FastqShards:
    """The rank-local reader of the multi-GPU driver (smash_fastq_shard_*):
    this rank scans only its share of the segments of both FASTQ lists,
    `allgather(bytes) -> [bytes of rank 0, ..., rank world-1]` exchanges the
    scans, and every rank gets the same plan.  Same interface as FastqIndex
    (.n planned pairs of .L bases, pack(k0, k1, out)), but a pack reads only
    the bytes of the pairs asked for.  Raises SmashError with .code
    SMASH_ERR_UNSUPPORTED where FastqIndex must take over (input not strict
    4-line FASTQ, or not in samtools sort -n order when sort_names)."""

    def __init__(self, r1_paths, r2_paths, rank, world, allgather, threads=0, read_len=0,
                 sort_names=False):
        a1 = _cstrs([os.fsencode(p) for p in r1_paths])
        a2 = _cstrs([os.fsencode(p) for p in r2_paths])
        T = threads or min(16, os.cpu_count() or 1)
        blob, nb = vp(), C.c_uint64()
        L = lib()
        rc = L.smash_fastq_shard_scan(a1, len(r1_paths), a2, len(r2_paths), world, rank, T,
                                      C.byref(blob), C.byref(nb))
        mine = b""
        err = None
        if rc == 0:
            mine = C.string_at(blob.value, nb.value)
            L.smash_fastq_shard_free_blob(blob)
        else:
            err = (rc, L.smash_last_error().decode(errors="replace"))
        blobs = allgather(mine)     # every rank joins, even after a local failure
        if err is not None:
            e = SmashError("smash_fastq_shard_scan failed (%d): %s" % err)
            e.code = err[0]
            raise e
        if any(len(b) == 0 for b in blobs):
            e = SmashError("smash_fastq_shard_scan failed on another rank")
            e.code = -1
            raise e
        bufs = [C.create_string_buffer(b, len(b)) for b in blobs]
        ptrs = (vp * world)(*[C.cast(b, vp) for b in bufs])
        sizes = np.array([len(b) for b in blobs], np.uint64)
        Lr = C.c_uint32(read_len)
        n = C.c_uint64()
        h = vp()
        rc = L.smash_fastq_shard_open(a1, len(r1_paths), a2, len(r2_paths), world, rank, ptrs,
                                      _p(sizes, u64p), T, C.byref(Lr), int(bool(sort_names)),
                                      C.byref(h), C.byref(n))
        if rc != 0:
            e = SmashError("smash_fastq_shard_open failed (%d): %s"
                           % (rc, L.smash_last_error().decode(errors="replace")))
            e.code = rc
            raise e
        self.h, self.n, self.L = h, n.value, Lr.value

    def pack(self, k0, k1, out):
        ptr = out.data_ptr() if hasattr(out, "data_ptr") else out.ctypes.data
        check(lib().smash_fastq_shard_pack(self.h, k0, k1, vp(ptr)), "smash_fastq_shard_pack")
        return out

    def stats(self):
        st = ShardStats()
        check(lib().smash_fastq_shard_stats(self.h, C.byref(st)), "smash_fastq_shard_stats")
        return st.as_dict()

    def close(self):
        if self.h:
            lib().smash_fastq_shard_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def first_read_length(paths):
    """bases in the first record of the first file (FASTQ / FASTA, gzip or
    plain): the read length a file-fed pipeline is built for."""
    import gzip
    with open(paths[0], "rb") as f:
        magic = f.read(2)
    op = gzip.open if magic == b"\x1f\x8b" else open
    with op(paths[0], "rb") as f:
        for line in f:
            t = line.strip()
            if not t:
                continue
            if t[:1] not in (b"@", b">"):
                raise SmashError("%s: not FASTQ / FASTA" % paths[0])
            return len(next(f).rstrip(b"\r\n"))
    raise SmashError("%s: no records" % paths[0])


def strnum_order(names):
    """Stable `samtools sort -n` order of a fixed-width bytes array
    (smash_strnum_order)."""
    names = np.ascontiguousarray(names)
    perm = np.empty(len(names), np.uint64)
    check(lib().smash_strnum_order(_p(names, vp), names.dtype.itemsize, len(names),
                                   _p(perm, u64p)), "smash_strnum_order")
    return perm.astype(np.int64)
