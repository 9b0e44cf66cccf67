"""tools/sm_emu/sm_emu.py -- ctypes wrapper of the single-lane host emulation
of the device MAM state machine (sm_emu.cpp).  Test tooling only."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libsmemu.so")
_lib = None


def build():
    srcs = [os.path.join(HERE, f) for f in ("sm_emu.cpp", "hip/hip_runtime.h")] + [
        os.path.join(HERE, "..", "..", "smash-paper_amd", "csrc", f)
        for f in ("mam_sm.hpp", "mam_device.hpp", "common.hpp")]
    if os.path.exists(LIB) and all(os.path.getmtime(LIB) >= os.path.getmtime(s) for s in srcs):
        return LIB
    tmp = "%s.%d.tmp" % (LIB, os.getpid())   # atomic: parallel test workers may build at once
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-I", HERE,
                           "-I", os.path.join(HERE, "..", "..", "include"),
                           "-o", tmp, os.path.join(HERE, "sm_emu.cpp")])
    os.replace(tmp, LIB)
    return LIB


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        _lib.sm_emu_map.restype = C.c_int
    return _lib


def _padded(a, dtype):
    """16-byte block loads may touch up to 15 bytes past an element: copy into
    a 64-byte aligned buffer with 64 bytes of zero padding."""
    a = np.ascontiguousarray(a, dtype)
    raw = np.zeros(a.nbytes + 128, np.uint8)
    off = (-raw.ctypes.data) % 64
    buf = raw[off:off + a.nbytes + 64]
    buf[:a.nbytes] = a.view(np.uint8).reshape(-1)
    return buf, raw


def in_text_words(in_text):
    w = np.zeros(4, np.uint64)
    for b in range(256):
        if in_text[b]:
            w[b >> 6] |= np.uint64(1) << np.uint64(b & 63)
    return w


# "bitmap": the window filter's probes (k-mer table entries since round 3)
ARRAYS = ("text", "sa", "isa", "lcp", "uniq", "kmer", "bitmap", "records")
# k_mam_sm lane states and ops (mam_sm.hpp enums), for the STATS counters
STATES = ("EXIT", "NEW", "ALU", "COPY", "BM", "KT", "IDX", "BYTE", "CMP", "USCAN", "EXL", "EXR", "EXB")
IDX_OPS = ("SAPOS", "SAPOS2", "BS_SA", "ISAJ", "NS_SA2", "NS_ISA2")
CMP_OPS = ("EXT", "BS")


POS_BITS = 33          # packed index words (smash-paper_amd/csrc/common.hpp)
POS_MASK = (1 << POS_BITS) - 1
WINDOW = 7


def pack_words(T, SA, ISA, L8, K):
    """The packed SA / ISA words (common.hpp layout; the device builds them in
    pack_index.hip) from plain arrays, on the host: u64 SA and ISA whose
    bits 33.. hold the BWT character / window tag, the L8 bytes around the
    rank and 7 bases of T[x + K ..) (SA), and L8[r - 1 .. r + 2] (ISA)."""
    N = len(SA)
    assert N <= POS_MASK
    x = np.asarray(SA, np.uint64)
    lut = np.full(256, 255, np.uint8)
    for i, ch in enumerate(b"acgt"):
        lut[ch] = i
    Tp = np.zeros(N + 64, np.uint8)
    Tp[:N] = np.asarray(T[:N], np.uint8)
    l8 = np.minimum(np.asarray(L8[:N], np.uint64), 127)
    l8p = np.zeros(N + 4, np.uint64)
    l8p[1:N + 1] = l8                      # l8p[r + 1] = L8[r], 0 outside [0, N)
    xi = x.astype(np.int64)
    bwt = np.where(xi > 0, lut[Tp[np.maximum(xi - 1, 0)]], 255).astype(np.uint64)
    tag = np.where(bwt < 4, bwt, 4).astype(np.uint64)
    win = np.zeros(N, np.uint64)
    dirty = np.zeros(N, bool)
    for i in range(WINDOW):
        c = lut[Tp[np.minimum(xi + K + i, N + 63)]]
        dirty |= c == 255
        win |= (c.astype(np.uint64) & np.uint64(3)) << np.uint64(2 * i)
    tag[dirty] = 5
    win[dirty] = 0
    r = np.arange(N, dtype=np.int64)
    sa = (x | (tag << np.uint64(33)) | (l8p[r + 1] << np.uint64(36)) | (l8p[r + 2] << np.uint64(43))
          | (win << np.uint64(50)))
    ri = np.asarray(ISA, np.int64)
    isa = (ri.astype(np.uint64) | (l8p[ri] << np.uint64(33)) | (l8p[ri + 1] << np.uint64(40))
           | (l8p[ri + 2] << np.uint64(47)) | (l8p[ri + 3] << np.uint64(54)))
    return sa, isa


class Emu:
    def __init__(self, ix, wide=False, copy=True, packed=False):
        """ix: oracle.Index with accel() built; wide: run the 8-byte SA/ISA
        instantiation (the device uses it when N >= 2^32); copy=False uses the
        index arrays in place (hg19-sized indexes: no second copy); packed:
        run with the packed index words (the device default at hg19) --
        built here from ix's plain arrays, or ix's own when they are packed
        already (ix.pos_mask, e.g. downloaded from the device)."""
        self.ix = ix
        self.packed = bool(packed)
        if packed:
            wide = True
        self.keep = []
        self.spans = []

        def P(a, dt):
            if copy or a.dtype != np.dtype(dt) or not a.flags.c_contiguous:
                buf, raw = _padded(a, dt)
                self.keep.append(raw)
                nb = np.ascontiguousarray(a, dt).nbytes
            else:
                buf, nb = a, a.nbytes
                self.keep.append(a)
            self.spans += [buf.ctypes.data, buf.ctypes.data + nb]
            return buf.ctypes.data
        self.T = P(ix.T, np.uint8)
        it = np.uint64 if wide else ix.SA.dtype
        if packed and not getattr(ix, "pos_mask", None):
            sa, isa = pack_words(ix.T, ix.SA, ix.ISA, ix.L8, ix.acc.K)
            self.SA = P(sa, np.uint64)
            self.ISA = P(isa, np.uint64)
        else:
            self.SA = P(ix.SA, it)
            self.ISA = P(ix.ISA, it)
        self.L8 = P(ix.L8, np.uint8)
        self.U = P(ix._U, np.uint8)
        self.KT = P(ix._KTF, np.uint64)          # the device layout (orc_build_ktf)
        self.BM = P(np.zeros(1, np.uint64), np.uint64)   # (unused since round 3)
        self.K = ix.acc.K
        self.B = ix.acc.B
        self.it = in_text_words(list(ix.acc.in_text))
        self.isz = np.dtype(it).itemsize

    def map(self, reads, min_len=20, cap=512, lin_blocks=8):   # = the device default (mam.hip)
        """reads: uint8 [n, L].  Returns (list of [(ref, q, len)], iterations);
        self.counters: {array: (16-byte probes, 64-byte line transitions)}."""
        reads = np.ascontiguousarray(reads, np.uint8)
        n, L = reads.shape
        out = np.zeros(n * cap, np.uint64)
        nout = np.zeros(n, np.uint32)
        iters = np.zeros(n, np.uint32)
        spans = np.array(self.spans, np.uint64)   # T SA ISA L8 U KT BM
        viol = np.zeros(10, np.uint64)
        ctr = np.zeros(16, np.uint64)
        from oracle import lib as olib
        logN = olib().orc_logN(C.c_uint64(self.ix.N))
        rc = lib().sm_emu_map(
            C.c_void_p(self.T), C.c_void_p(self.SA), C.c_void_p(self.ISA), self.isz,
            C.c_void_p(self.L8), C.c_void_p(self.U), C.c_void_p(self.KT), self.K,
            C.c_void_p(self.BM), self.B, self.it.ctypes.data_as(C.c_void_p),
            C.c_uint64(self.ix.N), C.c_uint64(logN), reads.ctypes.data_as(C.c_void_p),
            C.c_uint64(L), C.c_uint32(L), C.c_uint64(n), C.c_uint32(min_len),
            out.ctypes.data_as(C.c_void_p), C.c_uint32(cap),
            nout.ctypes.data_as(C.c_void_p), iters.ctypes.data_as(C.c_void_p),
            spans.ctypes.data_as(C.c_void_p), viol.ctypes.data_as(C.c_void_p),
            C.c_uint32(lin_blocks), ctr.ctypes.data_as(C.c_void_p), C.c_int(int(self.packed)))
        assert rc == 0
        assert viol[0] == 0, ("out-of-range probe", viol.tolist())
        res = []
        for i in range(n):
            k = min(int(nout[i]), cap)
            w = out[i * cap:i * cap + k]
            res.append([(int(x & 0xFFFFFFFFFFFF), int((x >> 48) & 0xFF), int(x >> 56)) for x in w])
        self.counters = {name: (int(ctr[k]), int(ctr[8 + k])) for k, name in enumerate(ARRAYS)}
        rq = np.zeros(2, np.uint64)
        lib().sm_emu_requests(rq.ctypes.data_as(C.c_void_p))
        self.requests = (int(rq[0]), int(rq[1]))   # device requests (all, speculative)
        ws = np.zeros(64, np.uint64)
        lib().sm_emu_ws(ws.ctypes.data_as(C.c_void_p))
        self.states = {}
        for k, nm in enumerate(STATES):
            if ws[2 + k]:
                self.states[nm] = int(ws[2 + k])
        for k, nm in enumerate(IDX_OPS):
            if ws[18 + k]:
                self.states["IDX." + nm] = int(ws[18 + k])
        for k, nm in enumerate(CMP_OPS):
            if ws[42 + k]:
                self.states["CMP." + nm] = int(ws[42 + k])
        return res, iters
