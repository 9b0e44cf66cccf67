"""tools/readgen.py -- host side of tools/readgen.hip (synthetic SMASH read
pairs generated on the device from the resident index text; test and bench
data, not part of the product).  The model is tools/synth.py make_reads'
(SURVEY.md §8d); pair q depends only on (seed, q), never on the batch split.

    g = Generator(dix, contigs, read_len=150, seed=3)
    d_reads = g.generate(25_000_000)          # torch uint8 [2n, L] on the device
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        p = os.path.join(HERE, "libreadgen.so")
        if not os.path.exists(p):
            raise RuntimeError("tools/libreadgen.so not built (__graft_entry__.build())")
        L = C.CDLL(p)
        vp = C.c_void_p
        L.rg_generate.argtypes = [vp, vp, vp, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64,
                                  C.c_uint64, C.c_uint32, vp, vp]
        L.rg_iv_bytes.restype = C.c_uint32
        L.rg_write_fastq.argtypes = [vp, C.c_uint64, C.c_uint32, C.c_uint64, C.c_char_p,
                                     C.c_char_p, C.c_int]
        L.rg_write_fastq_lanes.argtypes = [vp, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint32,
                                           C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.c_int]
        _LIB = L
    return _LIB


class Generator:
    def __init__(self, index, contigs, read_len, seed, exclude=("chrM",)):
        import torch
        import synth
        self.torch = torch
        self.index = index
        self.L = int(read_len)
        self.seed = int(seed) * 0x9E3779B1 + 17
        ivs = [iv for iv in synth._allowed_intervals(contigs)
               if contigs[iv[0]][0] not in exclude and "_" not in contigs[iv[0]][0]]
        sizes = index.sizes            # 2 per contig: forward, reverse complement
        arr = np.zeros((len(ivs), 4), np.uint64)
        sp = S_startpos(index)
        for k, (ci, a, b) in enumerate(ivs):
            arr[k] = (a, b, sp[2 * ci], sp[2 * ci + 1] + sizes[2 * ci])
        assert lib().rg_iv_bytes() == 32
        lens = (arr[:, 1] - arr[:, 0]).astype(np.uint64)
        cum = np.cumsum(lens).astype(np.uint64)
        self.total = int(cum[-1])
        dev = torch.device("cuda", torch.cuda.current_device())
        self.d_iv = torch.from_numpy(arr.view(np.int64)).to(dev)
        self.d_cum = torch.from_numpy(cum.view(np.int64)).to(dev)
        self.n_iv = len(ivs)

    def generate(self, n_pairs, q0=0, out=None, stream=None):
        torch = self.torch
        if out is None:
            out = torch.empty((2 * n_pairs, self.L), dtype=torch.uint8, device="cuda")
        s = torch.cuda.current_stream().cuda_stream if stream is None else stream
        rc = lib().rg_generate(self.index.info.d_text, self.d_iv.data_ptr(),
                               self.d_cum.data_ptr(), self.n_iv, self.total, self.seed, q0,
                               n_pairs, self.L, out.data_ptr(), s)
        if rc:
            raise RuntimeError("rg_generate: hip error %d" % rc)
        return out


def write_fastq(h_reads, path1, path2, gz=False, q0=0):
    """pairs of h_reads (numpy uint8 [2n, L], prepared bytes) as a FASTQ pair
    of files in name order (rg_write_fastq)."""
    h = np.ascontiguousarray(h_reads)
    n, L = h.shape[0] // 2, h.shape[1]
    rc = lib().rg_write_fastq(h.ctypes.data, n, L, q0, os.fsencode(path1), os.fsencode(path2),
                              int(gz))
    if rc:
        raise RuntimeError("rg_write_fastq failed (%d)" % rc)


def write_fastq_lanes(h_reads, prefix, lanes, gz=False, q0=0):
    """pairs of h_reads as `lanes` consecutive lane files per mate
    (prefix_L<k>_R<1|2>.fq[.gz], names in order; rg_write_fastq_lanes, one
    thread per file); returns (read-1 paths, read-2 paths)."""
    h = np.ascontiguousarray(h_reads)
    n, L = h.shape[0] // 2, h.shape[1]
    ext = ".fq.gz" if gz else ".fq"
    p1 = ["%s_L%03d_R1%s" % (prefix, k, ext) for k in range(lanes)]
    p2 = ["%s_L%03d_R2%s" % (prefix, k, ext) for k in range(lanes)]
    a1 = (C.c_char_p * lanes)(*[os.fsencode(x) for x in p1])
    a2 = (C.c_char_p * lanes)(*[os.fsencode(x) for x in p2])
    rc = lib().rg_write_fastq_lanes(h.ctypes.data, n, L, q0, lanes, a1, a2, int(gz))
    if rc:
        raise RuntimeError("rg_write_fastq_lanes failed (%d)" % rc)
    return p1, p2


def S_startpos(index):
    """startpos of the doubled text from the contig sizes (fasta.cpp layout:
    c1 ` rc(c1) ` c2 ... rc(cn) $)."""
    sp, pos = [], 0
    sizes = index.sizes
    for k in range(0, len(sizes), 2):
        sp.append(pos)
        pos += sizes[k] + 1
        sp.append(pos)
        pos += sizes[k] + 1
    return sp
