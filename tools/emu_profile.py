"""tools/emu_profile.py [--genome chr21] [--reads 4000] -- the search kernel's
work per read on the CPU: runs k_mam_sm (tools/sm_emu: the kernel source, one
lane) over a host index of a synthetic genome and SMASH reads made exactly as
bench.py makes them, and prints lane iterations per read by state, 16-byte
probes and 64-byte line transitions per array, and whether the matches equal
the oracle's (orc_mam_fast).

The chr21-sized genome (N = 96 M, k-mer table K = 13) has the same suffixes
per table k-mer as hg19 (K = 16): 1.43 vs 1.44, so root descents, runs and
chains look alike; the GPU's STATS run on hg19 (tools/diag_sq.sh) is the
check.  The index is cached under /tmp.  Test tooling only.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("smash-paper_amd", "tools", "tools/sm_emu", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import oracle as O  # noqa: E402
import sm_emu  # noqa: E402
import synth  # noqa: E402


def load_index(kind):
    cache = "/tmp/emu_ix_%s.npz" % kind
    contigs = synth.make_genome(kind)
    T, sp, sz, names = O.text_from_contigs(contigs)
    if os.path.exists(cache):
        z = np.load(cache)
        ix = O.Index(T, sp, sz, names, SA=z["SA"], ISA=z["ISA"], L8=z["L8"], ovf=z["ovf"])
    else:
        t = time.time()
        ix = O.Index(T, sp, sz, names)
        print("[emu] index %s N=%d built in %.0fs" % (kind, ix.N, time.time() - t), file=sys.stderr)
        np.savez(cache, SA=ix.SA, ISA=ix.ISA, L8=ix.L8, ovf=ix.ovf)
    ix.accel()
    return contigs, ix


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--genome", default="chr21")
    ap.add_argument("--reads", type=int, default=4000)
    ap.add_argument("--len", type=int, default=150)
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--packed", action="store_true",
                    help="the packed SA / ISA words (8-byte elements, as the device at hg19)")
    a = ap.parse_args()
    import smashgpu as S
    contigs, ix = load_index(a.genome)
    r1, r2 = synth.make_reads(contigs, a.reads // 2, a.len, seed=3000)
    reads = np.empty((a.reads, a.len), np.uint8)
    reads[0::2] = r1
    reads[1::2] = r2
    reads = S.prepare_reads(reads)
    emu = sm_emu.Emu(ix, copy=False, packed=a.packed)
    t = time.time()
    got, iters = emu.map(reads)
    dt = time.time() - t
    n = len(reads)
    print("[emu] %s: %d reads x %d bp, %.1f s; lane iterations/read %.1f"
          % (a.genome, n, a.len, dt, iters.mean()))
    print("  by state: " + " ".join("%s %.2f" % (k, v / n) for k, v in emu.states.items()))
    pr = {k: v[0] / n for k, v in emu.counters.items()}
    ln = {k: v[1] / n for k, v in emu.counters.items()}
    print("  probes/read %.1f: " % sum(pr.values()) + " ".join("%s %.2f" % kv for kv in pr.items()))
    print("  lines/read  %.1f: " % sum(ln.values()) + " ".join("%s %.2f" % kv for kv in ln.items()))
    print("  matches/read %.2f" % (sum(len(g) for g in got) / n))
    print("  requests/read %.2f (speculative %.2f)" % (emu.requests[0] / n, emu.requests[1] / n))
    import ctypes as C
    rq = np.zeros((128, 4), np.uint64)
    sm_emu.lib().sm_emu_req_by_state(rq.ctypes.data_as(C.c_void_p))
    stn = ["EXIT", "NEW", "ALU", "COPY", "BM", "KT", "IDX", "BYTE", "CMP", "USCAN", "EXL", "EXR", "EXB"]
    idxop = ["SAPOS", "SAPOS2", "BS_SA", "ISAJ", "NS_SA2", "NS_ISA2"]
    print("  requests/read by state.op: all / re-probe (line among the lane's last 8) / speculative / crossing")
    for k in range(128):
        if rq[k, 0]:
            st, op = k >> 3, k & 7
            nm = stn[st] + ("." + (idxop[op] if st == 6 else ("EXT" if op == 0 else "BS")) if st in (6, 8) else "")
            print("    %-14s %6.2f %6.2f %6.2f %6.2f" % ((nm,) + tuple(rq[k] / n)))
    import ctypes as C
    hs, hd = np.zeros(65, np.uint64), np.zeros(256, np.uint64)
    sm_emu.lib().sm_emu_bs_hist(hs.ctypes.data_as(C.c_void_p), hd.ctypes.data_as(C.c_void_p), 1)
    tot = max(1, int(hs.sum()))
    print("  binary searches/read %.2f; by interval size: " % (tot / n)
          + " ".join("%d:%.1f%%" % (k, 100.0 * hs[k] / tot) for k in range(1, 65) if hs[k] * 200 >= tot))
    bm = hd[244:256].copy()
    hd[244:256] = 0
    print("  by start depth: " + " ".join("%d:%.1f%%" % (k, 100.0 * hd[k] / tot)
                                          for k in range(244) if hd[k] * 50 >= tot))
    if bm.sum():
        print("  (F) cover policy per read, mode:probe1 probe2 present: " + " ".join(
            "%d:%d%d %.2f" % (k // 4, (k >> 1) & 1, k & 1, bm[k] / n) for k in range(12) if bm[k]))
    if not a.no_check:
        bad = 0
        for i in range(n):
            exp = sorted(ix.search_fast(reads[i].tobytes()))
            if sorted(got[i]) != exp:
                bad += 1
        print("  oracle check: %d / %d reads differ" % (bad, n))
        if bad:
            sys.exit(1)


if __name__ == "__main__":
    main()
