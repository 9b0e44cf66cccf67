"""Oracle-backed stand-in for smashgpu.Pipeline's multi-GPU phase API, on CPU
tensors.  TEST INFRASTRUCTURE: lets tests/test_dist_gloo.py drive the real
exchange code (smash-paper_amd/dist.py) over torch.distributed/gloo with
world_size 2 on the CPU, checking its collectives, shard bookkeeping and the
adjacent-dup boundary against a single-process oracle run."""
import hashlib

import numpy as np
import torch

import oracle as O


def key_hash(key):
    d = hashlib.blake2b(repr(key).encode(), digest_size=16).digest()
    hi = int.from_bytes(d[:8], "little") | 1
    lo = int.from_bytes(d[8:], "little") | 1
    return hi, lo


def to_i64(u):
    return u - (1 << 64) if u >= (1 << 63) else u


def to_u64(i):
    return i + (1 << 64) if i < 0 else i


class OraclePhasePipeline:
    def __init__(self, oix, mapbin, chrom_sizes, bin_starts, max_pairs):
        self.oix = oix
        self.map = mapbin
        self.max_pairs = max_pairs
        sizes = [int(x) for x in oix.sizes[0::2]]
        self.offs = np.cumsum([0] + sizes[:-1]).astype(np.uint32)
        self.small = [1 if ("_gl000" in c or "chrM" in c) else 0 for c in oix.contigs]
        self.major = O.major_flags(oix.contigs, chrom_sizes)
        self.coff = [chrom_sizes.get(c, 0) for c in oix.contigs]
        self.bins = np.asarray(bin_starts, np.int64)
        self.reset()

    def reset(self):
        self.seen = set()
        self.total = self.dups = self.kept = 0

    def phase_map(self, d_reads, n_pairs):
        reads = d_reads.numpy()
        self.kept_hits = []
        self.hashes = []
        for q in range(n_pairs):
            hs = []
            for m in (0, 1):
                P = reads[2 * q + m].tobytes()
                h, _ = self.oix.resolve(P, self.oix.search(P))
                for x in h:
                    O.tag(x, self.offs, self.map, self.small[x.tid])
                hs.append(h)
            k = O.smash_pair(hs[0], hs[1])
            self.kept_hits.append(k)
            self.hashes.append(key_hash(tuple(k)) if k is not None else None)
        self.n = n_pairs

    def phase_export(self, world, gbase, d_send):
        first = {}
        for q, h in enumerate(self.hashes):
            if h is not None and h not in first:
                first[h] = q
        groups = [[] for _ in range(world)]
        for h, q in first.items():
            groups[h[0] % world].append((h, q))
        self.order = []
        rows = []
        for w in range(world):
            for h, q in sorted(groups[w], key=lambda t: t[1]):
                rows.append((to_i64(h[0]), to_i64(h[1]), gbase + q))
                self.order.append(q)
        if rows:
            d_send[:len(rows)] = torch.tensor(rows, dtype=torch.int64)
        return np.array([len(g) for g in groups], np.int64)

    def dedup_owner(self, d_recv, n_recv, d_flags):
        rows = d_recv[:n_recv].tolist()
        best = {}
        for j, (hi, lo, g) in enumerate(rows):
            k = (to_u64(hi), to_u64(lo))
            if k not in best or g < rows[best[k]][2]:
                best[k] = j
        flags = np.zeros(n_recv, np.uint8)
        for k, j in best.items():
            if k not in self.seen:
                flags[j] = 1
        self.seen.update(best.keys())
        if n_recv:
            d_flags[:n_recv] = torch.from_numpy(flags)

    def phase_import(self, d_back):
        self.keep = np.zeros(self.n, bool)
        for o, q in enumerate(self.order):
            self.keep[q] = bool(d_back[o].item())

    def phase_positions(self, d_tail):
        self.pos = []
        for q in range(self.n):
            if self.keep[q]:
                for tid, p in self.kept_hits[q]:
                    if self.major[tid]:
                        self.pos.append((p, p + self.coff[tid]))
        d_tail[0] = len(self.pos)
        d_tail[1] = self.pos[-1][0] if self.pos else -1

    def phase_bin(self, d_prev, d_counts):
        st = O.OrcVarbinState(0, 0, 0, int(d_prev.reshape(-1)[0].item()))
        if self.pos:
            c, st = O.varbin([p for p, _ in self.pos], [a for _, a in self.pos],
                             self.bins, state=st)
            d_counts += torch.from_numpy(c.astype(np.int64))
        self.total += st.total
        self.dups += st.dups
        self.kept += st.kept
