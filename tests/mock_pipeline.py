"""Oracle-backed stand-in for smashgpu.Pipeline's multi-GPU phase API, on CPU
tensors.  TEST INFRASTRUCTURE: lets tests/test_dist_gloo.py drive the real
exchange code (smash-paper_amd/dist.py) over torch.distributed/gloo with
world_size 2 on the CPU, checking its collectives, shard bookkeeping and the
adjacent-dup boundary against a single-process oracle run."""
import hashlib
import os

import numpy as np
import torch

import oracle as O


def key_hash(key):
    d = hashlib.blake2b(repr(key).encode(), digest_size=16).digest()
    hi = int.from_bytes(d[:8], "little") | 1
    lo = int.from_bytes(d[8:], "little") | 1
    bits = int(os.environ.get("SMASH_KEY_HASH_BITS", "0") or 0)   # (as the library: tests)
    if 0 < bits < 64:
        hi = (hi & ((1 << bits) - 1)) | 1
    return hi, lo


def to_i64(u):
    return u - (1 << 64) if u >= (1 << 63) else u


def to_u64(i):
    return i + (1 << 64) if i < 0 else i


class OraclePhasePipeline:
    def __init__(self, oix, mapbin, chrom_sizes, bin_starts, max_pairs, key_capacity=1 << 40):
        self.oix = oix
        self.map = mapbin
        self.max_pairs = max_pairs
        self.key_capacity = key_capacity   # smash_pipeline_key_capacity
        self.error = 0
        sizes = [int(x) for x in oix.sizes[0::2]]
        self.offs = np.cumsum([0] + sizes[:-1]).astype(np.uint32)
        self.small = [1 if ("_gl000" in c or "chrM" in c) else 0 for c in oix.contigs]
        self.major = O.major_flags(oix.contigs, chrom_sizes)
        self.coff = [chrom_sizes.get(c, 0) for c in oix.contigs]
        self.bins = np.asarray(bin_starts, np.int64)
        self.reset()

    def reset(self, keep_search=False):
        # (keep_search: no look-ahead searches to keep here -- phase_map
        # searches synchronously)
        self.seen = set()
        self.total = self.dups = self.kept = 0
        self.error = 0

    def reserve_keys(self, keys):
        # (the library moves held keys into the larger set: smash_gpu.h)
        self.key_capacity = max(self.key_capacity, int(keys))

    def data_error(self, stream=None):
        return self.error

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

    def phase_map_ahead(self, d_reads, n_pairs, d_next, n_next):
        self.phase_map(d_reads, n_pairs)   # (no streams: the look-ahead is a no-op)

    def phase_search_ahead(self, d_reads, n_pairs):
        pass                               # (likewise)

    def phase_export(self, world, gbase):
        """smash_phase_export's layout: per owner, in pair order, 1-word
        headers {nk << 40 | word offset in the owner segment} and the keys'
        hit words (tid << 48 | pos0).  No pair index or hash travels: the
        receive order is the global order (dedup_owner relies on it), and
        the owner recomputes the hashes from the words."""
        first = {}
        for q, k in enumerate(self.kept_hits):
            if k is not None and tuple(k) not in first:
                first[tuple(k)] = q
        groups = [[] for _ in range(world)]
        for k, q in first.items():
            groups[(self.hashes[q][0] >> 1) % world].append((k, q))   # key_owner
        self.order = []
        rows, words, counts, wcounts = [], [], [], []
        for w in range(world):
            seg = []
            for k, q in sorted(groups[w], key=lambda t: t[1]):
                rows.append(((len(k) << 40) | len(seg),))
                seg += [to_i64((tid << 48) | pos) for tid, pos in k]
                self.order.append(q)
            words += seg
            counts.append(len(groups[w]))
            wcounts.append(len(seg))
        hdr = torch.tensor(rows, dtype=torch.int64).reshape(-1, 1)
        return (hdr, torch.tensor(words, dtype=torch.int64), np.array(counts, np.int64),
                np.array(wcounts, np.int64))

    def dedup_owner(self, d_recv, n_recv, d_recv_words, recv_counts, recv_words, d_flags):
        rows = d_recv[:n_recv].tolist()
        words = d_recv_words.tolist()
        hb = np.cumsum([0] + list(recv_counts))
        wb = np.cumsum([0] + list(recv_words))
        best = {}
        keys = []
        for j, (nw,) in enumerate(rows):
            nk, off = nw >> 40, nw & ((1 << 40) - 1)
            src = int(np.searchsorted(hb, j, side="right")) - 1
            a = int(wb[src]) + off
            k = tuple((to_u64(w) >> 48, to_u64(w) & 0xFFFFFFFFFFFF) for w in words[a:a + nk])
            keys.append(k)
            if k not in best:   # the first in receive order = global pair order
                best[k] = j
        flags = np.zeros(n_recv, np.uint8)
        for k, j in best.items():
            if k not in self.seen:
                flags[j] = 1
        self.seen.update(best.keys())
        if len(self.seen) > self.key_capacity:
            self.error = -4   # SMASH_ERR_NOMEM: the device's full set (k_owner_claim)
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
