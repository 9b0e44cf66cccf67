// smash-paper_amd/csrc/mam_device.hpp -- device-side MAM search (one lane).
//
// Semantics of longSA::MAM (longSA.cpp:503-536), traverse (:297-316),
// top_down_faster (:322-380), expand_link (longSA.h:158-174) and
// is_leftmaximal (:540-546); characters compare as signed chars widened to
// int64 like the reference.
#pragma once
#include "common.hpp"

namespace smash {

template <class IdxT>
struct DevIndex {
  const uint8_t *T;     // text (+64 zero bytes)
  IdxArr<IdxT> SA;      // positions only (the packed hints masked off)
  IdxArr<IdxT> ISA;
  const uint8_t *L8;    // min(LCP,255)
  const uint8_t *U;     // per-position unique-length bytes (aux_build.hip)
  const uint64_t *KT;   // k-mer -> {lo, hi} + (k+2)-mer presence bits (common.hpp)
  uint64_t N, logN;
  int K, B;
  uint64_t in_text[4];  // bytes that occur in the text
};

template <class IdxT>
inline DevIndex<IdxT> make_dev_index(const smash_index *ix) {
  DevIndex<IdxT> x;
  x.T = ix->d_text;
  x.SA = IdxArr<IdxT>{static_cast<const IdxT *>(ix->d_sa), ix->pos_mask};
  x.ISA = IdxArr<IdxT>{static_cast<const IdxT *>(ix->d_isa), ix->pos_mask};
  x.L8 = ix->d_lcp8;
  x.U = ix->d_uniq;
  x.KT = ix->d_kmer;
  x.N = ix->N;
  x.logN = ix->logN;
  x.K = int(ix->kmer_k);
  x.B = int(ix->bitmap_b);
  for (int k = 0; k < 4; ++k) x.in_text[k] = ix->in_text[k];
  return x;
}

struct MatchSink {
  uint64_t *out;
  uint32_t cap, n;
  __device__ void emit(uint64_t ref, uint64_t q, uint64_t len) {
    if (n < cap) out[n] = pack_match(ref, uint32_t(q), uint32_t(len));
    ++n;
  }
};

__device__ __forceinline__ int64_t sch(uint8_t c) { return int64_t(int8_t(c)); }

// top_down_faster: narrow [start,end] at depth i by character c.
template <class IdxT>
__device__ __forceinline__ bool td_faster(const DevIndex<IdxT> &x, int64_t c,
                                          uint64_t i, uint64_t &start,
                                          uint64_t &end) {
  uint64_t l, r, m, r2 = end, l2 = start;
  int64_t v;
  bool found = false;
  const int64_t cf = c - sch(x.T[uint64_t(x.SA[start]) + i]);
  const int64_t cl = c - sch(x.T[uint64_t(x.SA[end]) + i]);
  if (cf < 0) {
    l = start + 1;
    l2 = start;
  } else if (cl > 0) {
    l = end + 1;
    l2 = end;
  } else {
    l = start;
    r = end;
    if (cf == 0) {
      found = true;
      r2 = r;
    } else {
      while (r > l + 1) {
        m = (l + r) >> 1;
        v = c - sch(x.T[uint64_t(x.SA[m]) + i]);
        if (v <= 0) {
          if (!found && v == 0) {
            found = true;
            l2 = m;
            r2 = r;
          }
          r = m;
        } else {
          l = m;
        }
      }
      l = r;
    }
    if (!found) l2 = l - 1;
    if (cl == 0) {
      l2 = end;
    } else {
      while (r2 > l2 + 1) {
        m = (l2 + r2) >> 1;
        v = c - sch(x.T[uint64_t(x.SA[m]) + i]);
        if (v < 0) r2 = m;
        else l2 = m;
      }
    }
  }
  start = l;
  end = l2;
  return l <= l2;
}

template <class IdxT>
__device__ __forceinline__ bool expand_link(const DevIndex<IdxT> &x,
                                            uint64_t depth, uint64_t &start,
                                            uint64_t &end) {
  const uint64_t thresh = 2 * depth * x.logN;
  uint64_t exp = 0, s = start, e = end;
  while (uint64_t(x.L8[s]) >= depth) {
    if (++exp >= thresh) return false;
    --s;
  }
  while (e < x.N - 1 && uint64_t(x.L8[e + 1]) >= depth) {
    if (++exp >= thresh) return false;
    ++e;
  }
  start = s;
  end = e;
  return true;
}

// P: this lane's read (LDS), length L.  The reference's probe sequence,
// statement by statement (SMASH_MODE_MAM_PLAIN).
template <class IdxT>
__device__ void mam_read_plain(const DevIndex<IdxT> &x, const uint8_t *P, uint32_t L,
                               uint32_t min_len, MatchSink &sink) {
  const uint64_t N = x.N;
  uint64_t depth = 0, start = 0, end = N - 1;
  uint64_t prefix = 0;
  while (prefix < L) {
    // traverse(P, prefix, cur, P.length())
    if (depth < L) {
      while (prefix + depth < L) {
        uint64_t s = start, e = end;
        if (!td_faster(x, sch(P[prefix + depth]), depth, s, e)) break;
        depth += 1;
        start = s;
        end = e;
        if (depth == L) break;
      }
    }
    if (depth <= 1) {
      depth = 0;
      start = 0;
      end = N - 1;
      ++prefix;
      continue;
    }
    if (end == start && depth >= min_len) {
      const uint64_t p2 = x.SA[start];
      const bool lm = (prefix == 0 || p2 == 0) ? true
                      : (sch(P[prefix - 1]) != sch(x.T[p2 - 1]));
      if (lm) sink.emit(p2, prefix, depth);
    }
    do {
      depth = depth - 1;
      start = x.ISA[uint64_t(x.SA[start]) + 1];
      end = x.ISA[uint64_t(x.SA[end]) + 1];
      ++prefix;
      if (depth == 0 || !expand_link(x, depth, start, end)) {
        depth = 0;
        start = 0;
        end = N - 1;
        break;
      }
    } while (depth > 0 && end == start);
  }
}

// ---------------------------------------------------------------------------
// Accelerated MAM (SMASH_MODE_MAM): the same state sequence at every point
// where the reference can emit or reset, reached with fewer dependent loads.
//  (A) singleton intervals extend by comparing P with T[pos + depth ...]
//      8 bytes per load (top_down_faster on [s,s] is exactly that compare);
//  (B) the suffix-link chain of a singleton (do-while, longSA.cpp:523-534)
//      keeps the interval a singleton while U[pos+j] < depth-j; the first j
//      where that fails is found by a sequential scan of U (8 bytes/load);
//      only there ISA[pos+j] and the real expand_link (threshold included)
//      run.  SA[ISA[y]] = y saves the SA loads of the chain.
//  (C) a descent from the root with k ACGT characters available starts at
//      depth k from KT[w]; an absent k-mer falls back to top_down_faster.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t load8(const uint8_t *T, uint64_t a) {
  const uint64_t *w = reinterpret_cast<const uint64_t *>(T);
  const uint64_t q = a >> 3, sh = (a & 7) * 8;
  const uint64_t lo = w[q];
  if (sh == 0) return lo;
  return (lo >> sh) | (w[q + 1] << (64 - sh));
}

__device__ __forceinline__ int acgt_code(uint8_t c) {
  return c == 'a' ? 0 : c == 'c' ? 1 : c == 'g' ? 2 : c == 't' ? 3 : -1;
}

template <class IdxT>
__device__ void mam_read(const DevIndex<IdxT> &x, const uint8_t *P, uint32_t L,
                         uint32_t min_len, MatchSink &sink) {
  const uint64_t N = x.N;
  uint64_t depth = 0, start = 0, end = N - 1;
  uint64_t prefix = 0;
  uint64_t pos = 0;            // SA[start] when start == end and known
  bool have_pos = false;
  while (prefix < L) {
    // ---- traverse(P, prefix, cur, L) ----
    if (depth == 0 && prefix + uint64_t(x.K) <= L) {   // (C) from the root
      uint32_t w = 0;
      bool ok = true;
      for (int k = 0; k < x.K; ++k) {
        const int v = acgt_code(P[prefix + k]);
        ok = ok && v >= 0;
        w = (w << 2) | uint32_t(v & 3);
      }
      if (ok) {
        const uint64_t lo = x.KT[2 * uint64_t(w)] & kKtMask, hi = x.KT[2 * uint64_t(w) + 1] & kKtMask;
        if (lo <= hi) {
          depth = uint64_t(x.K);
          start = lo;
          end = hi;
          have_pos = false;
        }
      }
    }
    if (depth < L) {
      while (prefix + depth < L) {
        if (start == end) {                              // (A)
          if (!have_pos) { pos = x.SA[start]; have_pos = true; }
          while (prefix + depth < L) {
            const uint64_t t = load8(x.T, pos + depth);
            const uint64_t rem = L - prefix - depth;
            const uint32_t lim = rem < 8 ? uint32_t(rem) : 8u;
            uint32_t k = 0;
            while (k < lim && P[prefix + depth + k] == uint8_t(t >> (8 * k))) ++k;
            depth += k;
            if (k < lim) break;
          }
          break;
        }
        uint64_t s = start, e = end;
        if (!td_faster(x, sch(P[prefix + depth]), depth, s, e)) break;
        depth += 1;
        start = s;
        end = e;
        have_pos = false;
        if (depth == L) break;
      }
    }
    if (depth <= 1) {
      depth = 0; start = 0; end = N - 1; have_pos = false;
      ++prefix;
      continue;
    }
    if (end == start) {
      if (!have_pos) { pos = x.SA[start]; have_pos = true; }
      if (depth >= min_len) {
        const bool lm = (prefix == 0 || pos == 0) ? true
                        : (sch(P[prefix - 1]) != sch(x.T[pos - 1]));
        if (lm) sink.emit(pos, prefix, depth);
      }
      // (B) singleton suffix-link chain
      const uint64_t d = depth;
      uint64_t j = 1;
      bool hit = false;
      while (j < d) {
        const uint64_t u = load8(x.U, pos + j);
        const uint64_t rem = d - j;
        const uint32_t lim = rem < 8 ? uint32_t(rem) : 8u;
        uint32_t k = 0;
        while (k < lim && uint64_t(uint8_t(u >> (8 * k))) < d - j - k) ++k;
        if (k < lim) { j += k; hit = true; break; }
        j += lim;
      }
      prefix += j;
      if (!hit) {                 // depth reached 0: reset (longSA.cpp:528)
        depth = 0; start = 0; end = N - 1; have_pos = false;
        continue;
      }
      depth = d - j;
      start = end = x.ISA[pos + j];
      have_pos = false;
      if (!expand_link(x, depth, start, end)) {
        depth = 0; start = 0; end = N - 1;
      } else if (start == end) {  // cannot happen (U said the interval widens)
        pos = pos + j;
        have_pos = true;
      }
      continue;
    }
    // non-singleton: one step of the do-while (the interval stays wider)
    depth = depth - 1;
    start = x.ISA[uint64_t(x.SA[start]) + 1];
    end = x.ISA[uint64_t(x.SA[end]) + 1];
    ++prefix;
    have_pos = false;
    if (depth == 0 || !expand_link(x, depth, start, end)) {
      depth = 0; start = 0; end = N - 1;
    }
  }
}

// ---------------------------------------------------------------------------
// v3 (SMASH_MODE_MAM): the MAM output is a function of the per-position
// matching statistics -- p emits iff ms(p) >= min_len, the ms(p)-prefix occurs
// once, and p is left-maximal -- so the streaming state may be dropped at any
// prefix that provably cannot emit.  On top of (A), (B), (C):
//  (F) while the state is shallow (depth < min_len), a prefix whose min_len
//      window holds a byte absent from the text, or whose first/last B-mer is
//      absent from the presence bitmap, cannot reach min_len: skip it with a
//      reset (the reference would walk the suffix links down instead);
//  (S) an interval of <= 32 suffixes finishes its traverse by comparing
//      every candidate with the read (independent loads instead of the
//      2*log2(n) dependent probes per character of top_down_faster); the
//      suffixes sharing the longest match are the traverse's final interval.
// ---------------------------------------------------------------------------
constexpr int kScan = 32;

// 8 read bytes at byte offset `off` of an LDS row (row 4-byte aligned and
// padded; bytes past the read are masked by the callers)
// (v_alignbyte_b32: the low dword of {hi, lo} >> 8 * (s & 3); the host
// emulation substitutes its own)
#ifndef SM_ALIGNBYTE
#define SM_ALIGNBYTE(hi, lo, s) __builtin_amdgcn_alignbyte(hi, lo, s)
#endif
__device__ __forceinline__ uint64_t lds_load8(const uint8_t *P, uint64_t off) {
  // three aligned words, two byte-aligns (no 64-bit shifts, no select on the
  // offset): the rows carry the third word's over-read
  const uint32_t *w = reinterpret_cast<const uint32_t *>(P);
  const uint32_t q = uint32_t(off) >> 2, s = uint32_t(off) & 3;
  const uint32_t w0 = w[q], w1 = w[q + 1], w2 = w[q + 2];
  return uint64_t(SM_ALIGNBYTE(w1, w0, s)) | (uint64_t(SM_ALIGNBYTE(w2, w1, s)) << 32);
}

// bytes of agreement of two 8-byte words, capped at lim (<= 8)
// (ctz with 64 for zero: v_ffbl pairs with no compare-and-select on the
// 64-bit difference; the host emulation substitutes its own)
#ifndef SM_CTZ64
#define SM_CTZ64(x) __builtin_ctzg(x, 64)
#endif
__device__ __forceinline__ uint32_t agree8(uint64_t a, uint64_t b, uint32_t lim) {
  const uint32_t k = uint32_t(SM_CTZ64(a ^ b)) >> 3;
  return k < lim ? k : lim;
}

template <class IdxT>
__device__ __forceinline__ bool in_text(const DevIndex<IdxT> &x, uint8_t b) {
  return (x.in_text[b >> 6] >> (b & 63)) & 1ull;
}

// lcp of P[off .. off+rem) with T[t ...]
template <class IdxT>
__device__ __forceinline__ uint64_t lcp_read_text(const DevIndex<IdxT> &x, const uint8_t *P,
                                                  uint64_t off, uint64_t rem, uint64_t t,
                                                  uint64_t first_word) {
  uint64_t l = 0;
  uint64_t tw = first_word;
  for (;;) {
    const uint32_t lim = rem - l < 8 ? uint32_t(rem - l) : 8u;
    const uint32_t k = agree8(tw, lds_load8(P, off + l), lim);
    l += k;
    if (k < 8 || l >= rem) return l;
    tw = load8(x.T, t + l);
  }
}

// (F): can P[p .. p+min_len) occur?  next_p: where to resume when not
template <class IdxT>
__device__ bool window_ok(const DevIndex<IdxT> &x, const uint8_t *P, uint64_t p,
                          uint32_t min_len, uint64_t &next_p) {
  next_p = p + 1;
  for (uint64_t k = p + min_len; k-- > p;)
    if (!in_text(x, P[k])) { next_p = k + 1; return false; }
  const int B = x.B;
  if (B <= 0 || uint32_t(B) > min_len) return true;
  const uint64_t mask = (1ull << (2 * B)) - 1;
  uint64_t c0 = 0, c1 = 0;
  const uint64_t q1 = p + min_len - B;
  for (int k = 0; k < B; ++k) {
    const int v0 = acgt_code(P[p + k]), v1 = acgt_code(P[q1 + k]);
    if (v0 < 0 || v1 < 0) return true;     // no bitmap verdict
    c0 = ((c0 << 2) | uint64_t(v0)) & mask;
    c1 = ((c1 << 2) | uint64_t(v1)) & mask;
  }
  return kt_bmer_present(x.KT, c0) && kt_bmer_present(x.KT, c1);
}

// (S): final traverse state over a small interval
template <class IdxT>
__device__ void scan_small(const DevIndex<IdxT> &x, const uint8_t *P, uint64_t L,
                           uint64_t p, uint64_t &depth, uint64_t &start, uint64_t &end,
                           uint64_t &pos) {
  const uint64_t d = depth, rem = L - p - d;
  const uint64_t pw = lds_load8(P, p + d);
  const uint32_t lim0 = rem < 8 ? uint32_t(rem) : 8u;
  int64_t best = -1;
  uint64_t bl = start, bh = start, bpos = 0;
  for (uint64_t m0 = start; m0 <= end; m0 += 4) {
    uint64_t sp[4], tw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) sp[k] = m0 + k <= end ? uint64_t(x.SA[m0 + k]) : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) tw[k] = m0 + k <= end ? load8(x.T, sp[k] + d) : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (m0 + k > end) break;
      uint64_t l = agree8(tw[k], pw, lim0);
      if (l == 8 && rem > 8)
        l = 8 + lcp_read_text(x, P, p + d + 8, rem - 8, sp[k] + d + 8, load8(x.T, sp[k] + d + 8));
      if (int64_t(l) > best) { best = int64_t(l); bl = bh = m0 + k; bpos = sp[k]; }
      else if (int64_t(l) == best) bh = m0 + k;
    }
  }
  depth = d + uint64_t(best);
  start = bl;
  end = bh;
  pos = bpos;
}

template <class IdxT>
__device__ void mam_read_v3(const DevIndex<IdxT> &x, const uint8_t *P, uint32_t L,
                            uint32_t min_len, MatchSink &sink) {
  const uint64_t N = x.N;
  uint64_t depth = 0, start = 0, end = N - 1;
  uint64_t prefix = 0, pos = 0;
  bool have_pos = false;
  while (prefix < L) {
    if (depth < min_len) {                                   // (F)
      if (prefix + min_len > L) break;
      uint64_t nxt;
      if (!window_ok(x, P, prefix, min_len, nxt)) {
        depth = 0; start = 0; end = N - 1; have_pos = false;
        prefix = nxt;
        continue;
      }
    }
    if (depth == 0 && prefix + uint64_t(x.K) <= L) {         // (C)
      uint32_t w = 0;
      bool ok = true;
      for (int k = 0; k < x.K; ++k) {
        const int v = acgt_code(P[prefix + k]);
        ok = ok && v >= 0;
        w = (w << 2) | uint32_t(v & 3);
      }
      if (ok) {
        const uint64_t lo = x.KT[2 * uint64_t(w)] & kKtMask, hi = x.KT[2 * uint64_t(w) + 1] & kKtMask;
        if (lo <= hi) { depth = uint64_t(x.K); start = lo; end = hi; have_pos = false; }
      }
    }
    if (depth < L) {
      while (prefix + depth < L) {
        if (start == end) {                                  // (A)
          if (!have_pos) { pos = x.SA[start]; have_pos = true; }
          depth += lcp_read_text(x, P, prefix + depth, L - prefix - depth, pos + depth,
                                 load8(x.T, pos + depth));
          break;
        }
        if (end - start + 1 <= uint64_t(kScan)) {           // (S)
          scan_small(x, P, L, prefix, depth, start, end, pos);
          have_pos = start == end;
          break;
        }
        uint64_t s = start, e = end;
        if (!td_faster(x, sch(P[prefix + depth]), depth, s, e)) break;
        depth += 1;
        start = s;
        end = e;
        have_pos = false;
        if (depth == L) break;
      }
    }
    if (depth <= 1) {
      depth = 0; start = 0; end = N - 1; have_pos = false;
      ++prefix;
      continue;
    }
    if (end == start) {
      if (!have_pos) { pos = x.SA[start]; have_pos = true; }
      if (depth >= min_len) {
        const bool lm = (prefix == 0 || pos == 0) ? true
                        : (sch(P[prefix - 1]) != sch(x.T[pos - 1]));
        if (lm) sink.emit(pos, prefix, depth);
      }
      const uint64_t d = depth;                              // (B)
      uint64_t j = 1;
      bool hit = false;
      while (j < d) {
        const uint64_t u = load8(x.U, pos + j);
        const uint64_t rem = d - j;
        const uint32_t lim = rem < 8 ? uint32_t(rem) : 8u;
        uint32_t k = 0;
        while (k < lim && uint64_t(uint8_t(u >> (8 * k))) < d - j - k) ++k;
        if (k < lim) { j += k; hit = true; break; }
        j += lim;
      }
      prefix += j;
      if (!hit) { depth = 0; start = 0; end = N - 1; have_pos = false; continue; }
      depth = d - j;
      start = end = x.ISA[pos + j];
      have_pos = false;
      if (!expand_link(x, depth, start, end)) { depth = 0; start = 0; end = N - 1; }
      continue;
    }
    depth = depth - 1;
    start = x.ISA[uint64_t(x.SA[start]) + 1];
    end = x.ISA[uint64_t(x.SA[end]) + 1];
    ++prefix;
    have_pos = false;
    if (depth == 0 || !expand_link(x, depth, start, end)) { depth = 0; start = 0; end = N - 1; }
  }
}

}  // namespace smash
