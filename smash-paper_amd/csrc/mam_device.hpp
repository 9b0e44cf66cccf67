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
  const IdxT *SA;
  const IdxT *ISA;
  const uint8_t *L8;    // min(LCP,255)
  const uint8_t *U;     // per-position unique-length bytes (aux_build.hip)
  const uint64_t *KT;   // k-mer -> {lo, hi}
  uint64_t N, logN;
  int K;
};

template <class IdxT>
inline DevIndex<IdxT> make_dev_index(const smash_index *ix) {
  DevIndex<IdxT> x;
  x.T = ix->d_text;
  x.SA = static_cast<const IdxT *>(ix->d_sa);
  x.ISA = static_cast<const IdxT *>(ix->d_isa);
  x.L8 = ix->d_lcp8;
  x.U = ix->d_uniq;
  x.KT = ix->d_kmer;
  x.N = ix->N;
  x.logN = ix->logN;
  x.K = int(ix->kmer_k);
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
        const uint64_t lo = x.KT[2 * uint64_t(w)], hi = x.KT[2 * uint64_t(w) + 1];
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

}  // namespace smash
