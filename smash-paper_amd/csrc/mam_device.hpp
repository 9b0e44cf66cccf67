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
  uint64_t N, logN;
};

template <class IdxT>
inline DevIndex<IdxT> make_dev_index(const smash_index *ix) {
  DevIndex<IdxT> x;
  x.T = ix->d_text;
  x.SA = static_cast<const IdxT *>(ix->d_sa);
  x.ISA = static_cast<const IdxT *>(ix->d_isa);
  x.L8 = ix->d_lcp8;
  x.N = ix->N;
  x.logN = ix->logN;
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

// P: this lane's read (LDS), length L.
template <class IdxT>
__device__ void mam_read(const DevIndex<IdxT> &x, const uint8_t *P, uint32_t L,
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

}  // namespace smash
