// smash-paper_amd/csrc/mem.hip -- the other two search modes of memsam on
// gfx950: -maxmatch (MEM) and -mum (MUM).
//
// MEM replaces longSA::MEM / findMEM / collectMEMs / find_Lmaximal
// (longSA.cpp:395-490, 587-590) with suffixlink (:383-392) and expand_link
// (longSA.h:158-174).  One lane runs one read, statement by statement, so the
// match sequence (order included) is the reference's.  Two accelerations
// change no probe outcome:
//  (A) a singleton interval extends by comparing 8 read bytes with 8 text
//      bytes per load (top_down_faster on [s, s] is that byte compare);
//  (C) a descent from the ROOT interval with k ACGT characters available and
//      k <= the traverse limit starts at depth k from the k-mer table.
// LCP is read exactly (u8 + the sorted overflow table, vec_uchar longSA.h:
// 34-39): unlike MAM, findMEM keeps the max-match interval even when its
// suffix link fails (longSA.cpp:423 ignores the result), and collectMEMs
// then compares depths with LCP values that can exceed 255.
//
// MUM replaces longSA::MUM (longSA.cpp:549-585): the MAM matches of a read
// (at most one per prefix, so at most L) sorted by (ref asc, len desc) and
// filtered as cleanMUMcand does.  Matches tying on (ref, len) are dropped
// together, so the unspecified order of std::sort among them never shows.
#include "common.hpp"
#include "mam_device.hpp"

#include <hipcub/hipcub.hpp>

#include <cstdlib>
#include <cstring>

namespace smash {
namespace {

template <class IdxT>
struct MemIx {
  DevIndex<IdxT> x;
  const uint64_t *ovf;   // {idx, val} for LCP >= 255, sorted by idx
  uint64_t n_ovf;
  bool pk;               // packed SA words: the BWT character in bits 33-35
};

template <class IdxT>
__device__ __forceinline__ uint64_t lcp_at(const MemIx<IdxT> &m, uint64_t i) {
  const uint32_t v = m.x.L8[i];
  if (v < 255) return v;
  uint64_t lo = 0, hi = m.n_ovf;   // lower_bound (longSA.h:36)
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (m.ovf[2 * mid] < i) lo = mid + 1;
    else hi = mid;
  }
  return lo < m.n_ovf ? m.ovf[2 * lo + 1] : 255;
}

struct Ival {
  uint64_t depth, start, end;
};

// LCP runs for a depth d <= 255, where the u8 byte decides LCP >= d exactly
// (L8 = min(LCP, 255)): no overflow-table bisection, 16 bytes per load.  A
// repeat family's suffixes share more than 255 characters, so the exact
// lcp_at of every step of its run cost a ~30-load bisection each.
//   run_down: the j = s, s - 1, ... (at most `lim`) with L8[j] >= d, counted
//   run_up:   the j = s, s + 1, ... < N (at most `lim`) with L8[j] >= d
// (d >= 1 and L8[0] = 0 stop run_down at 0; the array has 64 pad bytes)
__host__ __device__ __forceinline__ uint32_t dword_sel(const uint4 &v, uint32_t i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}
__host__ __device__ __forceinline__ uint64_t run_down(const uint8_t *L8, uint64_t s, uint32_t d,
                                             uint64_t lim) {
  uint64_t n = 0;
  while (n < lim) {
    const uint64_t j = s - n, base = j & ~15ull;
    const uint4 v = *reinterpret_cast<const uint4 *>(L8 + base);
    for (int o = int(j - base); o >= 0; --o) {
      if (((dword_sel(v, uint32_t(o) >> 2) >> (8 * (o & 3))) & 0xFF) < d || n >= lim) return n;
      ++n;
    }
  }
  return n;
}
__host__ __device__ __forceinline__ uint64_t run_up(const uint8_t *L8, uint64_t s, uint64_t N, uint32_t d,
                                           uint64_t lim) {
  uint64_t n = 0;
  if (s >= N) return 0;
  if (lim > N - s) lim = N - s;
  while (n < lim) {
    const uint64_t j = s + n, base = j & ~15ull;
    const uint4 v = *reinterpret_cast<const uint4 *>(L8 + base);
    for (uint32_t o = uint32_t(j - base); o < 16; ++o) {
      if (((dword_sel(v, o >> 2) >> (8 * (o & 3))) & 0xFF) < d || n >= lim) return n;
      ++n;
    }
  }
  return n;
}

// expand_link (longSA.h:158-174) over the exact LCP.  It fails iff the two
// runs together reach thresh (each step counts, left run first): for
// depth <= 255 both runs come from run_down / run_up, capped there
template <class IdxT>
__device__ bool expand_link_x(const MemIx<IdxT> &m, Ival &l) {
  const uint64_t thresh = 2 * l.depth * m.x.logN;
  if (l.depth <= 255) {
    const uint32_t d = uint32_t(l.depth);
    const uint64_t a = run_down(m.x.L8, l.start, d, thresh < l.start + 1 ? thresh : l.start + 1);
    if (a >= thresh) return false;
    const uint64_t b = run_up(m.x.L8, l.end + 1, m.x.N, d, thresh - a);
    if (a + b >= thresh) return false;
    l.start -= a;
    l.end += b;
    return true;
  }
  uint64_t exp = 0, s = l.start, e = l.end;
  while (lcp_at(m, s) >= l.depth) {
    if (++exp >= thresh) return false;
    --s;
  }
  while (e < m.x.N - 1 && lcp_at(m, e + 1) >= l.depth) {
    if (++exp >= thresh) return false;
    ++e;
  }
  l.start = s;
  l.end = e;
  return true;
}

// suffixlink (longSA.cpp:383-392)
template <class IdxT>
__device__ bool suffixlink_x(const MemIx<IdxT> &m, Ival &v) {
  if (v.depth <= 1) {
    v.depth = 0;
    return false;
  }
  --v.depth;
  v.start = m.x.ISA[uint64_t(m.x.SA[v.start]) + 1];
  v.end = m.x.ISA[uint64_t(m.x.SA[v.end]) + 1];
  return expand_link_x(m, v);
}

// traverse (longSA.cpp:297-316) with (A) and (C)
template <class IdxT>
__device__ void traverse_x(const MemIx<IdxT> &m, const uint8_t *P, uint64_t L, uint64_t prefix,
                           Ival &cur, uint64_t limit) {
  const DevIndex<IdxT> &x = m.x;
  if (cur.depth >= limit) return;
  if (cur.depth == 0 && cur.start == 0 && cur.end == x.N - 1 && x.K > 0 &&
      uint64_t(x.K) <= limit && prefix + uint64_t(x.K) <= L) {   // (C)
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
        cur.depth = uint64_t(x.K);
        cur.start = lo;
        cur.end = hi;
        if (cur.depth == limit) return;
      }
    }
  }
  while (prefix + cur.depth < L) {
    if (cur.start == cur.end) {                                   // (A)
      const uint64_t pos = x.SA[cur.start];
      while (prefix + cur.depth < L && cur.depth < limit) {
        const uint64_t rem_r = L - prefix - cur.depth, rem_l = limit - cur.depth;
        const uint64_t rem = rem_r < rem_l ? rem_r : rem_l;
        const uint32_t lim = rem < 8 ? uint32_t(rem) : 8u;
        const uint32_t k = agree8(load8(x.T, pos + cur.depth), lds_load8(P, prefix + cur.depth), lim);
        cur.depth += k;
        if (k < lim) break;
      }
      return;
    }
    uint64_t s = cur.start, e = cur.end;
    if (!td_faster(x, sch(P[prefix + cur.depth]), cur.depth, s, e)) return;
    cur.depth += 1;
    cur.start = s;
    cur.end = e;
    if (cur.depth == limit) return;
  }
}

// A collectMEMs call over a large interval, left to k_mem_jobs (a wave per
// call, its runs and left-maximality checks 64 ranks at a time): in SIMT a
// lane walking a repeat family's million suffixes holds its whole wave, the
// other 63 lanes' next reads included, for the walk.  The lane leaves a hole
// in its read's records: `inl` records of its own came before it, hole h of
// the read (k_mem_fix places the records around the holes afterwards).
struct MemJob {
  uint64_t r;                 // read
  uint32_t prefix, inl, h;
  uint32_t pb;                // P[prefix - 1] (prefix > 0)
  uint64_t md, ms, me;        // mli {depth, start, end}
  uint64_t xd, xs, xe;        // xmi
};

struct MemSink {
  uint4 *out;
  uint32_t cap, n;
  // deferral (jobs == nullptr: every collectMEMs inline)
  MemJob *jobs;
  unsigned long long *n_jobs;
  uint64_t job_cap, defer, r;
  uint32_t holes;
  __device__ void emit(uint64_t ref, uint64_t q, uint64_t len) {
    if (n < cap)
      out[n] = make_uint4(uint32_t(ref), uint32_t(ref >> 32), uint32_t(q), uint32_t(len));
    ++n;
  }
};

// find_Lmaximal's test (longSA.cpp:438-457) for the suffix at x whose SA
// word is `raw`: a packed word with tag 0..3 names T[x - 1] (a c g t), so
// no text byte is loaded for it (oracle orc_mem_dev counts the same)
template <class IdxT>
__device__ __forceinline__ bool left_max(const MemIx<IdxT> &m, uint64_t prefix, uint32_t pb,
                                         uint64_t raw, uint64_t x) {
  if (prefix == 0 || x == 0) return true;
  if (m.pk) {
    const uint32_t tag = uint32_t(raw >> kPkPosBits) & 7u;
    if (tag < 4) return pb != ((0x74676361u >> (8 * tag)) & 0xFFu);
  }
  return pb != m.x.T[x - 1];
}

// find_Lmaximal (longSA.cpp:438-457) of the suffix at SA rank `rank`
template <class IdxT>
__device__ __forceinline__ void find_lmax(const MemIx<IdxT> &m, const uint8_t *P, uint32_t min_len,
                                          uint64_t prefix, uint64_t rank, uint64_t len, MemSink &s) {
  const uint64_t raw = uint64_t(m.x.SA.p[rank]), x = raw & m.x.SA.mask;
  if (left_max(m, prefix, prefix ? P[prefix - 1] : 0u, raw, x) && len >= min_len) s.emit(x, prefix, len);
}

// find_Lmaximal of `count` ranks in order (first, first - 1, ... when down,
// else first, first + 1, ...) at one length, 8 at a time: their SA elements
// and text bytes are independent loads, all in flight before the first
// emission (an interval of a repeat family holds millions of suffixes, and
// one lane walks it); emissions stay in the given order
template <class IdxT>
__device__ void lmax_ranks(const MemIx<IdxT> &m, const uint8_t *P, uint32_t min_len,
                           uint64_t prefix, uint64_t first, bool down, uint64_t count,
                           uint64_t len, MemSink &s) {
  if (len < min_len) return;                 // find_lmax emits nothing
  const uint32_t pb = prefix ? P[prefix - 1] : 0u;
  uint64_t k0 = 0;
  for (; k0 + 8 <= count; k0 += 8) {
    uint64_t w[8];
    bool e[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = uint64_t(m.x.SA.p[down ? first - k0 - k : first + k0 + k]);
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = left_max(m, prefix, pb, w[k], w[k] & m.x.SA.mask);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (e[k]) s.emit(w[k] & m.x.SA.mask, prefix, len);
  }
  for (; k0 < count; ++k0) find_lmax(m, P, min_len, prefix, down ? first - k0 : first + k0, len, s);
}

// collectMEMs (longSA.cpp:461-490); xmi by value as in the reference
template <class IdxT>
__device__ void collect_mems(const MemIx<IdxT> &m, const uint8_t *P, uint32_t min_len,
                             uint64_t prefix, const Ival &mli, Ival xmi, MemSink &s) {
  const uint64_t N = m.x.N;
  // every rank of mli is visited (xmi grows to mli): a large one goes to a job
  if (s.jobs && mli.end >= mli.start && mli.end - mli.start + 1 >= s.defer && s.holes < 0xFFFFu) {
    const unsigned long long j = atomicAdd(s.n_jobs, 1ull);
    if (j < s.job_cap) {
      MemJob &J = s.jobs[j];
      J.r = s.r; J.prefix = uint32_t(prefix); J.inl = s.n; J.h = s.holes;
      J.pb = prefix ? P[prefix - 1] : 0u;
      J.md = mli.depth; J.ms = mli.start; J.me = mli.end;
      J.xd = xmi.depth; J.xs = xmi.start; J.xe = xmi.end;
      ++s.holes;
      return;
    }
    // (the job list is full: inline, as without deferral)
  }
  lmax_ranks(m, P, min_len, prefix, xmi.start, false,
             xmi.end >= xmi.start ? xmi.end - xmi.start + 1 : 0, xmi.depth, s);
  if (mli.start == xmi.start && mli.end == xmi.end) return;
  while (xmi.depth >= mli.depth) {
    if (xmi.end + 1 < N) {
      const uint64_t a = lcp_at(m, xmi.start), b = lcp_at(m, xmi.end + 1);
      xmi.depth = a > b ? a : b;
    } else {
      xmi.depth = lcp_at(m, xmi.start);
    }
    if (xmi.depth >= mli.depth && xmi.depth <= 255) {
      // the two loops below as runs of the u8 LCP (run_down / run_up), the
      // left run's ranks emitted downwards, then the right run's upwards
      const uint32_t d = uint32_t(xmi.depth);
      const uint64_t nl = run_down(m.x.L8, xmi.start, d, xmi.start + 1);
      lmax_ranks(m, P, min_len, prefix, xmi.start - 1, true, nl, xmi.depth, s);
      xmi.start -= nl;
      const uint64_t nr = run_up(m.x.L8, xmi.end + 1, N, d, N);
      lmax_ranks(m, P, min_len, prefix, xmi.end + 1, false, nr, xmi.depth, s);
      xmi.end += nr;
    } else if (xmi.depth >= mli.depth) {
      while (lcp_at(m, xmi.start) >= xmi.depth) {
        --xmi.start;
        find_lmax(m, P, min_len, prefix, xmi.start, xmi.depth, s);
      }
      while (xmi.end + 1 < N && lcp_at(m, xmi.end + 1) >= xmi.depth) {
        ++xmi.end;
        find_lmax(m, P, min_len, prefix, xmi.end, xmi.depth, s);
      }
    }
  }
}

// findMEM (longSA.cpp:395-431)
template <class IdxT>
__device__ void mem_read(const MemIx<IdxT> &m, const uint8_t *P, uint32_t L, uint32_t min_len,
                         MemSink &s) {
  const uint64_t N = m.x.N;
  const Ival root{0, 0, N - 1};
  uint64_t prefix = 1;                     // longSA.cpp:398 (sic)
  Ival mli = root, xmi = root;
  while (prefix <= L) {
    traverse_x(m, P, L, prefix, mli, min_len);
    if (mli.depth > xmi.depth) xmi = mli;
    if (mli.depth <= 1) {
      mli = root;
      xmi = root;
      ++prefix;
      continue;
    }
    if (mli.depth >= min_len) {
      traverse_x(m, P, L, prefix, xmi, L);
      collect_mems(m, P, min_len, prefix, mli, xmi, s);
      ++prefix;
      if (!suffixlink_x(m, mli)) {
        mli = root;
        xmi = root;
        continue;
      }
      suffixlink_x(m, xmi);                // result ignored (longSA.cpp:423)
    } else {
      ++prefix;
      if (!suffixlink_x(m, mli)) {
        mli = root;
        xmi = root;
        continue;
      }
      xmi = mli;
    }
  }
}

// Persistent lanes pulling reads from a device work counter (a repetitive
// read only delays its own lane); the read is copied into the lane's LDS row.
template <class IdxT, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_mem(MemIx<IdxT> m, const uint8_t *__restrict__ seqs,
                                               uint64_t stride, const uint16_t *__restrict__ lens,
                                               uint32_t len0, uint64_t n_reads, uint32_t min_len,
                                               uint4 *__restrict__ out, uint32_t cap,
                                               uint32_t *__restrict__ n_out, uint32_t row,
                                               unsigned long long *work, MemJob *jobs,
                                               unsigned long long *n_jobs, uint64_t job_cap,
                                               uint64_t defer, uint32_t *__restrict__ n_holes) {
  extern __shared__ uint8_t lds[];
  uint8_t *P = lds + threadIdx.x * row;
  for (;;) {
    const uint64_t r = atomicAdd(work, 1ull);
    if (r >= n_reads) break;
    const uint32_t L = lens ? lens[r] : len0;
    const uint8_t *src = seqs + r * stride;
    for (uint32_t k = 0; k < row; ++k) P[k] = k < L ? src[k] : 0;
    MemSink s{out + r * cap, cap, 0, jobs, n_jobs, job_cap, defer, r, 0};
    mem_read(m, P, L, min_len, s);
    n_out[r] = s.n;                 // (the holes' records are added by k_mem_fix)
    if (n_holes) n_holes[r] = s.holes;
  }
}

// ---- deferred collectMEMs (MemJob): one wave per job ----------------------
// the lane's 64-bit mask of the lanes below it
__device__ __forceinline__ uint64_t lanes_below() {
  const uint32_t lane = threadIdx.x & 63;
  return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// positions s, s - 1, ... with L8 >= d (d in 1..255), counted by the wave:
// lane l tests positions s - n - 16 l - t, t = 0..15 (below 0: a stop)
__device__ uint64_t wave_run_down(const uint8_t *L8, uint64_t s, uint32_t d) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t n = 0;; n += 1024) {
    uint32_t stop = 16;
    for (uint32_t t = 0; t < 16; ++t) {
      const uint64_t k = n + 16ull * lane + t;
      if (k > s || L8[s - k] < d) { stop = t; break; }
    }
    const uint64_t b = __ballot(stop < 16);
    if (b) {
      const int fl = __builtin_ctzll(b);
      return n + 16ull * uint64_t(fl) + uint64_t(__shfl(int(stop), fl, 64));
    }
  }
}
// positions s, s + 1, ... < N with L8 >= d, counted by the wave
__device__ uint64_t wave_run_up(const uint8_t *L8, uint64_t s, uint64_t N, uint32_t d) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t n = 0;; n += 1024) {
    uint32_t stop = 16;
    for (uint32_t t = 0; t < 16; ++t) {
      const uint64_t q = s + n + 16ull * lane + t;
      if (q >= N || L8[q] < d) { stop = t; break; }
    }
    const uint64_t b = __ballot(stop < 16);
    if (b) {
      const int fl = __builtin_ctzll(b);
      return n + 16ull * uint64_t(fl) + uint64_t(__shfl(int(stop), fl, 64));
    }
  }
}

// COUNT (WRITE = false): the records each job emits -> E[j].  WRITE: a job
// whose first record lands below cap (base[j], k_mem_fix) writes them, in
// the order collectMEMs emits them, until cap.  Control flow is wave-uniform.
template <class IdxT, bool WRITE>
__global__ __launch_bounds__(256) void k_mem_jobs(MemIx<IdxT> m, const MemJob *__restrict__ jobs,
                                                  const unsigned long long *n_jobs, uint64_t job_cap,
                                                  uint32_t min_len, uint4 *__restrict__ out,
                                                  uint32_t cap, uint32_t *__restrict__ E,
                                                  const uint32_t *__restrict__ base) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t nj = *n_jobs < job_cap ? *n_jobs : job_cap;
  const uint64_t waves = uint64_t(gridDim.x) * (blockDim.x / 64);
  const uint64_t N = m.x.N;
  const uint64_t below = lanes_below();
  for (uint64_t j = uint64_t(blockIdx.x) * (blockDim.x / 64) + threadIdx.x / 64; j < nj; j += waves) {
    const MemJob J = jobs[j];
    uint64_t pos = WRITE ? base[j] : 0;
    if (WRITE && pos >= cap) continue;
    uint4 *o = out + J.r * cap;
    uint64_t emitted = 0;
    bool full = false;
    // find_Lmaximal of `count` ranks (first, first -/+ 1, ...) at length len
    auto ranks = [&](uint64_t first, bool down, uint64_t count, uint64_t len) {
      if (len < min_len || full) return;
      for (uint64_t k0 = 0; k0 < count; k0 += 64) {
        const uint64_t k = k0 + lane;
        bool e = false;
        uint64_t x = 0;
        if (k < count) {
          const uint64_t w = uint64_t(m.x.SA.p[down ? first - k : first + k]);
          x = w & m.x.SA.mask;
          e = left_max(m, J.prefix, J.pb, w, x);
        }
        const uint64_t b = __ballot(e);
        if (WRITE) {
          const uint64_t p = pos + uint64_t(__popcll(b & below));
          if (e && p < cap)
            o[p] = make_uint4(uint32_t(x), uint32_t(x >> 32), J.prefix, uint32_t(len));
        }
        pos += uint64_t(__popcll(b));
        emitted += uint64_t(__popcll(b));
        if (WRITE && pos >= cap) { full = true; return; }
      }
    };
    uint64_t xd = J.xd, xs = J.xs, xe = J.xe;
    ranks(xs, false, xe >= xs ? xe - xs + 1 : 0, xd);
    if (!(J.ms == xs && J.me == xe)) {
      while (xd >= J.md && !full) {
        if (xe + 1 < N) {
          const uint64_t a = lcp_at(m, xs), b = lcp_at(m, xe + 1);
          xd = a > b ? a : b;
        } else {
          xd = lcp_at(m, xs);
        }
        if (xd < J.md) break;
        if (xd <= 255) {
          const uint64_t nl = wave_run_down(m.x.L8, xs, uint32_t(xd));
          ranks(xs - 1, true, nl, xd);
          xs -= nl;
          const uint64_t nr = wave_run_up(m.x.L8, xe + 1, N, uint32_t(xd));
          ranks(xe + 1, false, nr, xd);
          xe += nr;
        } else {
          while (!full && lcp_at(m, xs) >= xd) { --xs; ranks(xs, false, 1, xd); }
          while (!full && xe + 1 < N && lcp_at(m, xe + 1) >= xd) { ++xe; ranks(xe, false, 1, xd); }
        }
      }
    }
    if (!WRITE && lane == 0) E[j] = uint32_t(emitted < 0xFFFFFFFFull ? emitted : 0xFFFFFFFFull);
  }
}

// job j -> slot off[r] + h: the read's jobs in hole order
__global__ void k_job_slots(const MemJob *__restrict__ jobs, const unsigned long long *n_jobs,
                            uint64_t job_cap, const uint32_t *__restrict__ off,
                            uint32_t *__restrict__ slot) {
  const uint64_t nj = *n_jobs < job_cap ? *n_jobs : job_cap;
  for (uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < nj;
       j += uint64_t(gridDim.x) * blockDim.x)
    slot[off[jobs[j].r] + jobs[j].h] = uint32_t(j);
}

// a read with holes: each job's first record index (its own records before
// it + the earlier holes' records), the read's total, and its own records
// moved up past the holes (from the last: a record only moves up)
__global__ void k_mem_fix(const MemJob *__restrict__ jobs, const uint32_t *__restrict__ E,
                          const uint32_t *__restrict__ n_holes, const uint32_t *__restrict__ off,
                          const uint32_t *__restrict__ slot, uint64_t n_reads, uint4 *__restrict__ out,
                          uint32_t cap, uint32_t *__restrict__ n_out, uint32_t *__restrict__ base) {
  const uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= n_reads || n_holes[r] == 0) return;
  const uint32_t nh = n_holes[r], o = off[r], own = n_out[r];
  uint64_t acc = 0;
  for (uint32_t h = 0; h < nh; ++h) {
    const uint32_t j = slot[o + h];
    base[j] = uint32_t(jobs[j].inl + acc < 0xFFFFFFFFull ? jobs[j].inl + acc : 0xFFFFFFFFull);
    acc += E[j];
  }
  n_out[r] = uint32_t(own + acc < 0xFFFFFFFFull ? own + acc : 0xFFFFFFFFull);
  uint4 *row = out + r * cap;
  uint64_t sh = acc;
  int64_t hh = int64_t(nh) - 1;
  for (uint32_t k = own < cap ? own : cap; k-- > 0;) {
    while (hh >= 0 && jobs[slot[o + hh]].inl > k) { sh -= E[slot[o + hh]]; --hh; }
    if (sh && k + sh < cap) row[k + sh] = row[k];
  }
}

// by_ref (longSA.cpp:492-499): ref ascending, then len descending
__device__ __forceinline__ bool by_ref_less(uint64_t a, uint64_t b) {
  const uint64_t ra = a & 0xFFFFFFFFFFFFull, rb = b & 0xFFFFFFFFFFFFull;
  if (ra != rb) return ra < rb;
  return (a >> 56) > (b >> 56);
}

// cleanMUMcand over each read's MAM matches (packed, `cap_m` slots per read;
// sorted in place), out: packed (wide == 0) or smash_match (wide == 1)
__global__ void k_mum(uint64_t *__restrict__ mam, const uint32_t *__restrict__ n_mam,
                      uint64_t n_reads, uint32_t cap_m, void *__restrict__ out, int wide,
                      uint32_t cap, uint32_t *__restrict__ n_out) {
  const uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= n_reads) return;
  uint64_t *a = mam + r * cap_m;
  const uint32_t n = n_mam[r] < cap_m ? n_mam[r] : cap_m;
  for (uint32_t i = 1; i < n; ++i) {                 // insertion sort (n <= read length)
    const uint64_t v = a[i];
    uint32_t j = i;
    while (j > 0 && by_ref_less(v, a[j - 1])) {
      a[j] = a[j - 1];
      --j;
    }
    a[j] = v;
  }
  uint32_t no = 0;
  auto emit = [&](uint64_t w) {
    if (no < cap) {
      if (wide) {
        const uint64_t ref = w & 0xFFFFFFFFFFFFull;
        reinterpret_cast<uint4 *>(out)[r * cap + no] =
            make_uint4(uint32_t(ref), uint32_t(ref >> 32), uint32_t((w >> 48) & 0xFF), uint32_t(w >> 56));
      } else {
        reinterpret_cast<uint64_t *>(out)[r * cap + no] = w;
      }
    }
    ++no;
  };
  uint64_t dbright = 0;
  bool ignoreprevious = false;
  for (uint32_t i = 0; i < n; ++i) {                 // longSA.cpp:561-579
    bool ignorecurrent = false;
    const uint64_t ref = a[i] & 0xFFFFFFFFFFFFull;
    const uint64_t currentright = ref + (a[i] >> 56) - 1;
    if (dbright > currentright) {
      ignorecurrent = true;
    } else if (dbright == currentright) {
      ignorecurrent = true;
      if (!ignoreprevious && (a[i - 1] & 0xFFFFFFFFFFFFull) == ref) ignoreprevious = true;
    } else {
      dbright = currentright;
    }
    if (i > 0 && !ignoreprevious) emit(a[i - 1]);
    ignoreprevious = ignorecurrent;
  }
  if (!ignoreprevious && n > 0) emit(a[n - 1]);
  n_out[r] = no;
}

// packed MAM words -> smash_match records
__global__ void k_widen(const uint64_t *__restrict__ mam, const uint32_t *__restrict__ n_mam,
                        uint64_t n_reads, uint32_t cap_m, uint4 *__restrict__ out, uint32_t cap,
                        uint32_t *__restrict__ n_out) {
  const uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (r >= n_reads) return;
  const uint32_t n = n_mam[r] < cap_m ? n_mam[r] : cap_m;
  for (uint32_t i = 0; i < n && i < cap; ++i) {
    const uint64_t w = mam[r * cap_m + i];
    const uint64_t ref = w & 0xFFFFFFFFFFFFull;
    out[r * cap + i] = make_uint4(uint32_t(ref), uint32_t(ref >> 32), uint32_t((w >> 48) & 0xFF),
                                  uint32_t(w >> 56));
  }
  n_out[r] = n_mam[r];
}

template <class IdxT>
int launch_mem(const smash_index *ix, uint32_t min_len, const uint8_t *seqs, uint64_t stride,
               const uint16_t *lens, uint32_t len, uint64_t n_reads, uint4 *out, uint32_t cap,
               uint32_t *n_out, hipStream_t s) {
  constexpr int B = 64;
  const uint32_t maxL = lens ? 255 : len;
  uint32_t row = ((maxL + 12 + 3) / 4) | 1;   // words (odd: conflict-free), lds_load8 over-read
  row *= 4;
  const size_t lds = size_t(B) * row;
  auto kern = k_mem<IdxT, B>;
  int per_cu = 0, cus = 0;
  SMASH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void *>(kern),
                                                         B, lds));
  SMASH_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix->device));
  if (per_cu < 1) per_cu = 1;
  uint64_t blocks = uint64_t(per_cu) * uint64_t(cus);
  const uint64_t want = (n_reads + B - 1) / B;
  if (blocks > want) blocks = want;
  MemIx<IdxT> m;
  m.x = make_dev_index<IdxT>(ix);
  m.ovf = ix->d_ovf;
  m.n_ovf = ix->n_ovf;
  m.pk = sizeof(IdxT) == 8 && ix->pos_mask == kPkPosMask;
  // deferral: collectMEMs calls over >= SMASH_MEM_DEFER ranks (default 64;
  // 0: none) become jobs, up to 4 per read on average (a full list: inline)
  uint64_t defer = 64;
  if (const char *e = std::getenv("SMASH_MEM_DEFER")) defer = uint64_t(std::strtoull(e, nullptr, 10));
  const uint64_t job_cap = defer ? std::min<uint64_t>(std::max<uint64_t>(4 * n_reads, 1 << 16),
                                                      (1ull << 31)) : 0;
  MemJob *jobs = nullptr;
  unsigned long long *n_jobs = nullptr;
  uint32_t *E = nullptr, *base = nullptr, *slot = nullptr, *holes = nullptr, *off = nullptr;
  void *tmp = nullptr;
  size_t tmp_bytes = 0;
  if (job_cap) {
    SMASH_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, holes, off, n_reads + 1, s));
    SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&jobs), job_cap * sizeof(MemJob), s));
    SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&n_jobs), 8, s));
    SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&E), job_cap * 4, s));
    SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&base), job_cap * 4, s));
    SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&slot), job_cap * 4, s));
    SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&holes), (n_reads + 1) * 4, s));
    SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&off), (n_reads + 1) * 4, s));
    SMASH_HIP(hipMallocAsync(&tmp, tmp_bytes + 16, s));
    SMASH_HIP(hipMemsetAsync(n_jobs, 0, 8, s));
    SMASH_HIP(hipMemsetAsync(holes + n_reads, 0, 4, s));
  }
  SMASH_HIP(hipMemsetAsync(ix->d_work, 0, 8, s));
  if (ix->kev[0]) SMASH_HIP(hipEventRecord(ix->kev[0], s));
  kern<<<unsigned(blocks), B, lds, s>>>(m, seqs, stride, lens, len, n_reads, min_len, out, cap,
                                        n_out, row, reinterpret_cast<unsigned long long *>(ix->d_work),
                                        jobs, n_jobs, job_cap, defer ? defer : ~0ull, holes);
  SMASH_HIP(hipGetLastError());
  if (job_cap) {
    // the jobs' record counts; each read's jobs in hole order; the reads'
    // totals and first job records; the records that land below cap
    const unsigned gj = unsigned(std::min<uint64_t>(std::max<uint64_t>(1, uint64_t(cus) * 8),
                                                    (job_cap + 3) / 4));
    k_mem_jobs<IdxT, false><<<gj, 256, 0, s>>>(m, jobs, n_jobs, job_cap, min_len, out, cap, E, base);
    SMASH_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, holes, off, n_reads + 1, s));
    k_job_slots<<<unsigned(std::min<uint64_t>(65535, (job_cap + 255) / 256)), 256, 0, s>>>(
        jobs, n_jobs, job_cap, off, slot);
    k_mem_fix<<<unsigned((n_reads + 255) / 256), 256, 0, s>>>(jobs, E, holes, off, slot, n_reads, out,
                                                            cap, n_out, base);
    k_mem_jobs<IdxT, true><<<gj, 256, 0, s>>>(m, jobs, n_jobs, job_cap, min_len, out, cap, E, base);
    SMASH_HIP(hipGetLastError());
    for (void *q : {(void *)jobs, (void *)n_jobs, (void *)E, (void *)base, (void *)slot, (void *)holes,
                    (void *)off, tmp})
      (void)hipFreeAsync(q, s);
  }
  if (ix->kev[1]) SMASH_HIP(hipEventRecord(ix->kev[1], s));
  return SMASH_OK;
}

// MAM into a scratch buffer of L slots per read (exact: one MAM per prefix
// at most), then k_mum or k_widen
int mam_then(const smash_index *ix, int mode, uint32_t min_len, const uint8_t *seqs,
             uint64_t stride, const uint16_t *lens, uint32_t len, uint64_t n_reads, void *out,
             int wide, uint32_t cap, uint32_t *n_out, hipStream_t s) {
  const uint32_t cap_m = lens ? 255 : len;
  uint64_t *tmp = nullptr;
  uint32_t *ntmp = nullptr;
  SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&tmp), n_reads * cap_m * 8 + 8, s));
  SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&ntmp), n_reads * 4 + 4, s));
  int rc = smash_map_batch(ix, SMASH_MODE_MAM, min_len, seqs, stride, lens, len, n_reads, tmp, cap_m,
                           ntmp, s);
  if (rc == SMASH_OK) {
    const unsigned g = unsigned((n_reads + 255) / 256);
    if (mode == SMASH_MODE_MUM)
      k_mum<<<g, 256, 0, s>>>(tmp, ntmp, n_reads, cap_m, out, wide, cap, n_out);
    else
      k_widen<<<g, 256, 0, s>>>(tmp, ntmp, n_reads, cap_m, static_cast<uint4 *>(out), cap, n_out);
    if (hipGetLastError() != hipSuccess) rc = SMASH_ERR_HIP;
  }
  (void)hipFreeAsync(tmp, s);
  (void)hipFreeAsync(ntmp, s);
  if (rc == SMASH_ERR_HIP) set_error(std::string("mam_then: ") + smash_last_error());
  return rc;
}

int check_args(const smash_index *ix, const uint8_t *seqs, const void *out, const uint32_t *n_out,
               uint32_t cap, const uint16_t *lens, uint32_t len, uint32_t min_len) {
  if (!ix || !seqs || !out || !n_out || cap == 0) {
    set_error("smash_match_batch: bad arguments");
    return SMASH_ERR_ARG;
  }
  if (!lens && (len == 0 || len > 255)) {
    set_error("smash_match_batch: read length must be 1..255");
    return SMASH_ERR_ARG;
  }
  if (min_len < 2) {   // "NOTE: min_len must be > 1" (longSA.h:194)
    set_error("smash_match_batch: min_len must be > 1");
    return SMASH_ERR_ARG;
  }
  return SMASH_OK;
}

}  // namespace

// smash_map_batch's MUM mode (packed records)
int map_batch_mum(const smash_index *ix, uint32_t min_len, const uint8_t *seqs, uint64_t stride,
                  const uint16_t *lens, uint32_t len, uint64_t n_reads, uint64_t *out, uint32_t cap,
                  uint32_t *n_out, hipStream_t s) {
  return mam_then(ix, SMASH_MODE_MUM, min_len, seqs, stride, lens, len, n_reads, out, 0, cap, n_out, s);
}

}  // namespace smash

using namespace smash;

extern "C" int smash_match_batch(const smash_index *ix, int mode, uint32_t min_len,
                                 const uint8_t *d_seqs, uint64_t stride, const uint16_t *d_lens,
                                 uint32_t len, uint64_t n_reads, smash_match *d_out,
                                 uint32_t cap_per_read, uint32_t *d_n_out, void *stream) {
  int rc = check_args(ix, d_seqs, d_out, d_n_out, cap_per_read, d_lens, len, min_len);
  if (rc != SMASH_OK) return rc;
  if (mode != SMASH_MODE_MAM && mode != SMASH_MODE_MUM && mode != SMASH_MODE_MEM) {
    set_error("smash_match_batch: mode must be SMASH_MODE_MAM, _MUM or _MEM");
    return SMASH_ERR_ARG;
  }
  if (mode == SMASH_MODE_MEM && !ix->d_kmer) {
    set_error("smash_match_batch: index lacks the k-mer table");
    return SMASH_ERR_ARG;
  }
  if (n_reads == 0) return SMASH_OK;
  SMASH_HIP(hipSetDevice(ix->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint4 *out = reinterpret_cast<uint4 *>(d_out);
  if (mode == SMASH_MODE_MEM) {
    if (ix->idx_bytes == 4)
      return launch_mem<uint32_t>(ix, min_len, d_seqs, stride, d_lens, len, n_reads, out,
                                  cap_per_read, d_n_out, s);
    return launch_mem<uint64_t>(ix, min_len, d_seqs, stride, d_lens, len, n_reads, out,
                                cap_per_read, d_n_out, s);
  }
  return mam_then(ix, mode, min_len, d_seqs, stride, d_lens, len, n_reads, out, 1, cap_per_read,
                  d_n_out, s);
}
