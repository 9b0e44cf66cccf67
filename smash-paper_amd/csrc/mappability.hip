// smash-paper_amd/csrc/mappability.hip -- the whole-genome mappability
// self-scan (BASELINE config C5): map.bin bytes for a range of forward bases
// from the resident ISA + LCP, and the derived unique-k-mer counts.
//
// map.bin (longSA::show, longSA.cpp:612-690): for forward base i of a contig
// of size S starting at text position sp,
//   right = m[ISA[sp + i]],  zeroed when right + i >= S   (:666)
//   left  = m[ISA[sp + 2S - i]], zeroed when left >= i     (:667)
//   m[r]  = max(LCP[r], LCP[r + 1]) + 1                     (:628-641)
// each stored min(., 255) as the byte pair [left, right].  The zeroing tests
// use the exact LCP (the u8 array + the overflow table), so a repeat longer
// than 255 near a contig end is handled as the reference handles it.
//
// The k-mer starting at forward base i is unique in the doubled text iff
// 1 <= right <= k.  Counts go per contig and per
// variable-width bin (abspos = chrom_sizes offset + i, bisect_right over the
// bin starts, i = 0 lands in the last bin as in varbin.py:89-92).
//
// Streaming form.  U[x] = min(255, max(LCP[ISA[x]], LCP[ISA[x] + 1])) is
// resident with the index (aux_build.hip), so m(x) = U[x] + 1 exactly when
// U[x] < 255: the scan reads U at the forward position sp + i and at the
// reverse-complement position sp + 2S - i, both sequentially, and writes the
// two bytes -- 4 B per base, HBM-streaming -- instead of two ISA reads and
// two random LCP lines per base.  When U[x] == 255 (m >= 256: N runs, long
// repeats) the byte is 255 unless the edge rule zeroes it, and that rule is
// decided without the exact m whenever possible:
//   * m >= 256, so right is zeroed if i + 256 >= S, left if i <= 256;
//   * m(x) <= m(y) + (y - x) for any y > x (the match that gives m(x), moved
//     y - x positions on, is a match of the suffix at y), so with y the next
//     text position holding U[y] < 255, m(x) <= U[y] + 1 + (y - x): right is
//     kept when i + that bound < S, left when the bound < i.
// Only the bases left undecided (saturated runs that reach a contig end:
// the N runs at chromosome ends) take the exact path: ISA, then the LCP
// bytes and the overflow table (a ~30-load bisection at hg19).  Their m is
// >= 256 > k, so the byte is 0 or 255 and the unique counts do not depend on
// it: the scan writes 255, lists {text position, byte index, zero threshold}
// and k_mapfix settles the listed bytes with one thread each, all in flight
// together, instead of a serial chain on the thread (and the launch tail) of
// the tile that meets them.  (k >= 255, or no map output, or a full list:
// the exact path runs inline as before.)  The
// next unsaturated position comes from the block's own U bytes, else from a
// directory holding, per 4096 text positions, the first unsaturated position
// at or after them (built once per index, 12 MB at hg19: one load per
// lookup, also inside N runs).
//
// Latency: a block's fixed work is one tile's loads and its LDS bin counts;
// the bin ordinal of each tile's first base comes from k_tilebins (one thread
// per tile, all bisections in flight at once) instead of a 16-load bisection
// on the block's critical path.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <iterator>

#include "common.hpp"

namespace smash {
namespace {

constexpr int kMB = 256;                    // threads per block
constexpr int kMPer = 16;                   // consecutive bases per thread
constexpr uint64_t kMTile = uint64_t(kMB) * kMPer;
constexpr int kDirShift = 12;               // directory: 4096 text positions per entry
constexpr int kLdsBins = 32;                // bins of a tile counted in LDS
constexpr uint64_t kNone = ~0ull;
constexpr int kMaxSegLds = 128;             // segment tables up to this size live in LDS

struct MapCtx {
  const uint8_t *L8;
  const uint64_t *ovf;
  uint64_t n_ovf, N;
  const int64_t *bins;
  uint32_t nbins, k;
  uint64_t *fix;                 // [fix_cap][3] {x, byte index in the scan's output, threshold}
  unsigned long long *nfix;
  uint64_t fix_cap;
  uint64_t pm;                   // position bits of an ISA word (packed hints masked off)
};
constexpr uint64_t kFixCap = uint64_t(1) << 23;

__device__ __forceinline__ uint64_t lcp_exact(const MapCtx &c, uint64_t r) {
  const uint32_t v = c.L8[r];
  if (v < 255) return v;
  uint64_t lo = 0, hi = c.n_ovf;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (c.ovf[2 * mid] < r) lo = mid + 1;
    else hi = mid;
  }
  return lo < c.n_ovf ? c.ovf[2 * lo + 1] : 255;
}

__device__ __forceinline__ uint64_t min_len_at(const MapCtx &c, uint64_t r) {
  const uint64_t a = lcp_exact(c, r), b = r + 1 < c.N ? lcp_exact(c, r + 1) : 0;
  return (a > b ? a : b) + 1;
}

__device__ __forceinline__ uint32_t bisect_right(const MapCtx &c, int64_t a) {
  uint32_t lo = 0, hi = c.nbins;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a < c.bins[mid]) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

__device__ __forceinline__ uint4 load16u(const uint8_t *p) {
  uint4 v;
  __builtin_memcpy(&v, p, 16);
  return v;
}
__device__ __forceinline__ uint32_t byte_of(const uint4 &v, uint32_t q) {
  const uint32_t w = q < 4 ? v.x : q < 8 ? v.y : q < 12 ? v.z : v.w;
  return (w >> (8 * (q & 3))) & 0xFF;
}

// an unsaturated text position >= p (kNone: none before N): the first one
// at or after the next multiple of 4096 (exact when p is a multiple; a later,
// looser bound otherwise, which the callers accept).  dir is the suffix-min
// directory (scan_t).
__device__ __forceinline__ uint64_t next_unsat_dir(const uint64_t *dir, uint64_t ndir, uint64_t p) {
  const uint64_t t = (p + (uint64_t(1) << kDirShift) - 1) >> kDirShift;
  return t < ndir ? dir[t] : kNone;
}

// one contig's part of the scan: bases [i0, i1) of the contig at text
// position sp (size S); its map.bin bytes at out + out_off; abs0 = its
// chrom_sizes offset (< 0: not binned); tiles [tile0, tile0 + tiles of it)
// of the launch
struct Seg {
  uint64_t sp, S, i0, i1, out_off, tile0;
  int64_t abs0;
  uint64_t contig;
};

// the segment holding launch tile T (segs ascending by tile0)
__device__ __forceinline__ uint32_t seg_of(const Seg *segs, uint32_t nseg, uint64_t T) {
  uint32_t lo = 0, hi = nseg;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (segs[mid].tile0 <= T) lo = mid;
    else hi = mid;
  }
  return lo;
}

// bit i (0..15): byte i of the block is 0xFF
__device__ __forceinline__ uint32_t sat_mask16(const uint4 &v) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    const uint32_t w = ~(k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w);
    // 0x80 in each byte of w that is non-zero (exact, no borrows)
    const uint32_t nz = (((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w) & 0x80808080u;
    const uint32_t z = ~nz & 0x80808080u;                 // bytes of v equal to 0xFF
    m |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * k);
  }
  return m;
}
// the 16-bit mask reversed (byte 15 - q of the rc block is base q)
__device__ __forceinline__ uint32_t rev16(uint32_t m) { return __brev(m) >> 16; }

// dir[t] = the first text position p in [t << 12, (t + 1) << 12) with
// U[p] < 255, else kNone: one wave per tile, 64 bytes per lane, the first
// lane holding an unsaturated byte found by a ballot (no LDS, no barrier)
__global__ __launch_bounds__(kMB) void k_nsdir(const uint8_t *__restrict__ U, uint64_t N,
                                               uint64_t *__restrict__ dir, uint64_t t0,
                                               uint64_t t1) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t waves = uint64_t(gridDim.x) * (blockDim.x >> 6);
  for (uint64_t t = t0 + uint64_t(blockIdx.x) * (blockDim.x >> 6) + (threadIdx.x >> 6); t < t1;
       t += waves) {
    const uint64_t p0 = (t << kDirShift) + uint64_t(lane) * 64;
    uint32_t q = 64;   // this lane's first unsaturated byte (64: none)
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      if (p0 + 16 * k < N && q == 64) {
        uint32_t m = ~sat_mask16(load16u(U + p0 + 16 * k)) & 0xFFFFu;
        if (p0 + 16 * k + 16 > N) m &= (1u << uint32_t(N - p0 - 16 * k)) - 1u;
        if (m) q = 16 * k + uint32_t(__builtin_ctz(m));
      }
    }
    const uint64_t b = __ballot(q < 64);
    const uint64_t mine = p0 + q;   // (every lane takes part in the shuffle)
    const uint64_t f = __shfl(mine, b ? int(__builtin_ctzll(b)) : 0, 64);
    if (lane == 0) dir[t] = b ? f : kNone;
  }
}

// dir[t] = min(dir[t], dir[t + 1], ...): the first unsaturated position at or
// after tile t, from each tile's own first (entries already propagated are
// fixed points of it).  Three small kernels: the minimum of each segment of
// kSegDir entries, a suffix minimum over the segments (one block), then each
// segment's own suffix minimum with the carry from the segments after it.
constexpr uint32_t kSegDir = 4096;
__global__ __launch_bounds__(kMB) void k_dir_segmin(const uint64_t *__restrict__ dir, uint64_t n,
                                                    uint64_t *__restrict__ segmin) {
  __shared__ unsigned long long s_m;
  if (threadIdx.x == 0) s_m = kNone;
  __syncthreads();
  const uint64_t a = uint64_t(blockIdx.x) * kSegDir;
  unsigned long long m = kNone;
  for (uint64_t t = a + threadIdx.x; t < a + kSegDir && t < n; t += blockDim.x)
    m = dir[t] < m ? dir[t] : m;
  atomicMin(&s_m, m);
  __syncthreads();
  if (threadIdx.x == 0) segmin[blockIdx.x] = s_m;
}
__global__ void k_dir_carry(uint64_t *segmin, uint32_t nseg) {   // one thread: nseg ~ 400
  if (threadIdx.x) return;
  uint64_t m = kNone;
  for (uint32_t k = nseg; k-- > 0;) {
    const uint64_t v = segmin[k];
    segmin[k] = m;   // the carry into segment k: the minimum after it
    m = v < m ? v : m;
  }
}
__global__ __launch_bounds__(kMB) void k_dir_apply(uint64_t *__restrict__ dir, uint64_t n,
                                                   const uint64_t *__restrict__ carry) {
  // kSegDir entries per block, 16 per thread: each thread's suffix minimum,
  // then the block's suffix scan of the thread minima (LDS), then apply
  __shared__ uint64_t s_t[kMB];
  constexpr uint32_t per = kSegDir / kMB;
  const uint64_t a = uint64_t(blockIdx.x) * kSegDir + uint64_t(threadIdx.x) * per;
  uint64_t v[per];
  uint64_t m = kNone;
#pragma unroll
  for (int k = int(per) - 1; k >= 0; --k) {
    v[k] = a + k < n ? dir[a + k] : kNone;
    m = v[k] < m ? v[k] : m;
    v[k] = m;
  }
  s_t[threadIdx.x] = m;
  __syncthreads();
  uint64_t after = carry[blockIdx.x];
  for (uint32_t u = threadIdx.x + 1; u < kMB; ++u) after = s_t[u] < after ? s_t[u] : after;
#pragma unroll
  for (uint32_t k = 0; k < per; ++k)
    if (a + k < n) dir[a + k] = v[k] < after ? v[k] : after;
}

hipError_t dir_suffix_min(uint64_t *dir, uint64_t ndir, hipStream_t s) {
  const uint32_t nseg = uint32_t((ndir + kSegDir - 1) / kSegDir);
  uint64_t *seg = nullptr;
  hipError_t e = hipMallocAsync(reinterpret_cast<void **>(&seg), 8 * (nseg + 1), s);
  if (e != hipSuccess) return e;
  k_dir_segmin<<<nseg, kMB, 0, s>>>(dir, ndir, seg);
  k_dir_carry<<<1, 64, 0, s>>>(seg, nseg);
  k_dir_apply<<<nseg, kMB, 0, s>>>(dir, ndir, seg);
  e = hipGetLastError();
  (void)hipFreeAsync(seg, s);
  return e;
}

// the directory entries of text positions [lo, hi) from U, then propagated
hipError_t build_nsdir(const smash_index *ix, uint64_t lo, uint64_t hi, hipStream_t s) {
  const uint64_t ndir = (ix->N + (uint64_t(1) << kDirShift) - 1) >> kDirShift;
  if (!ix->d_nsdir) {
    hipError_t e = hipMalloc(&ix->d_nsdir, 8 * ndir);
    if (e != hipSuccess) return e;
    lo = 0;
    hi = ix->N;
  }
  const uint64_t t0 = lo >> kDirShift;
  const uint64_t t1 = std::min(ndir, (hi + (uint64_t(1) << kDirShift) - 1) >> kDirShift);
  if (t0 < t1)   // (one wave per tile)
    k_nsdir<<<unsigned(std::min<uint64_t>((t1 - t0 + 3) / 4, 65536)), kMB, 0, s>>>(
        ix->d_uniq, ix->N, ix->d_nsdir, t0, t1);
  hipError_t e = hipGetLastError();
  // (the scan covers entry t1 too: a window tile without an unsaturated
  // position takes the propagated entry after the window)
  return e == hipSuccess ? dir_suffix_min(ix->d_nsdir, std::min(ndir, t1 + 1), s) : e;
}


// bin ordinal (bisect_right of abs0 + the tile's first base) per tile
__global__ void k_tilebins(MapCtx c, const Seg *segs, uint32_t nseg, uint64_t ntiles,
                           uint64_t tile, uint32_t *o0) {
  const uint64_t T = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (T >= ntiles) return;
  const Seg g = segs[seg_of(segs, nseg, T)];
  o0[T] = g.abs0 >= 0 ? bisect_right(c, g.abs0 + int64_t(g.i0 + (T - g.tile0) * tile)) : 0;
}

// every contig's bases in ONE launch (per-contig launches and their tails
// dominated the scan): block-stride over the tiles of all segments; out: the
// scan's map.bin bytes (or null)
template <class IdxT, int W, bool PF_U, int SUB>
__global__ __launch_bounds__(kMB, W) void k_mapscan(MapCtx c, const IdxT *__restrict__ ISA,
                                                 const uint8_t *__restrict__ U,
                                                 const uint64_t *__restrict__ dir, uint64_t ndir,
                                                 const Seg *__restrict__ segs, uint32_t nseg,
                                                 uint64_t ntiles_all, uint8_t *__restrict__ out,
                                                 const uint32_t *__restrict__ tile_o0,
                                                 unsigned long long *bin_counts,
                                                 unsigned long long *contig_counts) {
  // per-tile LDS, double-buffered by tile parity: a tile's counts are read
  // and cleared by their flushers while the faster threads already count the
  // next tile into the other buffer (two barriers per tile, not four)
  __shared__ unsigned long long s_bin[2][kLdsBins + 1];
  __shared__ int64_t s_bs[2][kLdsBins];
  __shared__ unsigned long long s_tot[2];
  __shared__ uint64_t s_f[kMB / 64], s_r[kMB / 64];   // per wave: first unsaturated (fwd / rc)
  __shared__ uint64_t s_ftail, s_rtail;
  __shared__ Seg s_segs[kMaxSegLds];   // the segment table, once per block
  // a tile is SUB sub-tiles of kMTile bases, one after the other: the
  // tile's fixed work (segment, bin ordinal, bin starts, the counts' flush,
  // two barriers) once per SUB x 4 096 bases
  static_assert(!PF_U || SUB == 1, "the U fetch ahead covers one sub-tile");
  constexpr uint64_t kTile = kMTile * SUB;
  const uint64_t N = c.N;
  const bool lds_segs = nseg <= uint32_t(kMaxSegLds);
  if (lds_segs)
    for (uint32_t k = threadIdx.x; k < nseg; k += blockDim.x) s_segs[k] = segs[k];
  if (threadIdx.x <= kLdsBins) s_bin[0][threadIdx.x] = s_bin[1][threadIdx.x] = 0;
  if (threadIdx.x == 0) s_tot[0] = s_tot[1] = 0;
  __syncthreads();
  const Seg *tab = lds_segs ? s_segs : segs;
  // thread 0's running unique count of the block's tiles in one contig,
  // added when the contig changes and at the end (an atomic per tile on ~25
  // contig addresses serialised ~60 k same-address atomics on chr1's)
  unsigned long long run_tot = 0;
  uint64_t run_contig = ~0ull;
  // a tile's inputs are fetched one trip ahead (its segment, bin ordinal,
  // bin starts, and with PF_U this thread's two U blocks): the waves waited
  // on these loads for most of their cycles (profiles/r04/c5pmc); PF_U's
  // registers cost more occupancy than the early U loads buy
  struct TileIn {
    uint32_t seg, o0;
    int64_t bs;
    uint4 fw, rw;
  };
  auto fetch = [&](uint64_t T) {
    TileIn x;
    x.seg = seg_of(tab, nseg, T);   // (every thread: same LDS words, broadcast)
    const Seg &g = tab[x.seg];
    const bool binned = g.abs0 >= 0 && c.nbins;
    x.o0 = binned ? tile_o0[T] : 0;
    x.bs = binned && threadIdx.x < kLdsBins
               ? (x.o0 + threadIdx.x < c.nbins ? c.bins[x.o0 + threadIdx.x] : INT64_MAX)
               : INT64_MAX;
    if (!PF_U) return x;
    const uint64_t ib = g.i0 + (T - g.tile0) * kTile + uint64_t(threadIdx.x) * kMPer;
    const uint64_t xf = g.sp + ib, xr = g.sp + 2 * g.S - ib;
    x.fw = xf + 16 <= N + 64 ? load16u(U + xf) : make_uint4(~0u, ~0u, ~0u, ~0u);
    x.rw = xr >= 15 ? load16u(U + xr - 15) : make_uint4(~0u, ~0u, ~0u, ~0u);
    return x;
  };
  uint32_t par = 0;
  TileIn cur{};
  if (uint64_t(blockIdx.x) < ntiles_all) cur = fetch(blockIdx.x);
  for (uint64_t T = blockIdx.x; T < ntiles_all; T += gridDim.x, par ^= 1u) {
    TileIn nxt{};
    if (T + gridDim.x < ntiles_all) nxt = fetch(T + gridDim.x);
    const Seg g = tab[cur.seg];
    const uint64_t sp = g.sp, S = g.S, i0 = g.i0, i1 = g.i1;
    const int64_t abs0 = g.abs0;
    const bool binned = abs0 >= 0 && c.nbins;
    const bool contig_count = contig_counts != nullptr;
    const uint64_t t0 = i0 + (T - g.tile0) * kTile;
    const uint32_t o0 = cur.o0;
    unsigned long long *sbin = s_bin[par];
    const int64_t *s_bsp = s_bs[par];
    if (binned && threadIdx.x < kLdsBins) s_bs[par][threadIdx.x] = cur.bs;   // (read after the barrier below)
    unsigned long long mine = 0;
    uint32_t d = 0;   // bin ordinal offset from o0 (monotone over the thread's bases)
    for (uint32_t r = 0; r < uint32_t(SUB); ++r) {
    // (block-uniform: a sub-tile past the segment's end is skipped whole, so
    // a thread's rc position xr never falls below the contig's own text)
    if (r && t0 + r * kMTile >= i1) break;
    // this thread's 16 bases: U at the forward positions (ascending) and at
    // the reverse-complement positions (descending; byte 15 - q is base q)
    const uint64_t ib = t0 + r * kMTile + uint64_t(threadIdx.x) * kMPer;
    const uint64_t xf = sp + ib, xr = sp + 2 * S - ib;   // xr - q: base ib + q
    uint4 fw = cur.fw, rw = cur.rw;
    if (!PF_U) {
      fw = xf + 16 <= N + 64 ? load16u(U + xf) : make_uint4(~0u, ~0u, ~0u, ~0u);
      rw = xr >= 15 ? load16u(U + xr - 15) : make_uint4(~0u, ~0u, ~0u, ~0u);
    }
    // bit q: U == 255 at base ib + q (or past the text), 4 bytes per step:
    // a byte is 0xFF iff its complement is zero
    uint32_t satf = sat_mask16(fw), satr = rev16(sat_mask16(rw));
    if (xf + 16 > N)
      for (uint32_t q = 0; q < uint32_t(kMPer); ++q) satf |= uint32_t(xf + q >= N) << q;
    if (xr < 15)
      for (uint32_t q = 0; q < uint32_t(kMPer); ++q) satr |= uint32_t(xr < q) << q;
    // lowest unsaturated fwd text position, lowest rc one (largest q)
    const uint64_t ff = (~satf & 0xFFFFu) ? xf + __builtin_ctz(~satf & 0xFFFFu) : kNone;
    const uint64_t fr = (~satr & 0xFFFFu) ? xr - (31 - __builtin_clz(~satr & 0xFFFFu)) : kNone;
    const bool any_sat = __syncthreads_or((satf | satr) != 0);
    uint64_t fnext = kNone, rnext = kNone;   // first unsaturated chunk after / before mine
    if (any_sat) {
      // the min of the forward chunk heads over later chunks, and of the rc
      // chunk heads over earlier chunks (higher text positions): within the
      // wave by shuffles, across the block's waves through LDS (one barrier;
      // a block-wide LDS scan took 16)
      const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
      uint64_t xs = ff, xp = fr;   // inclusive suffix-min / prefix-min in the wave
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t a = __shfl_down(xs, d, 64), b = __shfl_up(xp, d, 64);
        if (lane + d < 64) xs = a < xs ? a : xs;
        if (lane >= d) xp = b < xp ? b : xp;
      }
      const uint64_t after = __shfl_down(xs, 1, 64), before = __shfl_up(xp, 1, 64);
      if (lane == 0) s_f[wv] = xs;    // the wave's minima
      if (lane == 63) s_r[wv] = xp;
      if (threadIdx.x == 0) {
        s_ftail = next_unsat_dir(dir, ndir, sp + t0 + (r + 1) * kMTile);
        s_rtail = next_unsat_dir(dir, ndir, xr + 1);       // above the tile's rc range
      }
      __syncthreads();
      fnext = lane < 63 ? after : kNone;
      rnext = lane > 0 ? before : kNone;
      for (uint32_t w = wv + 1; w < uint32_t(kMB / 64); ++w) fnext = s_f[w] < fnext ? s_f[w] : fnext;
      for (uint32_t w = 0; w < wv; ++w) rnext = s_r[w] < rnext ? s_r[w] : rnext;
      if (fnext == kNone) fnext = s_ftail;
      if (rnext == kNone) rnext = s_rtail;
    }
    uint32_t ob[2 * kMPer / 4] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t fixr = 0, fixl = 0;   // bases whose right / left byte k_mapfix settles
    const bool defer = out && c.fix && c.k < 255;
    // fast path (most chunks): no saturated byte and every base inside
    // [i0, i1): straight-line selects, the unique bases as a mask, and their
    // bin counted with one LDS atomic when the 16 bases share a bin
    const bool fast = (satf | satr) == 0 && ib + kMPer <= i1;
    uint32_t umask = 0;
    if (fast) {
      // the output byte pairs [left, right] = [rc U + 1, fwd U + 1] by byte
      // permutes (U < 255 here: + 0x01 per byte cannot carry): word 2m holds
      // bases 4m, 4m + 1 (fwd dword m bytes 0, 1; rc dword 3 - m bytes 3, 2),
      // word 2m + 1 bases 4m + 2, 4m + 3 (bytes 2, 3; 1, 0)
      const uint32_t f1[4] = {fw.x + 0x01010101u, fw.y + 0x01010101u, fw.z + 0x01010101u,
                              fw.w + 0x01010101u};
      const uint32_t r1[4] = {rw.x + 0x01010101u, rw.y + 0x01010101u, rw.z + 0x01010101u,
                              rw.w + 0x01010101u};
#pragma unroll
      for (uint32_t m = 0; m < 4; ++m) {
        ob[2 * m] = __builtin_amdgcn_perm(f1[m], r1[3 - m], 0x05020403u);
        ob[2 * m + 1] = __builtin_amdgcn_perm(f1[m], r1[3 - m], 0x07000601u);
      }
#pragma unroll
      for (uint32_t q = 0; q < uint32_t(kMPer); ++q)
        umask |= uint32_t(byte_of(fw, q) < c.k) << q;      // 1 <= right = U + 1 <= k
      // the edge rules can zero a byte only near the contig ends (m <= 256):
      // a separate pass for those chunks
      if (ib < 272 || ib + kMPer + 256 > S) {
        const uint32_t rem = S - ib < 0xFFFFFFFFull ? uint32_t(S - ib) : 0xFFFFFFFFu, ib32 = uint32_t(ib < 272 ? ib : 272);
#pragma unroll
        for (uint32_t q = 0; q < uint32_t(kMPer); ++q) {
          const uint32_t sh = 16 * (q & 1);
          if (byte_of(fw, q) + 1 + q >= rem) {             // right + i >= S (:666)
            ob[q >> 1] &= ~(0xFF00u << sh);
            umask &= ~(1u << q);
          }
          if (byte_of(rw, 15 - q) + 1 >= ib32 + q) ob[q >> 1] &= ~(0xFFu << sh);   // left >= i
        }
      }
      mine += uint32_t(__popc(umask));
      if (binned && umask) {
        const int64_t a0 = abs0 + int64_t(ib) + __builtin_ctz(umask);
        const int64_t a1 = abs0 + int64_t(ib) + 31 - __builtin_clz(umask);
        while (d < uint32_t(kLdsBins) && a0 >= s_bsp[d]) ++d;
        if (d < uint32_t(kLdsBins) && a1 < s_bsp[d]) {       // [a0, a1] in one bin
          atomicAdd(&sbin[d], (unsigned long long)__popc(umask));
        } else {
          for (uint32_t m = umask; m; m &= m - 1) {
            const int64_t a = abs0 + int64_t(ib) + __builtin_ctz(m);
            while (d < uint32_t(kLdsBins) && a >= s_bsp[d]) ++d;
            if (d < uint32_t(kLdsBins)) {
              atomicAdd(&sbin[d], 1ull);
            } else {
              const uint32_t o = bisect_right(c, a);
              atomicAdd(&bin_counts[o == 0 ? c.nbins - 1 : o - 1], 1ull);
            }
          }
        }
      }
    }
    // U at the first unsaturated position after / above the chunk, loaded
    // once (the saturated bases of the chunk all bound through it)
    const uint32_t ufn = !fast && satf && fnext != kNone ? uint32_t(U[fnext]) : 0u;
    const uint32_t urn = !fast && satr && rnext != kNone ? uint32_t(U[rnext]) : 0u;
#pragma unroll 1
    for (uint32_t q = 0; q < uint32_t(kMPer) && !fast; ++q) {
      const uint64_t i = ib + q;
      if (i >= i1) break;
      // right: m at the forward position, zeroed when m + i >= S (:666)
      uint64_t right;
      if (!((satf >> q) & 1)) {
        right = byte_of(fw, q) + 1;
        if (right + i >= S) right = 0;
      } else if (i + 256 >= S) {
        right = 0;
      } else {
        // the next unsaturated text position after xf + q: in the chunk (its
        // U byte is in fw), else fnext
        const uint32_t above = ~satf & 0xFFFFu & (0xFFFFFFFEu << q);
        const uint32_t q2 = above ? uint32_t(__builtin_ctz(above)) : 0u;
        const uint64_t ub = above ? uint64_t(byte_of(fw, q2)) + 1 + (q2 - q)
                            : fnext == kNone ? kNone : ufn + 1 + (fnext - (xf + q));
        if (ub != kNone && i + ub < S) right = 255;
        else if (defer) {
          right = 255;
          fixr |= 1u << q;
        } else {
          right = min_len_at(c, uint64_t(ISA[xf + q]) & c.pm);
          if (right + i >= S) right = 0;
        }
      }
      // left: m at the reverse-complement position, zeroed when m >= i (:667)
      uint64_t left;
      if (!((satr >> q) & 1)) {
        left = byte_of(rw, 15 - q) + 1;
        if (left >= i) left = 0;
      } else if (i <= 256) {
        left = 0;
      } else {
        // the next unsaturated text position above xr - q: in the chunk
        // (base q2 < q, the largest: rw byte 15 - q2), else rnext
        const uint32_t below = ~satr & ((1u << q) - 1u);
        const uint32_t q2 = below ? 31u - uint32_t(__builtin_clz(below)) : 0u;
        const uint64_t ub = below ? uint64_t(byte_of(rw, 15 - q2)) + 1 + (q - q2)
                            : rnext == kNone ? kNone : urn + 1 + (rnext - (xr - q));
        if (ub != kNone && ub < i) left = 255;
        else if (defer) {
          left = 255;
          fixl |= 1u << q;
        } else {
          left = min_len_at(c, uint64_t(ISA[xr - q]) & c.pm);
          if (left >= i) left = 0;
        }
      }
      const uint32_t lb = uint32_t(left < 255 ? left : 255), rb = uint32_t(right < 255 ? right : 255);
      ob[q >> 1] |= (lb | (rb << 8)) << (16 * (q & 1));
      if (rb >= 1 && rb <= c.k) {
        ++mine;
        if (binned) {
          const int64_t a = abs0 + int64_t(i);
          while (d < uint32_t(kLdsBins) && a >= s_bsp[d]) ++d;
          if (d < uint32_t(kLdsBins)) {
            atomicAdd(&sbin[d], 1ull);
          } else {
            const uint32_t o = bisect_right(c, a);
            atomicAdd(&bin_counts[o == 0 ? c.nbins - 1 : o - 1], 1ull);
          }
        }
      }
    }
    if (c.fix && __ballot((fixr | fixl) != 0)) {   // list the deferred bytes: one atomic per wave
      const uint32_t nf = uint32_t(__popc(fixr) + __popc(fixl));
      const uint32_t lane = threadIdx.x & 63;
      uint32_t x = nf;
      for (int dd = 1; dd < 64; dd <<= 1) {
        const uint32_t y = __shfl_up(x, dd, 64);
        if (lane >= uint32_t(dd)) x += y;
      }
      const uint32_t tot = __shfl(x, 63, 64);
      unsigned long long fb = 0;
      if (lane == 63 && tot) fb = atomicAdd(c.nfix, (unsigned long long)tot);
      fb = __shfl(fb, 63, 64) + (x - nf);
      for (uint32_t q = 0; q < uint32_t(kMPer); ++q) {
        for (uint32_t side = 0; side < 2; ++side) {
          if (!(((side ? fixl : fixr) >> q) & 1)) continue;
          const uint64_t i = ib + q;
          const uint64_t x = side ? xr - q : xf + q;
          const uint64_t bi = g.out_off + 2 * (i - i0) + (side ? 0 : 1);
          const uint64_t thr = side ? i : S - i;   // zeroed when m >= thr
          if (fb < c.fix_cap) {
            c.fix[3 * fb] = x; c.fix[3 * fb + 1] = bi; c.fix[3 * fb + 2] = thr;
          } else {                                 // list full: exact path here
            const uint64_t mm = min_len_at(c, uint64_t(ISA[x]) & c.pm);
            const uint32_t byte = mm >= thr ? 0u : (mm < 255 ? uint32_t(mm) : 255u);
            const uint32_t sh = 16 * (q & 1) + (side ? 0 : 8);
            ob[q >> 1] = (ob[q >> 1] & ~(0xFFu << sh)) | (byte << sh);
          }
          ++fb;
        }
      }
    }
    if (out && ib < i1) {
      uint8_t *o = out + g.out_off + 2 * (ib - i0);
      if (ib + kMPer <= i1) {   // 32 bytes (the caller's pointer need not be aligned)
        __builtin_memcpy(o, ob, 32);
      } else {
        for (uint32_t q = 0; q < uint32_t(i1 - ib); ++q) {
          o[2 * q] = uint8_t(ob[q >> 1] >> (16 * (q & 1)));
          o[2 * q + 1] = uint8_t(ob[q >> 1] >> (16 * (q & 1) + 8));
        }
      }
    }
    }   // sub-tiles
    if (mine) atomicAdd(&s_tot[par], mine);
    __syncthreads();
    // flush this tile's buffer and clear it for tile T + 2 gridDim.x (the
    // next tile counts into the other one; every thread passes the next
    // tile's barrier, after these clears, before it counts into this one)
    if (threadIdx.x <= kLdsBins) {
      const unsigned long long v = sbin[threadIdx.x];
      if (binned && v) {
        const uint32_t o = o0 + threadIdx.x;   // ordinal o counts into bin o - 1 (0: the last)
        atomicAdd(&bin_counts[o == 0 ? c.nbins - 1 : o - 1], v);
      }
      sbin[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0 && contig_count) {
      if (g.contig != run_contig) {
        if (run_tot) atomicAdd(contig_counts + run_contig, run_tot);
        run_tot = 0;
        run_contig = g.contig;
      }
      run_tot += s_tot[par];
    }
    if (threadIdx.x == 0) s_tot[par] = 0;
    cur = nxt;
  }
  if (threadIdx.x == 0 && run_tot) atomicAdd(contig_counts + run_contig, run_tot);
}

// settle the listed bytes: exact m, zeroed at its threshold, else min(m, 255)
template <class IdxT>
__global__ void k_mapfix(MapCtx c, const IdxT *__restrict__ ISA, uint8_t *out) {
  const uint64_t n = *c.nfix < c.fix_cap ? *c.nfix : c.fix_cap;
  for (uint64_t e = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; e < n;
       e += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t m = min_len_at(c, uint64_t(ISA[c.fix[3 * e]]) & c.pm);
    out[c.fix[3 * e + 1]] = uint8_t(m >= c.fix[3 * e + 2] ? 0 : (m < 255 ? m : 255));
  }
}

template <class IdxT>
int scan_t(const smash_index *ix, uint64_t begin, uint64_t end, uint32_t k, uint8_t *out,
           const int64_t *h_chrom_off, const int64_t *d_bins, uint32_t nbins,
           uint64_t *d_bin_counts, uint64_t *d_contig_counts, hipStream_t s) {
  MapCtx c;
  c.L8 = ix->d_lcp8;
  c.ovf = ix->d_ovf;
  c.n_ovf = ix->n_ovf;
  c.N = ix->N;
  c.bins = d_bins;
  c.nbins = d_bins ? nbins : 0;
  c.k = k;
  c.fix = nullptr;
  c.nfix = nullptr;
  c.fix_cap = 0;
  c.pm = ix->pos_mask;
  if (out && k < 255) {
    SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&c.fix), 24 * kFixCap, s));
    SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&c.nfix), 8, s));
    SMASH_HIP(hipMemsetAsync(c.nfix, 0, 8, s));
    c.fix_cap = kFixCap;
  }
  // the directory of unsaturated U positions, once per index (unless
  // smash_mappability_prepare built it): first one per 4096 positions, then
  // the suffix minimum (12 MB at hg19)
  const uint64_t ndir = (ix->N + (uint64_t(1) << kDirShift) - 1) >> kDirShift;
  if (!ix->d_nsdir) SMASH_HIP(build_nsdir(ix, 0, ix->N, s));
  // the register budget: 5 waves per SIMD (96 VGPRs, a few spilled) with
  // the U blocks loaded in their own trip beat the compiler's choice (3
  // waves at 150+ VGPRs) with them fetched a trip ahead: 6.9 vs 8.5 ms
  // over hg19 (profiles/r04/c5waves).  SMASH_MAPSCAN_WAVES (A/B): 0 (the
  // compiler's choice), 4, 5 or 6, a trailing 'n' = no fetch a trip ahead.
  // Sub-tiles: the tile's fixed work once per 16 x 4 096 bases cut the scan
  // from 6.9 to ~4.3 ms (profiles/r04/c5sub).  SMASH_MAPSCAN_SUB (A/B): 1,
  // 2, 4, 8, 16 or 32 sub-tiles per tile at 5 waves without the fetch
  // ahead; the other budgets take 1
  const char *ev = getenv("SMASH_MAPSCAN_WAVES");
  if (!ev || !*ev) ev = "5n";
  const int wv = atoi(ev);
  const bool pf = !strchr(ev, 'n');
  const char *es = getenv("SMASH_MAPSCAN_SUB");
  int sub = es && *es ? atoi(es) : 16;
  if (pf || wv != 5 || (sub != 2 && sub != 4 && sub != 8 && sub != 16 && sub != 32)) sub = 1;
  const uint64_t tile = kMTile * uint64_t(sub);
  // the segments of [begin, end): one per contig part, tiles numbered across
  std::vector<Seg> segs;
  uint64_t ntiles = 0, g0 = 0;
  for (uint32_t q = 0; q < ix->n_seq; q += 2) {
    const uint64_t S = ix->sizes[q];
    const uint64_t a = begin > g0 ? begin - g0 : 0;
    const uint64_t b = end < g0 + S ? end - g0 : S;
    if (a < b && g0 < end) {
      Seg sg;
      sg.sp = ix->startpos[q]; sg.S = S; sg.i0 = a; sg.i1 = b;
      sg.out_off = 2 * (g0 + a - begin);
      sg.tile0 = ntiles;
      sg.abs0 = h_chrom_off ? h_chrom_off[q / 2] : -1;
      sg.contig = q / 2;
      segs.push_back(sg);
      ntiles += (b - a + tile - 1) / tile;
    }
    g0 += S;
  }
  uint32_t *d_o0 = nullptr;
  Seg *d_segs = nullptr;
  if (!segs.empty()) {
    SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&d_segs), sizeof(Seg) * segs.size(), s));
    SMASH_HIP(hipMemcpyAsync(d_segs, segs.data(), sizeof(Seg) * segs.size(), hipMemcpyHostToDevice,
                             s));
    SMASH_HIP(hipStreamSynchronize(s));   // segs is a host local: copied before the launches
    SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&d_o0), 4 * ntiles, s));
    const uint32_t nseg = uint32_t(segs.size());
    if (c.nbins) {
      k_tilebins<<<unsigned((ntiles + 255) / 256), 256, 0, s>>>(c, d_segs, nseg, ntiles, tile, d_o0);
      SMASH_HIP(hipGetLastError());
    }
    int cus = 0;
    SMASH_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix->device));
    // resident blocks only: the tiles are dealt block-stride, so a block that
    // is not resident from the start waits for a whole block's share of the
    // tiles (the occupancy query, not a fixed cus * 8)
    const IdxT *isa = static_cast<const IdxT *>(ix->d_isa);
    auto *bcp = reinterpret_cast<unsigned long long *>(d_bin_counts);
    auto *ccp = reinterpret_cast<unsigned long long *>(d_contig_counts);
    auto launch = [&](auto kfn) -> hipError_t {
      int per_cu = 0;
      hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, reinterpret_cast<const void *>(kfn), kMB, 0);
      if (e != hipSuccess) return e;
      if (per_cu < 1) per_cu = 1;
      const uint64_t grid = std::min<uint64_t>(ntiles, uint64_t(cus) * uint64_t(per_cu));
      kfn<<<unsigned(grid), kMB, 0, s>>>(c, isa, ix->d_uniq, ix->d_nsdir, ndir, d_segs, nseg,
                                         ntiles, out, d_o0, bcp, ccp);
      return hipGetLastError();
    };
    hipError_t le;
    if (wv == 5 && !pf && sub == 2) le = launch(k_mapscan<IdxT, 5, false, 2>);
    else if (wv == 5 && !pf && sub == 4) le = launch(k_mapscan<IdxT, 5, false, 4>);
    else if (wv == 5 && !pf && sub == 8) le = launch(k_mapscan<IdxT, 5, false, 8>);
    else if (wv == 5 && !pf && sub == 16) le = launch(k_mapscan<IdxT, 5, false, 16>);
    else if (wv == 5 && !pf && sub == 32) le = launch(k_mapscan<IdxT, 5, false, 32>);
    else if (wv == 4) le = pf ? launch(k_mapscan<IdxT, 4, true, 1>) : launch(k_mapscan<IdxT, 4, false, 1>);
    else if (wv == 5) le = pf ? launch(k_mapscan<IdxT, 5, true, 1>) : launch(k_mapscan<IdxT, 5, false, 1>);
    else if (wv == 6) le = pf ? launch(k_mapscan<IdxT, 6, true, 1>) : launch(k_mapscan<IdxT, 6, false, 1>);
    else le = pf ? launch(k_mapscan<IdxT, 1, true, 1>) : launch(k_mapscan<IdxT, 1, false, 1>);
    SMASH_HIP(le);
  }
  if (d_segs) SMASH_HIP(hipFreeAsync(d_segs, s));
  if (d_o0) SMASH_HIP(hipFreeAsync(d_o0, s));
  if (c.fix) {
    k_mapfix<IdxT><<<4096, 256, 0, s>>>(c, static_cast<const IdxT *>(ix->d_isa), out);
    SMASH_HIP(hipGetLastError());
    SMASH_HIP(hipFreeAsync(c.fix, s));
    SMASH_HIP(hipFreeAsync(c.nfix, s));
  }
  return SMASH_OK;
}

}  // namespace
}  // namespace smash

using namespace smash;

extern "C" int smash_mappability_scan(const smash_index *ix, uint64_t begin, uint64_t end,
                                      uint32_t k, uint8_t *d_map_out,
                                      const int64_t *h_chrom_off, const int64_t *d_bin_starts,
                                      uint32_t nbins, uint64_t *d_bin_counts,
                                      uint64_t *d_contig_counts, void *stream) {
  if (!ix || end < begin || (d_bin_starts && (nbins == 0 || !d_bin_counts))) {
    set_error("smash_mappability_scan: bad arguments");
    return SMASH_ERR_ARG;
  }
  if (!ix->rcref) {   // mummer.cpp:145-146
    set_error("smash_mappability_scan: -mappability requires -rcref");
    return SMASH_ERR_ARG;
  }
  uint64_t total = 0;
  for (uint32_t q = 0; q < ix->n_seq; q += 2) total += ix->sizes[q];
  if (end > total) {
    set_error("smash_mappability_scan: range past the last forward base");
    return SMASH_ERR_ARG;
  }
  if (begin == end) return SMASH_OK;
  if (!ix->d_uniq) {
    set_error("smash_mappability_scan: index lacks U (aux_build)");
    return SMASH_ERR_ARG;
  }
  SMASH_HIP(hipSetDevice(ix->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (ix->idx_bytes == 4)
    return scan_t<uint32_t>(ix, begin, end, k, d_map_out, h_chrom_off, d_bin_starts, nbins,
                            d_bin_counts, d_contig_counts, s);
  return scan_t<uint64_t>(ix, begin, end, k, d_map_out, h_chrom_off, d_bin_starts, nbins,
                          d_bin_counts, d_contig_counts, s);
}

// The text window the scan of forward bases [begin, end) reads U in: every
// contig piece's forward positions and their reverse-complement positions
// (sp + 2S - i, longSA.cpp:667), with a 4 096-position margin (the scan's
// neighbouring-chunk loads and directory tiles)
static void scan_window(const smash_index *ix, uint64_t begin, uint64_t end, uint64_t *lo,
                        uint64_t *hi) {
  uint64_t a0 = ~0ull, b0 = 0, g0 = 0;
  for (uint32_t q = 0; q < ix->n_seq; q += 2) {
    const uint64_t S = ix->sizes[q], sp = ix->startpos[q];
    const uint64_t a = begin > g0 ? begin - g0 : 0;
    const uint64_t b = end < g0 + S ? end - g0 : S;
    if (a < b && g0 < end) {
      a0 = std::min(a0, sp + a);
      b0 = std::max(b0, sp + 2 * S - a + 1);
    }
    g0 += S;
  }
  const uint64_t m = uint64_t(1) << kDirShift;
  *lo = a0 == ~0ull ? 0 : (a0 > m ? a0 - m : 0);
  *hi = a0 == ~0ull ? 0 : std::min(ix->N, b0 + m);
}

extern "C" int smash_mappability_prepare(const smash_index *ix, uint64_t begin, uint64_t end,
                                         void *stream) {
  if (!ix || end < begin || !ix->rcref || !ix->d_uniq) {
    set_error("smash_mappability_prepare: bad arguments (or an index without -rcref / U)");
    return SMASH_ERR_ARG;
  }
  uint64_t total = 0;
  for (uint32_t q = 0; q < ix->n_seq; q += 2) total += ix->sizes[q];
  if (end > total) {
    set_error("smash_mappability_prepare: range past the last forward base");
    return SMASH_ERR_ARG;
  }
  if (begin == end) return SMASH_OK;
  SMASH_HIP(hipSetDevice(ix->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint64_t lo = 0, hi = 0;
  scan_window(ix, begin, end, &lo, &hi);
  try {
    build_uniq_range(const_cast<smash_index *>(ix), lo, hi, s);
  } catch (hip_failure &f) {
    set_error(f.what);
    return f.what.find("hipMalloc") != std::string::npos ? SMASH_ERR_NOMEM : SMASH_ERR_HIP;
  }
  SMASH_HIP(build_nsdir(ix, lo & ~uint64_t(63), hi, s));
  return SMASH_OK;
}

extern "C" int smash_mappability_release(const smash_index *ix) {
  if (!ix) return SMASH_ERR_ARG;
  SMASH_HIP(hipSetDevice(ix->device));
  SMASH_HIP(hipDeviceSynchronize());
  release_uniq_scratch(const_cast<smash_index *>(ix));
  return SMASH_OK;
}

extern "C" int smash_mappability_window(const smash_index *ix, uint64_t begin, uint64_t end,
                                        uint64_t *lo, uint64_t *hi) {
  if (!ix || !lo || !hi || end < begin) return SMASH_ERR_ARG;
  scan_window(ix, begin, end, lo, hi);
  *lo &= ~uint64_t(63);
  return SMASH_OK;
}
