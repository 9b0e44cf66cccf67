// smash-paper_amd/csrc/uniq_build.hip -- U from the suffix array, by
// partitioning instead of gathering (round 5).
//
//   U[x] = min(255, max(LCP[ISA[x]], LCP[ISA[x] + 1]))
//
// is the per-position minimum-unique length of longSA::show before its edge
// rules (longSA.cpp:628-641: m[r] = max(LCP[r], LCP[r + 1]) + 1, read at
// ISA[pos], :666-667); the search (accelerator B) and the C5 scan read it.
// Read in rank order it is a stream: v(r) = max(L8[r], L8[r + 1]) belongs at
// text position SA[r].  The gather form (k_uniq_gather: one random L8 line per
// position, 143 ms over hg19's 6.19 G positions, at the random-line rate)
// is replaced by a scatter in three streaming passes whose destinations are
// known in advance -- SA is a permutation, so every aligned window of 2^k
// positions receives exactly 2^k entries:
//
//   pass 1 (k_upart1): ranks in tiles (round 6: 16 384); each entry {x mod 2^24, v}
//     (one u32) goes to the level-1 bucket of x >> 24; a tile is sorted by
//     bucket in LDS and each bucket's run is stored contiguously at an
//     atomically claimed offset inside the bucket's fixed slice of E1 (u32
//     per position).  Reads SA (8 B) + L8 (1 B), writes 4 B.
//   pass 2 (k_upart2): a chunk of level-1 buckets at a time, each entry to
//     its 2^16-position window ((x >> 16) & 255) in the same way (E2, one
//     chunk of 32 buckets = 2 GB).  Reads 4 B, writes 4 B.
//   pass 3 (k_upart3): one block per window: its 65 536 entries land as
//     bytes in 64 KB of LDS, and the window of U is stored with 16-byte
//     stores.  Reads 4 B, writes 1 B.
//
// 22 B of HBM traffic per position, all of it streaming, against one random
// 64-byte line per position for the gather.  Windows past 2^33 positions
// (the u32 entry holds 24 position bits) fall back to the gather.
//
// Round 6: passes 1 and 2 were latency-bound (2.7 and 2.0 TB/s): a tile's
// loads, its LDS placement and its run stores ran one after the other with
// two blocks per CU.  Now each lane loads whole vectors (a pair of SA
// elements + their LCP bytes, four E1 entries) and the next tile's loads
// are issued before the current tile is placed; the tiles are 16 384
// entries in one 1024-thread block per CU (runs twice as long as with
// 8 192; SMASH_UPART_NT / _NT2=512 for the two-block form).
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "common.hpp"

namespace smash {
namespace {

constexpr int kUT = 512;                         // threads per block of the 8 192-entry form
constexpr int kUPer = 16;                        // entries per thread per tile
constexpr uint32_t kUTile = uint32_t(kUT) * kUPer;   // 8 192: 54 KB of LDS, 2 blocks per CU
constexpr int kU3 = 1024;                        // threads per block (pass 3)
constexpr uint32_t kNB1Max = 512;                // level-1 buckets
constexpr uint32_t kNB2 = 256;                   // windows per level-1 bucket (S1 - S2 = 8)

__host__ __device__ inline uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

template <class IdxT>
__global__ void k_uniq_gather(const IdxT *__restrict__ ISA, uint64_t pm,
                              const uint8_t *__restrict__ L8, uint64_t N, uint64_t lo,
                              uint64_t hi, uint8_t *U) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t x = lo + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; x < hi; x += stride) {
    const uint64_t r = uint64_t(ISA[x]) & pm;
    const uint8_t a = L8[r];
    const uint8_t b = r + 1 < N ? L8[r + 1] : 0;
    U[x] = a > b ? a : b;
  }
}

// The block's tile sorted by bucket in LDS, then each bucket's run stored at
// its claimed offset: dst(b) + claimed + rank in run.  nb <= kNB1Max.
// ent[] / bk[] (bk = 0xFFFF: no entry) are the thread's entries.
template <int NT>
struct TileLds {
  uint32_t cnt[kNB1Max];
  uint32_t off[kNB1Max + 1];
  uint32_t gb[kNB1Max];
  uint32_t ent[NT * kUPer];
  uint16_t bk[NT * kUPer];
};

// exclusive scan of cnt[0..nb) into off[0..nb] (block-wide, nb <= 1024)
template <int NT>
__device__ __forceinline__ void block_excl_scan(TileLds<NT> &t, uint32_t nb) {
  __shared__ uint32_t s_w[NT / 64];
  const uint32_t i = threadIdx.x, lane = i & 63, w = i >> 6;
  uint32_t x = i < nb ? t.cnt[i] : 0u, inc = x;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (lane >= uint32_t(d)) inc += y;
  }
  if (lane == 63) s_w[w] = inc;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t v = 0; v < w; ++v) before += s_w[v];
  if (i < nb) t.off[i] = before + inc - x;
  if (i == nb - 1) t.off[nb] = before + inc;
  __syncthreads();
}

// rank-local part of one tile: claim each bucket's run, place the entries
// in LDS by bucket, store the runs (dst: slice base of bucket b in elements).
// The runs' global claims are issued before the LDS placement, so their
// round trip overlaps it.
template <int NT, class Dst>
__device__ __forceinline__ void tile_scatter(TileLds<NT> &t, uint32_t nb, const uint32_t (&ent)[kUPer],
                                             uint32_t (&bk)[kUPer], unsigned int *cur,
                                             Dst dst, uint32_t *out) {
  // bk[k] becomes bucket << 16 | rank in the bucket's run (0xFFFF: no entry)
#pragma unroll
  for (int k = 0; k < kUPer; ++k)
    if (bk[k] != 0xFFFF) bk[k] = (bk[k] << 16) | atomicAdd(&t.cnt[bk[k]], 1u);
  __syncthreads();
  block_excl_scan(t, nb);
  for (uint32_t b = threadIdx.x; b < nb; b += NT)
    t.gb[b] = t.cnt[b] ? atomicAdd(&cur[b], t.cnt[b]) : 0u;
#pragma unroll
  for (int k = 0; k < kUPer; ++k)
    if (bk[k] != 0xFFFF) {
      const uint32_t b = bk[k] >> 16;
      const uint32_t j = t.off[b] + (bk[k] & 0xFFFF);
      t.ent[j] = ent[k];
      t.bk[j] = uint16_t(b);
    }
  __syncthreads();
  const uint32_t total = t.off[nb];
  for (uint32_t j = threadIdx.x; j < total; j += NT) {
    const uint32_t b = t.bk[j];
    out[dst(b) + t.gb[b] + (j - t.off[b])] = t.ent[j];
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += NT) t.cnt[b] = 0;
  __syncthreads();
}

// two consecutive SA elements as one load (8 or 16 bytes)
template <class IdxT> struct Pair2;
template <> struct Pair2<uint64_t> { using V = ulong2; };
template <> struct Pair2<uint32_t> { using V = uint2; };

// a thread's share of one pass-1 tile as loaded: rank pairs p = k * kUT +
// thread (k < kUPer / 2), each instruction reads 64 consecutive pairs
template <class IdxT>
struct P1Raw {
  typename Pair2<IdxT>::V sa[kUPer / 2];
  uint16_t l2[kUPer / 2];   // L8[2p], L8[2p + 1]
  uint8_t l3[kUPer / 2];    // L8[2p + 2] (0 past the end)
};

template <class IdxT, int NT>
__device__ __forceinline__ void p1_load(const IdxT *__restrict__ SA, const uint8_t *__restrict__ L8,
                                        uint64_t N, uint64_t tile, P1Raw<IdxT> &w) {
  const uint64_t r0 = tile * (NT * kUPer);
  if (r0 + NT * kUPer < N) {   // (block-uniform) every rank and L8[r + 1] in range
#pragma unroll
    for (int k = 0; k < kUPer / 2; ++k) {
      const uint64_t r = r0 + 2 * (uint64_t(k) * NT + threadIdx.x);
      w.sa[k] = *reinterpret_cast<const typename Pair2<IdxT>::V *>(SA + r);
      w.l2[k] = *reinterpret_cast<const uint16_t *>(L8 + r);
      w.l3[k] = L8[r + 2];
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < kUPer / 2; ++k) {
    const uint64_t r = r0 + 2 * (uint64_t(k) * NT + threadIdx.x);
    w.sa[k].x = r < N ? SA[r] : IdxT(0);
    w.sa[k].y = r + 1 < N ? SA[r + 1] : IdxT(0);
    w.l2[k] = uint16_t((r < N ? L8[r] : 0) | ((r + 1 < N ? L8[r + 1] : 0) << 8));
    w.l3[k] = r + 2 < N ? L8[r + 2] : uint8_t(0);
  }
}

// pass 1: ranks -> level-1 buckets (2^S1 positions) of the window [lo, hi);
// the next tile's loads are in flight while this one is placed
template <class IdxT, int S1, int NT>
__global__ __launch_bounds__(NT, 2048 / NT) void k_upart1(const IdxT *__restrict__ SA, uint64_t pm,
                                                const uint8_t *__restrict__ L8, uint64_t N,
                                                uint64_t lo, uint64_t hi, uint32_t nb,
                                                unsigned int *cur, uint32_t *E1) {
  static_assert(S1 <= 24, "an entry holds 24 position bits and the 8-bit value");
  constexpr uint32_t kTile = NT * kUPer;
  __shared__ TileLds<NT> t;
  for (uint32_t b = threadIdx.x; b < nb; b += NT) t.cnt[b] = 0;
  __syncthreads();
  const uint64_t ntiles = (N + kTile - 1) / kTile;
  uint64_t tile = blockIdx.x;
  P1Raw<IdxT> w;
  if (tile < ntiles) p1_load<IdxT, NT>(SA, L8, N, tile, w);
  for (; tile < ntiles; tile += gridDim.x) {
    uint32_t ent[kUPer];
    uint32_t bk[kUPer];
#pragma unroll
    for (int k = 0; k < kUPer / 2; ++k) {
      const uint64_t r = tile * kTile + 2 * (uint64_t(k) * NT + threadIdx.x);
      const uint32_t a = w.l2[k] & 0xFF, b = w.l2[k] >> 8, c = w.l3[k];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint64_t x = uint64_t(h ? w.sa[k].y : w.sa[k].x) & pm;
        const uint32_t v = h ? (b > c ? b : c) : (a > b ? a : b);
        const bool in = r + h < N && x >= lo && x < hi;
        bk[2 * k + h] = in ? uint32_t((x - lo) >> S1) : 0xFFFFu;
        ent[2 * k + h] = uint32_t((x - lo) & ((1u << S1) - 1)) | (v << 24);
      }
    }
    if (tile + gridDim.x < ntiles) p1_load<IdxT, NT>(SA, L8, N, tile + gridDim.x, w);
    tile_scatter(t, nb, ent, bk, cur, [](uint32_t b) { return uint64_t(b) << S1; }, E1);
  }
}

// pass 2: level-1 buckets [c0, c0 + nc) -> their windows of 2^S2 positions
// (E2 chunk-local); entries read 4 per lane per load, the next tile's in
// flight while this one is placed
template <int S1, int S2, int NT>
__global__ __launch_bounds__(NT, 2048 / NT) void k_upart2(const uint32_t *__restrict__ E1, uint64_t n,
                                                uint32_t c0, uint32_t nc, unsigned int *cur,
                                                uint32_t *E2) {
  static_assert(S1 - S2 == 8, "256 windows per level-1 bucket");
  constexpr uint32_t kTile = NT * kUPer;
  __shared__ TileLds<NT> t;
  const uint64_t tpb = (uint64_t(1) << S1) / kTile;   // tiles per bucket
  const uint64_t ntiles = uint64_t(nc) * tpb;
  for (uint32_t b = threadIdx.x; b < kNB2; b += NT) t.cnt[b] = 0;
  __syncthreads();
  // a tile is live when it starts inside its bucket (block-uniform)
  auto live = [&](uint64_t tile, uint64_t &bbeg, uint64_t &bsize) {
    const uint64_t b = c0 + tile / tpb;
    bbeg = b << S1;
    bsize = umin64(uint64_t(1) << S1, n - bbeg);
    return (tile % tpb) * kTile < bsize;
  };
  auto load = [&](uint64_t tile, uint4 (&v)[kUPer / 4]) {
    uint64_t bbeg, bsize;
    live(tile, bbeg, bsize);
    const uint64_t e0 = (tile % tpb) * kTile;
#pragma unroll
    for (int k = 0; k < kUPer / 4; ++k) {
      const uint64_t e = e0 + 4 * (uint64_t(k) * NT + threadIdx.x);
      if (e + 4 <= bsize) {
        v[k] = *reinterpret_cast<const uint4 *>(E1 + bbeg + e);
      } else {
        v[k].x = e < bsize ? E1[bbeg + e] : 0u;
        v[k].y = e + 1 < bsize ? E1[bbeg + e + 1] : 0u;
        v[k].z = e + 2 < bsize ? E1[bbeg + e + 2] : 0u;
        v[k].w = e + 3 < bsize ? E1[bbeg + e + 3] : 0u;
      }
    }
  };
  auto next_live = [&](uint64_t tile) {
    uint64_t bbeg, bsize;
    while (tile < ntiles && !live(tile, bbeg, bsize)) tile += gridDim.x;
    return tile;
  };
  uint4 v[kUPer / 4];
  uint64_t tile = next_live(blockIdx.x);
  if (tile < ntiles) load(tile, v);
  while (tile < ntiles) {
    uint64_t bbeg, bsize;
    live(tile, bbeg, bsize);
    const uint32_t bl = uint32_t(tile / tpb);   // chunk-local bucket
    const uint64_t e0 = (tile % tpb) * kTile;
    uint32_t ent[kUPer];
    uint32_t bk[kUPer];
#pragma unroll
    for (int k = 0; k < kUPer / 4; ++k) {
      const uint64_t e = e0 + 4 * (uint64_t(k) * NT + threadIdx.x);
      const uint32_t q[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        ent[4 * k + h] = q[h];
        bk[4 * k + h] = e + h < bsize ? (q[h] >> S2) & (kNB2 - 1) : 0xFFFFu;
      }
    }
    const uint64_t nxt = next_live(tile + gridDim.x);
    if (nxt < ntiles) load(nxt, v);
    tile_scatter(t, kNB2, ent, bk, cur + uint64_t(bl) * kNB2,
                 [bl](uint32_t w) { return (uint64_t(bl) << S1) + (uint64_t(w) << S2); }, E2);
    tile = nxt;
  }
}

// pass 3: one block per window of 2^S2 positions: entries -> LDS bytes -> U
template <int S1, int S2>
__global__ __launch_bounds__(kU3) void k_upart3(const uint32_t *__restrict__ E2, uint64_t n,
                                                uint32_t c0, uint32_t nc, uint64_t lo,
                                                uint8_t *U) {
  __shared__ uint32_t s_u[(1u << S2) / 4];
  uint8_t *sb = reinterpret_cast<uint8_t *>(s_u);
  constexpr uint32_t kM = (1u << S2) - 1;
  const uint64_t nwin = uint64_t(nc) * kNB2;
  for (uint64_t w = blockIdx.x; w < nwin; w += gridDim.x) {
    const uint64_t wbeg = (uint64_t(c0) << S1) + (w << S2);   // window-relative position
    if (wbeg >= n) continue;                                     // (block-uniform)
    const uint32_t wsize = uint32_t(umin64(uint64_t(1) << S2, n - wbeg));
    const uint32_t *src = E2 + (w << S2);
    for (uint32_t j = threadIdx.x * 4; j < wsize; j += kU3 * 4) {
      if (j + 4 <= wsize) {
        const uint4 v = *reinterpret_cast<const uint4 *>(src + j);
        sb[v.x & kM] = uint8_t(v.x >> 24);
        sb[v.y & kM] = uint8_t(v.y >> 24);
        sb[v.z & kM] = uint8_t(v.z >> 24);
        sb[v.w & kM] = uint8_t(v.w >> 24);
      } else {
        for (uint32_t q = j; q < wsize; ++q) sb[src[q] & kM] = uint8_t(src[q] >> 24);
      }
    }
    __syncthreads();
    uint8_t *dst = U + lo + wbeg;   // lo is a multiple of 64: 16-byte aligned stores
    for (uint32_t j = threadIdx.x * 16; j < wsize; j += kU3 * 16) {
      if (j + 16 <= wsize) {
        *reinterpret_cast<uint4 *>(dst + j) = *reinterpret_cast<const uint4 *>(sb + j);
      } else {
        for (uint32_t q = j; q < wsize; ++q) dst[q] = sb[q];
      }
    }
    __syncthreads();
  }
}

template <class IdxT, int S1, int S2>
void uniq_range_g(smash_index *ix, uint64_t lo, uint64_t hi, hipStream_t s) {
  const uint64_t N = ix->N;
  const uint64_t n = hi - lo;
  const uint32_t nb1 = uint32_t((n + (uint64_t(1) << S1) - 1) >> S1);
  int cus = 0;
  SMASH_HIPX(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix->device));
  // scratch: E1 (4 B per window position), E2 (one chunk of level-1 buckets,
  // SMASH_UPART_E2MB, default 2 GB), the cursors -- kept in the index between
  // calls (release_uniq_scratch)
  uint64_t e2mb = 2048;
  if (const char *e = getenv("SMASH_UPART_E2MB")) e2mb = std::max<uint64_t>(1, strtoull(e, 0, 10));
  const uint32_t kc = uint32_t(std::max<uint64_t>(1, (e2mb << 18) >> S1));   // buckets per chunk
  const uint32_t chunk = std::min(kc, nb1);
  // SMASH_UPART_2S=1: the chunks alternate between the caller's stream and
  // a second one, each with its own E2 and cursors, so one chunk's pass 2
  // runs beside the other's pass 3 (prepare 39.8-42.2 vs 41.4-43.5 ms at
  // hg19 on two boxes, profiles/r06/upart4).  Off by default: two of its
  // fourteen C5 lines there had one rep whose scan took ~1.2 s longer (the
  // GPU idle between the scan's events), never seen with one stream.
  const char *ts = getenv("SMASH_UPART_2S");
  const bool two = ts && ts[0] == '1' && nb1 > chunk;
  const uint64_t b_e1 = (4 * n + 255) & ~uint64_t(255);
  const uint64_t b_e2 = 4 * (uint64_t(chunk) << S1);
  const uint64_t b_cur = (4 * uint64_t(std::max(chunk * kNB2, nb1)) + 255) & ~uint64_t(255);
  const uint64_t need = b_e1 + (two ? 2 : 1) * (b_e2 + b_cur);
  if (ix->uscratch_bytes < need) {
    release_uniq_scratch(ix);
    ix->d_uscratch = dalloc<uint8_t>(need);
    ix->uscratch_bytes = need;
  }
  if (two && !ix->uaux) {
    SMASH_HIPX(hipStreamCreateWithFlags(&ix->uaux, hipStreamNonBlocking));
    for (int q = 0; q < 2; ++q)
      SMASH_HIPX(hipEventCreateWithFlags(&ix->uev[q], hipEventDisableTiming));
  }
  uint32_t *E1 = reinterpret_cast<uint32_t *>(ix->d_uscratch);
  // [E1][E2 | cursors] (+ [E2 | cursors] of the second stream)
  uint32_t *E2s[2] = {reinterpret_cast<uint32_t *>(ix->d_uscratch + b_e1),
                      reinterpret_cast<uint32_t *>(ix->d_uscratch + b_e1 + b_e2 + b_cur)};
  unsigned int *curs[2] = {
      reinterpret_cast<unsigned int *>(ix->d_uscratch + b_e1 + b_e2),
      reinterpret_cast<unsigned int *>(ix->d_uscratch + b_e1 + 2 * b_e2 + b_cur)};
  unsigned int *cur = curs[0];
  SMASH_HIPX(hipMemsetAsync(cur, 0, 4 * nb1, s));
  // SMASH_UPART_NT=512: pass-1 tiles of 8 192 ranks (two blocks per CU)
  // instead of 16 384 (one block per CU, runs twice as long: 21.5 vs 23.5 ms
  // at hg19, profiles/r06/upart2); SMASH_UPART_NT2 likewise for pass 2
  const char *nt = getenv("SMASH_UPART_NT");
  const char *nt2e = getenv("SMASH_UPART_NT2");
  const int nt2 = nt2e ? atoi(nt2e) : 1024;
  if (!(nt && atoi(nt) == 512)) {
    const uint64_t t1 = (N + 1024 * kUPer - 1) / (1024 * kUPer);
    k_upart1<IdxT, S1, 1024><<<unsigned(std::min<uint64_t>(t1, uint64_t(cus))), 1024, 0, s>>>(
        static_cast<const IdxT *>(ix->d_sa), ix->pos_mask, ix->d_lcp8, N, lo, hi, nb1, cur, E1);
  } else {
    const uint64_t t1 = (N + kUTile - 1) / kUTile;
    k_upart1<IdxT, S1, kUT><<<unsigned(std::min<uint64_t>(t1, 2 * uint64_t(cus))), kUT, 0, s>>>(
        static_cast<const IdxT *>(ix->d_sa), ix->pos_mask, ix->d_lcp8, N, lo, hi, nb1, cur, E1);
  }
  SMASH_HIPX(hipGetLastError());
  const unsigned per_cu3 = (1u << S2) > 65536 ? 1u : 2u;   // LDS: one window per block
  if (two) {   // the second stream starts after pass 1
    SMASH_HIPX(hipEventRecord(ix->uev[0], s));
    SMASH_HIPX(hipStreamWaitEvent(ix->uaux, ix->uev[0], 0));
  }
  for (uint32_t c0 = 0, ci = 0; c0 < nb1; c0 += chunk, ++ci) {
    const uint32_t nc = std::min(chunk, nb1 - c0);
    const int h = two ? int(ci & 1) : 0;
    hipStream_t st = h ? ix->uaux : s;
    uint32_t *E2 = E2s[h];
    unsigned int *cc = curs[h];
    SMASH_HIPX(hipMemsetAsync(cc, 0, 4 * uint64_t(nc) * kNB2, st));
    if (nt2 == 1024) {
      const uint64_t t2 = uint64_t(nc) * ((uint64_t(1) << S1) / (1024 * kUPer));
      k_upart2<S1, S2, 1024><<<unsigned(std::min<uint64_t>(t2, uint64_t(cus))), 1024, 0, st>>>(
          E1, n, c0, nc, cc, E2);
    } else {
      const uint64_t t2 = uint64_t(nc) * ((uint64_t(1) << S1) / kUTile);
      k_upart2<S1, S2, kUT><<<unsigned(std::min<uint64_t>(t2, 2 * uint64_t(cus))), kUT, 0, st>>>(
          E1, n, c0, nc, cc, E2);
    }
    k_upart3<S1, S2><<<unsigned(std::min<uint64_t>(uint64_t(nc) * kNB2, uint64_t(cus) * per_cu3)),
                       kU3, 0, st>>>(E2, n, c0, nc, lo, ix->d_uniq);
    SMASH_HIPX(hipGetLastError());
  }
  if (two) {   // the caller's stream continues after both
    SMASH_HIPX(hipEventRecord(ix->uev[1], ix->uaux));
    SMASH_HIPX(hipStreamWaitEvent(s, ix->uev[1], 0));
  }
}

template <class IdxT>
void uniq_range_t(smash_index *ix, uint64_t lo, uint64_t hi, hipStream_t s) {
  const uint64_t n = hi - lo;
  const char *g = getenv("SMASH_UNIQ_GATHER");   // 1: the gather form (A/B)
  const uint32_t nb1 = uint32_t((n + (uint64_t(1) << 24) - 1) >> 24);
  if (nb1 > kNB1Max || (g && g[0] == '1')) {
    k_uniq_gather<IdxT><<<grid_for(n, 256, 1u << 20), 256, 0, s>>>(
        static_cast<const IdxT *>(ix->d_isa), ix->pos_mask, ix->d_lcp8, ix->N, lo, hi, ix->d_uniq);
    SMASH_HIPX(hipGetLastError());
    return;
  }
  uniq_range_g<IdxT, 24, 16>(ix, lo, hi, s);
}

}  // namespace

void release_uniq_scratch(smash_index *ix) {
  if (ix->uaux) {
    (void)hipStreamSynchronize(ix->uaux);
    (void)hipStreamDestroy(ix->uaux);
    ix->uaux = nullptr;
    for (int q = 0; q < 2; ++q) {
      (void)hipEventDestroy(ix->uev[q]);
      ix->uev[q] = nullptr;
    }
  }
  if (ix->d_uscratch) (void)hipFree(ix->d_uscratch);
  ix->d_uscratch = nullptr;
  ix->uscratch_bytes = 0;
}

// U for the text positions [lo, hi) (lo rounded down to a multiple of 64),
// in ix->d_uniq; the rest of U is left as it is
void build_uniq_range(smash_index *ix, uint64_t lo, uint64_t hi, hipStream_t s) {
  lo &= ~uint64_t(63);
  hi = std::min(hi, ix->N);
  if (lo >= hi) return;
  if (ix->idx_bytes == 4) uniq_range_t<uint32_t>(ix, lo, hi, s);
  else uniq_range_t<uint64_t>(ix, lo, hi, s);
}

}  // namespace smash
