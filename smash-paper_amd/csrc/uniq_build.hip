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
//   pass 1 (k_upart1): ranks in tiles of 8 192; each entry {x mod 2^24, v}
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
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "common.hpp"

namespace smash {
namespace {

constexpr int kUT = 512;                         // threads per block (passes 1, 2)
constexpr int kUPer = 16;                        // entries per thread per tile
constexpr uint32_t kUTile = uint32_t(kUT) * kUPer;   // 8 192: 54 KB of LDS, 2 blocks per CU
constexpr int kU3 = 1024;                        // threads per block (pass 3)
constexpr int kS1 = 24;                          // level-1 bucket: 2^24 positions
constexpr int kS2 = 16;                          // window: 2^16 positions
constexpr uint32_t kNB1Max = 512;                // level-1 buckets (2^33 positions)
constexpr uint32_t kNB2 = 1u << (kS1 - kS2);     // windows per bucket (256)
constexpr uint32_t kChunk = 32;                  // level-1 buckets per pass-2/3 chunk

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
struct TileLds {
  uint32_t cnt[kNB1Max];
  uint32_t off[kNB1Max + 1];
  uint32_t gb[kNB1Max];
  uint32_t ent[kUTile];
  uint16_t bk[kUTile];
};

// exclusive scan of cnt[0..nb) into off[0..nb] (block-wide, nb <= 1024)
__device__ __forceinline__ void block_excl_scan(TileLds &t, uint32_t nb) {
  __shared__ uint32_t s_w[kUT / 64];
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
// in LDS by bucket, store the runs (dst: slice base of bucket b in elements)
template <class Dst>
__device__ __forceinline__ void tile_scatter(TileLds &t, uint32_t nb, const uint32_t (&ent)[kUPer],
                                             const uint16_t (&bk)[kUPer], unsigned int *cur,
                                             Dst dst, uint32_t *out) {
  uint32_t slot[kUPer];
#pragma unroll
  for (int k = 0; k < kUPer; ++k)
    slot[k] = bk[k] != 0xFFFF ? atomicAdd(&t.cnt[bk[k]], 1u) : 0u;
  __syncthreads();
  block_excl_scan(t, nb);
  for (uint32_t b = threadIdx.x; b < nb; b += kUT)
    t.gb[b] = t.cnt[b] ? atomicAdd(&cur[b], t.cnt[b]) : 0u;
#pragma unroll
  for (int k = 0; k < kUPer; ++k)
    if (bk[k] != 0xFFFF) {
      const uint32_t j = t.off[bk[k]] + slot[k];
      t.ent[j] = ent[k];
      t.bk[j] = bk[k];
    }
  __syncthreads();
  const uint32_t total = t.off[nb];
  for (uint32_t j = threadIdx.x; j < total; j += kUT) {
    const uint32_t b = t.bk[j];
    out[dst(b) + t.gb[b] + (j - t.off[b])] = t.ent[j];
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += kUT) t.cnt[b] = 0;
  __syncthreads();
}

// pass 1: ranks -> level-1 buckets of the window [lo, hi)
template <class IdxT>
__global__ __launch_bounds__(kUT) void k_upart1(const IdxT *__restrict__ SA, uint64_t pm,
                                                const uint8_t *__restrict__ L8, uint64_t N,
                                                uint64_t lo, uint64_t hi, uint32_t nb,
                                                unsigned int *cur, uint32_t *E1) {
  __shared__ TileLds t;
  for (uint32_t b = threadIdx.x; b < nb; b += kUT) t.cnt[b] = 0;
  __syncthreads();
  const uint64_t ntiles = (N + kUTile - 1) / kUTile;
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // entry k of the thread: rank tile * kUTile + k * kUT + thread (each load
    // instruction reads 64 consecutive SA elements and LCP bytes)
    const uint64_t r0 = tile * kUTile + threadIdx.x;
    uint32_t ent[kUPer];
    uint16_t bk[kUPer];
#pragma unroll
    for (int k = 0; k < kUPer; ++k) {
      const uint64_t r = r0 + uint64_t(k) * kUT;
      bk[k] = 0xFFFF;
      ent[k] = 0;
      if (r < N) {
        const uint64_t x = uint64_t(SA[r]) & pm;
        const uint8_t a = L8[r], c = r + 1 < N ? L8[r + 1] : uint8_t(0);
        if (x >= lo && x < hi) {
          bk[k] = uint16_t((x - lo) >> kS1);
          ent[k] = uint32_t((x - lo) & ((1u << kS1) - 1)) | (uint32_t(a > c ? a : c) << 24);
        }
      }
    }
    tile_scatter(t, nb, ent, bk, cur, [](uint32_t b) { return uint64_t(b) << kS1; }, E1);
  }
}

// pass 2: level-1 buckets [c0, c0 + nc) -> their windows (E2 chunk-local)
__global__ __launch_bounds__(kUT) void k_upart2(const uint32_t *__restrict__ E1, uint64_t n,
                                                uint32_t c0, uint32_t nc, unsigned int *cur,
                                                uint32_t *E2) {
  __shared__ TileLds t;
  const uint64_t tiles_per_bucket = (uint64_t(1) << kS1) / kUTile;   // 2048
  const uint64_t ntiles = uint64_t(nc) * tiles_per_bucket;
  for (uint32_t b = threadIdx.x; b < kNB2; b += kUT) t.cnt[b] = 0;
  __syncthreads();
  for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint32_t bl = uint32_t(tile / tiles_per_bucket);       // chunk-local bucket
    const uint64_t b = c0 + bl;
    const uint64_t bbeg = b << kS1;
    const uint64_t bsize = umin64(uint64_t(1) << kS1, n - bbeg);
    const uint64_t e0 = (tile % tiles_per_bucket) * kUTile + threadIdx.x;
    if ((tile % tiles_per_bucket) * kUTile >= bsize) continue;   // (block-uniform)
    uint32_t ent[kUPer];
    uint16_t bk[kUPer];
#pragma unroll
    for (int k = 0; k < kUPer; ++k) {   // (coalesced: entry k of the thread is e0 + k * kUT)
      const uint64_t e = e0 + uint64_t(k) * kUT;
      ent[k] = e < bsize ? E1[bbeg + e] : 0u;
      bk[k] = e < bsize ? uint16_t((ent[k] >> kS2) & (kNB2 - 1)) : uint16_t(0xFFFF);
    }
    tile_scatter(t, kNB2, ent, bk, cur + uint64_t(bl) * kNB2,
                 [bl](uint32_t w) { return (uint64_t(bl) << kS1) + (uint64_t(w) << kS2); }, E2);
  }
}

// pass 3: one block per window of 2^16 positions: entries -> LDS bytes -> U
__global__ __launch_bounds__(kU3) void k_upart3(const uint32_t *__restrict__ E2, uint64_t n,
                                                uint32_t c0, uint32_t nc, uint64_t lo,
                                                uint8_t *U) {
  __shared__ uint32_t s_u[(1u << kS2) / 4];
  uint8_t *sb = reinterpret_cast<uint8_t *>(s_u);
  const uint64_t nwin = uint64_t(nc) * kNB2;
  for (uint64_t w = blockIdx.x; w < nwin; w += gridDim.x) {
    const uint64_t wbeg = (uint64_t(c0) << kS1) + (w << kS2);   // window-relative position
    if (wbeg >= n) continue;                                     // (block-uniform)
    const uint32_t wsize = uint32_t(umin64(uint64_t(1) << kS2, n - wbeg));
    const uint32_t *src = E2 + (w << kS2);
    for (uint32_t j = threadIdx.x * 4; j < wsize; j += kU3 * 4) {
      if (j + 4 <= wsize) {
        const uint4 v = *reinterpret_cast<const uint4 *>(src + j);
        sb[v.x & 0xFFFF] = uint8_t(v.x >> 24);
        sb[v.y & 0xFFFF] = uint8_t(v.y >> 24);
        sb[v.z & 0xFFFF] = uint8_t(v.z >> 24);
        sb[v.w & 0xFFFF] = uint8_t(v.w >> 24);
      } else {
        for (uint32_t q = j; q < wsize; ++q) sb[src[q] & 0xFFFF] = uint8_t(src[q] >> 24);
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

template <class IdxT>
void uniq_range_t(smash_index *ix, uint64_t lo, uint64_t hi, hipStream_t s) {
  const uint64_t N = ix->N;
  const uint64_t n = hi - lo;
  const uint32_t nb1 = uint32_t((n + (uint64_t(1) << kS1) - 1) >> kS1);
  const char *e = getenv("SMASH_UNIQ_GATHER");   // 1: the gather form (A/B)
  if (nb1 > kNB1Max || (e && e[0] == '1')) {
    k_uniq_gather<IdxT><<<grid_for(n, 256, 1u << 20), 256, 0, s>>>(
        static_cast<const IdxT *>(ix->d_isa), ix->pos_mask, ix->d_lcp8, N, lo, hi, ix->d_uniq);
    SMASH_HIPX(hipGetLastError());
    return;
  }
  int cus = 0;
  SMASH_HIPX(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix->device));
  // scratch: E1 (4 B per window position), E2 (one chunk), the cursors --
  // kept in the index between calls (release_uniq_scratch)
  const uint32_t chunk = std::min(kChunk, nb1);
  const uint64_t b_e1 = (4 * n + 255) & ~uint64_t(255);
  const uint64_t b_e2 = 4 * (uint64_t(chunk) << kS1);
  const uint64_t need = b_e1 + b_e2 + 4 * uint64_t(kChunk) * kNB2;
  if (ix->uscratch_bytes < need) {
    release_uniq_scratch(ix);
    ix->d_uscratch = dalloc<uint8_t>(need);
    ix->uscratch_bytes = need;
  }
  uint32_t *E1 = reinterpret_cast<uint32_t *>(ix->d_uscratch);
  uint32_t *E2 = reinterpret_cast<uint32_t *>(ix->d_uscratch + b_e1);
  unsigned int *cur = reinterpret_cast<unsigned int *>(ix->d_uscratch + b_e1 + b_e2);
  SMASH_HIPX(hipMemsetAsync(cur, 0, 4 * nb1, s));
  const uint64_t t1 = (N + kUTile - 1) / kUTile;
  k_upart1<IdxT><<<unsigned(std::min<uint64_t>(t1, 2 * uint64_t(cus))), kUT, 0, s>>>(
      static_cast<const IdxT *>(ix->d_sa), ix->pos_mask, ix->d_lcp8, N, lo, hi, nb1, cur, E1);
  SMASH_HIPX(hipGetLastError());
  for (uint32_t c0 = 0; c0 < nb1; c0 += kChunk) {
    const uint32_t nc = std::min(kChunk, nb1 - c0);
    SMASH_HIPX(hipMemsetAsync(cur, 0, 4 * uint64_t(nc) * kNB2, s));
    const uint64_t t2 = uint64_t(nc) * ((uint64_t(1) << kS1) / kUTile);
    k_upart2<<<unsigned(std::min<uint64_t>(t2, 2 * uint64_t(cus))), kUT, 0, s>>>(E1, n, c0, nc,
                                                                               cur, E2);
    k_upart3<<<unsigned(std::min<uint64_t>(uint64_t(nc) * kNB2, uint64_t(cus) * 2)), kU3, 0, s>>>(
        E2, n, c0, nc, lo, ix->d_uniq);
    SMASH_HIPX(hipGetLastError());
  }
}

}  // namespace

void release_uniq_scratch(smash_index *ix) {
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
