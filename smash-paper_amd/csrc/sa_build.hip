// smash-paper_amd/csrc/sa_build.hip -- device index construction for gfx950.
//
// Replaces the single-threaded host build of the reference:
//   suffixsort (qsufsort.cpp:266-344, Larsson-Sadakane) -> SA, ISA
//   longSA::computeLCP (longSA.cpp:224-237, Kasai)      -> LCP
//   longSA::show (longSA.cpp:612-690)                   -> map.bin
// The SA of a text whose last character '$' is unique and smallest is
// unique, so this builder reproduces rc1.i*.index.sa.bin byte for byte.
//
// Algorithm (HBM-resident, radix sorts from hipcub):
//  1. bucket every suffix by its first 2 characters (dense alphabet codes);
//  2. per bucket, radix-sort by the next k packed characters (k*bits <= 64);
//     rank[i] = head position of i's group; mark non-singleton groups;
//  3. prefix doubling over the still-tied suffixes only: key = (group
//     ordinal, rank[i+h]) packed into one u64, one radix sort per round,
//     h = 2+k, 2(2+k), ... until every group is a singleton (ISA = rank).
//  4. LCP: Kasai's carry in 2^k-position text chunks, one lane per chunk,
//     8-byte word compares; exact u32 values.
//  5. map.bin: one lane per forward base.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <chrono>
#include <cstdlib>

#include "common.hpp"

namespace smash {
namespace {

constexpr int kBlock = 256;

double wall() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
// SMASH_VERBOSE=1: per-phase timings of the device index build on stderr
void vlog(const char *fmt, double t0, uint64_t a = 0, uint64_t b = 0) {
  static const bool on = getenv("SMASH_VERBOSE") && getenv("SMASH_VERBOSE")[0] == '1';
  if (!on) return;
  fprintf(stderr, "[smash-index %7.2fs] ", wall() - t0);
  fprintf(stderr, fmt, (unsigned long long)a, (unsigned long long)b);
  fprintf(stderr, "\n");
  fflush(stderr);
}

__global__ void k_hist256(const uint8_t *__restrict__ T, uint64_t N,
                          unsigned long long *cnt) {
  __shared__ unsigned int h[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += stride)
    atomicAdd(&h[T[i]], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x)
    if (h[i]) atomicAdd(&cnt[i], (unsigned long long)h[i]);
}

struct CodeMap {
  uint8_t c[256];
};

__device__ inline uint32_t bucket_of(const uint8_t *T, const uint8_t *cm,
                                     uint64_t i, uint32_t base) {
  return uint32_t(cm[T[i]]) * base + cm[T[i + 1]];
}

// Per-block chunk: count buckets in LDS, reserve ranges, scatter.
constexpr int kItems = 64;
__global__ void k_bucket_count(const uint8_t *__restrict__ T, uint64_t N,
                               CodeMap cmap, uint32_t base, uint32_t nb,
                               unsigned long long *cnt) {
  __shared__ unsigned int h[64];
  __shared__ uint8_t cm[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) cm[i] = cmap.c[i];
  for (int i = threadIdx.x; i < 64; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const uint64_t beg = uint64_t(blockIdx.x) * kBlock * kItems;
  for (int k = 0; k < kItems; ++k) {
    uint64_t i = beg + uint64_t(k) * kBlock + threadIdx.x;
    if (i < N) atomicAdd(&h[bucket_of(T, cm, i, base)], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x)
    if (h[b]) atomicAdd(&cnt[b], (unsigned long long)h[b]);
}

template <class IdxT>
__global__ void k_bucket_scatter(const uint8_t *__restrict__ T, uint64_t N,
                                 CodeMap cmap, uint32_t base, uint32_t nb,
                                 unsigned long long *cursor, IdxT *SA) {
  __shared__ unsigned int h[64];
  __shared__ unsigned long long off[64];
  __shared__ uint8_t cm[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) cm[i] = cmap.c[i];
  for (int i = threadIdx.x; i < 64; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const uint64_t beg = uint64_t(blockIdx.x) * kBlock * kItems;
  for (int k = 0; k < kItems; ++k) {
    uint64_t i = beg + uint64_t(k) * kBlock + threadIdx.x;
    if (i < N) atomicAdd(&h[bucket_of(T, cm, i, base)], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += blockDim.x) {
    off[b] = h[b] ? atomicAdd(&cursor[b], (unsigned long long)h[b]) : 0;
    h[b] = 0;
  }
  __syncthreads();
  for (int k = 0; k < kItems; ++k) {
    uint64_t i = beg + uint64_t(k) * kBlock + threadIdx.x;
    if (i < N) {
      uint32_t b = bucket_of(T, cm, i, base);
      unsigned int r = atomicAdd(&h[b], 1u);
      SA[off[b] + r] = IdxT(i);
    }
  }
}

template <class IdxT>
__global__ void k_make_keys(const IdxT *__restrict__ sa, uint64_t n,
                            const uint8_t *__restrict__ T, CodeMap cmap,
                            int skip, int kchars, int bits, uint64_t *keys,
                            IdxT *vals) {
  __shared__ uint8_t cm[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) cm[i] = cmap.c[i];
  __syncthreads();
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < n; j += stride) {
    const uint64_t i = sa[j];
    uint64_t key = 0;
    for (int c = 0; c < kchars; ++c) key = (key << bits) | cm[T[i + skip + c]];
    keys[j] = key;
    vals[j] = IdxT(i);
  }
}

// boundary -> candidate head index (max-scan turns it into the group start)
__global__ void k_bounds(const uint64_t *__restrict__ key, uint64_t n,
                         uint64_t *hd) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < n; j += stride)
    hd[j] = (j == 0 || key[j] != key[j - 1]) ? j : 0;
}

template <class IdxT>
__global__ void k_bucket_finish(const uint64_t *__restrict__ key,
                                const IdxT *__restrict__ val,
                                const uint64_t *__restrict__ start, uint64_t n,
                                uint64_t o, IdxT *SA, IdxT *rank, uint8_t *act) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < n; j += stride) {
    const IdxT i = val[j];
    SA[o + j] = i;
    rank[i] = IdxT(o + start[j]);
    const bool tie = (j > 0 && key[j] == key[j - 1]) || (j + 1 < n && key[j] == key[j + 1]);
    act[o + j] = tie ? 1 : 0;
  }
}

template <class IdxT>
__global__ void k_round_head(const IdxT *__restrict__ P, uint64_t n,
                             const IdxT *__restrict__ SA,
                             const IdxT *__restrict__ rank, IdxT *is_head) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t a = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; a < n; a += stride) {
    const IdxT p = P[a];
    is_head[a] = rank[SA[p]] == p ? 1 : 0;
  }
}

template <class IdxT>
__global__ void k_round_pack(const IdxT *__restrict__ P, const IdxT *__restrict__ ord,
                             uint64_t n, const IdxT *__restrict__ SA,
                             const IdxT *__restrict__ rank, uint64_t h,
                             uint64_t N, int bits_rank, uint64_t *keys,
                             IdxT *vals) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t a = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; a < n; a += stride) {
    const uint64_t i = SA[P[a]];
    // tied suffixes are longer than h (a shorter one contains the unique '$')
    const uint64_t r2 = (i + h < N) ? uint64_t(rank[i + h]) : 0;
    keys[a] = (uint64_t(ord[a] - 1) << bits_rank) | r2;
    vals[a] = IdxT(i);
  }
}

template <class IdxT>
__global__ void k_round_apply(const uint64_t *__restrict__ key,
                              const IdxT *__restrict__ val,
                              const IdxT *__restrict__ P, uint64_t n, IdxT *SA,
                              uint64_t *bnd) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t a = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; a < n; a += stride) {
    SA[P[a]] = val[a];
    bnd[a] = (a == 0 || key[a] != key[a - 1]) ? uint64_t(P[a]) : 0;
  }
}

template <class IdxT>
__global__ void k_round_rank(const uint64_t *__restrict__ key,
                             const IdxT *__restrict__ val,
                             const uint64_t *__restrict__ head, uint64_t n,
                             IdxT *rank, uint8_t *act) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t a = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; a < n; a += stride) {
    rank[val[a]] = IdxT(head[a]);
    const bool tie = (a > 0 && key[a] == key[a - 1]) || (a + 1 < n && key[a] == key[a + 1]);
    act[a] = tie ? 1 : 0;
  }
}

// ---- LCP (Kasai carry per chunk) -------------------------------------------
__device__ inline uint64_t load8(const uint8_t *T, uint64_t a) {
  const uint64_t *w = reinterpret_cast<const uint64_t *>(T);
  const uint64_t q = a >> 3, s = (a & 7) * 8;
  const uint64_t lo = w[q];
  if (s == 0) return lo;
  return (lo >> s) | (w[q + 1] << (64 - s));
}

template <class IdxT>
__global__ void k_kasai(const uint8_t *__restrict__ T, uint64_t N,
                        const IdxT *__restrict__ SA, const IdxT *__restrict__ ISA,
                        uint32_t *lcp, uint64_t chunk) {
  const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t i0 = t * chunk;
  if (i0 >= N) return;
  const uint64_t i1 = i0 + chunk < N ? i0 + chunk : N;
  uint64_t h = 0;
  for (uint64_t i = i0; i < i1; ++i) {
    const uint64_t r = ISA[i];
    if (r == 0) {
      lcp[0] = 0;
    } else {
      const uint64_t j = SA[r - 1];
      for (;;) {
        const uint64_t x = load8(T, i + h) ^ load8(T, j + h);
        if (x) { h += uint64_t(__builtin_ctzll(x) >> 3); break; }
        h += 8;
      }
      lcp[r] = h > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(h);
    }
    h = h ? h - 1 : 0;
  }
}

// The first offset >= h at which T[a ..] and T[b ..] differ (the bytes
// before h are known equal).  A compare that runs past its first word goes
// on 64 bytes at a time, eight independent word pairs per trip: a chunk
// that starts inside a long repeat (an N run: millions of equal bytes)
// compared one dependent 8-byte word per memory round trip, and those
// chunks set the kernel's time.  (Blocks stay inside the text's 64-byte pad:
// the compare ends at or before the last text byte, a unique '$'.)
__device__ inline uint64_t lcp_from(const uint8_t *T, uint64_t N, uint64_t a, uint64_t b,
                                    uint64_t h) {
  uint64_t x = load8(T, a + h) ^ load8(T, b + h);
  if (x) return h + uint64_t(__builtin_ctzll(x) >> 3);
  h += 8;
  const uint64_t hi = (a > b ? a : b);
  while (hi + h + 72 <= N + 64) {
    uint64_t xs[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) xs[k] = load8(T, a + h + 8 * k) ^ load8(T, b + h + 8 * k);
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (xs[k]) return h + 8 * k + uint64_t(__builtin_ctzll(xs[k]) >> 3);
    h += 64;
  }
  for (;;) {
    x = load8(T, a + h) ^ load8(T, b + h);
    if (x) return h + uint64_t(__builtin_ctzll(x) >> 3);
    h += 8;
  }
}

// The same carry in text order, written in text order (PLCP, Karkkainen et
// al.'s permuted LCP): plcp[i] = lcp(suffix i, its SA predecessor).  Kasai's
// lcp[ISA[i]] store is a random 4-byte write per position (a partial-line
// read-modify-write at the memory); here every thread stores its chunk's
// values consecutively and k_lcp_gather puts them in rank order with one
// random 4-byte READ per rank.  The predecessor of position i + 1 is loaded
// while position i is compared (its rank one position earlier still).
template <class IdxT>
__global__ void k_plcp(const uint8_t *__restrict__ T, uint64_t N, const IdxT *__restrict__ SA,
                       const IdxT *__restrict__ ISA, uint32_t *plcp, uint64_t chunk) {
  // chunk: a multiple of kPB.  A lane takes its chunk kPB positions at a
  // time: their ranks in one 64/128-byte read, their predecessors' text
  // positions (kPB independent random loads) at once, then the kPB compares
  // (the carried h chains them), and the kPB values stored as one 64-byte
  // line -- every line a lane touches is read or written whole (a lane's
  // element-wise walk left 1 000 partial lines per CU in flight, more than
  // the caches hold, and each store a partial-line write)
  constexpr int kPB = 16;
  const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t i0 = t * chunk;
  if (i0 >= N) return;
  const uint64_t i1 = i0 + chunk < N ? i0 + chunk : N;
  uint64_t h = 0;
  for (uint64_t ib = i0; ib < i1; ib += kPB) {
    const uint32_t nb = i1 - ib < uint64_t(kPB) ? uint32_t(i1 - ib) : uint32_t(kPB);
    uint64_t r[kPB], j[kPB];
#pragma unroll
    for (int k = 0; k < kPB; ++k) r[k] = uint32_t(k) < nb ? uint64_t(ISA[ib + k]) : 0;
#pragma unroll
    for (int k = 0; k < kPB; ++k) j[k] = r[k] ? uint64_t(SA[r[k] - 1]) : 0;
    uint32_t v[kPB];
#pragma unroll
    for (int k = 0; k < kPB; ++k) {
      v[k] = 0;
      if (uint32_t(k) < nb) {
        if (r[k]) {
          h = lcp_from(T, N, ib + k, j[k], h);
          v[k] = h > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(h);
        }
        h = h ? h - 1 : 0;
      }
    }
    if (nb == uint32_t(kPB)) {
      uint4 *o = reinterpret_cast<uint4 *>(plcp + ib);
#pragma unroll
      for (int k = 0; k < kPB / 4; ++k)
        o[k] = make_uint4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
    } else {
      for (uint32_t k = 0; k < nb; ++k) plcp[ib + k] = v[k];
    }
  }
}

template <class IdxT>
__global__ void k_lcp_gather(const IdxT *__restrict__ SA, uint64_t N,
                             const uint32_t *__restrict__ plcp, uint32_t *lcp) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < N; r += stride)
    lcp[r] = r ? plcp[SA[r]] : 0u;
}

__global__ void k_lcp8(const uint32_t *__restrict__ lcp, uint64_t N, uint8_t *l8,
                       uint8_t *ovf_flag) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < N; r += stride) {
    const uint32_t v = lcp[r];
    l8[r] = v >= 255 ? 255 : uint8_t(v);
    ovf_flag[r] = v >= 255 ? 1 : 0;
  }
}

__global__ void k_ovf_fill(const uint64_t *__restrict__ idx, uint64_t n,
                           const uint32_t *__restrict__ lcp, uint64_t *ovf) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t a = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; a < n; a += stride) {
    ovf[2 * a] = idx[a];
    ovf[2 * a + 1] = lcp[idx[a]];
  }
}

// ---- map.bin (longSA.cpp:628-688) -----------------------------------------
template <class IdxT>
__global__ void k_map(const IdxT *__restrict__ ISA, const uint32_t *__restrict__ lcp,
                      uint64_t N, uint64_t sp, uint64_t sz, uint64_t out_off,
                      uint8_t *out) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < sz; i += stride) {
    const uint64_t sapos = ISA[sp + i];
    const uint64_t rcsapos = ISA[sp + 2 * sz - i];
    // min_lengths[r] = max(LCP[r], LCP[r+1]) + 1 (:628-641)
    uint64_t a = lcp[sapos], b = sapos + 1 < N ? lcp[sapos + 1] : 0;
    uint64_t right = (a > b ? a : b) + 1;
    a = lcp[rcsapos]; b = rcsapos + 1 < N ? lcp[rcsapos + 1] : 0;
    uint64_t left = (a > b ? a : b) + 1;
    if (right + i >= sz) right = 0;                  // :666
    if (left >= i) left = 0;                         // :667
    out[out_off + 2 * i] = uint8_t(left < 255 ? left : 255);
    out[out_off + 2 * i + 1] = uint8_t(right < 255 ? right : 255);
  }
}

template <class KeyT, class ValT>
size_t sort_temp_bytes(uint64_t n, int end_bit) {
  size_t bytes = 0;
  hipcub::DoubleBuffer<KeyT> k(nullptr, nullptr);
  hipcub::DoubleBuffer<ValT> v(nullptr, nullptr);
  SMASH_HIPX(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, k, v, n, 0, end_bit));
  return bytes;
}

template <class IdxT>
void build_sa_isa_t(smash_index *ix, hipStream_t s) {
  const uint64_t N = ix->N;
  const uint8_t *T = ix->d_text;
  const double t0 = wall();
  vlog("suffix sort: N=%llu idx_bytes=%llu", t0, N, sizeof(IdxT));
  // alphabet
  unsigned long long *d_cnt = dalloc<unsigned long long>(256);
  SMASH_HIPX(hipMemsetAsync(d_cnt, 0, 256 * 8, s));
  k_hist256<<<grid_for(N, kBlock, 4096), kBlock, 0, s>>>(T, N, d_cnt);
  unsigned long long hcnt[256];
  SMASH_HIPX(hipMemcpyAsync(hcnt, d_cnt, sizeof(hcnt), hipMemcpyDeviceToHost, s));
  SMASH_HIPX(hipStreamSynchronize(s));
  if (hcnt[0]) throw hip_failure{"text contains a NUL byte"};
  CodeMap cmap{};
  uint32_t sigma = 0;
  for (int c = 0; c < 256; ++c) cmap.c[c] = hcnt[c] ? uint8_t(++sigma) : 0;
  if (sigma + 1 > 7 * 7 && false) {}
  const uint32_t base = sigma + 1;
  int bits = int(ceil_log2(base));
  if (bits < 1) bits = 1;
  const uint32_t nb = base * base;
  if (nb > 64) throw hip_failure{"alphabet too large for 2-char buckets (" + std::to_string(sigma) + ")"};
  const int kchars = 64 / bits;
  const int bits_rank = int(ceil_log2(N + 1));

  IdxT *SA = dalloc<IdxT>(N);
  IdxT *rank = dalloc<IdxT>(N);
  uint8_t *act = dalloc<uint8_t>(N);
  // 1. buckets
  SMASH_HIPX(hipMemsetAsync(d_cnt, 0, 64 * 8, s));
  const unsigned gb = unsigned((N + uint64_t(kBlock) * kItems - 1) / (uint64_t(kBlock) * kItems));
  k_bucket_count<<<gb, kBlock, 0, s>>>(T, N, cmap, base, nb, d_cnt);
  unsigned long long bcnt[64];
  SMASH_HIPX(hipMemcpyAsync(bcnt, d_cnt, 64 * 8, hipMemcpyDeviceToHost, s));
  SMASH_HIPX(hipStreamSynchronize(s));
  unsigned long long boff[65];
  boff[0] = 0;
  uint64_t maxb = 0;
  for (uint32_t b = 0; b < nb; ++b) {
    boff[b + 1] = boff[b] + bcnt[b];
    maxb = std::max<uint64_t>(maxb, bcnt[b]);
  }
  SMASH_HIPX(hipMemcpyAsync(d_cnt, boff, 64 * 8, hipMemcpyHostToDevice, s));
  k_bucket_scatter<IdxT><<<gb, kBlock, 0, s>>>(T, N, cmap, base, nb, d_cnt, SA);
  vlog("buckets: %llu (largest %llu)", t0, nb, maxb);

  // 2. per-bucket sort by the next kchars characters
  {
    uint64_t *k0 = dalloc<uint64_t>(maxb), *k1 = dalloc<uint64_t>(maxb);
    IdxT *v0 = dalloc<IdxT>(maxb), *v1 = dalloc<IdxT>(maxb);
    uint64_t *hd = dalloc<uint64_t>(maxb), *st = dalloc<uint64_t>(maxb);
    size_t tb = sort_temp_bytes<uint64_t, IdxT>(maxb, kchars * bits);
    size_t sb = 0;
    SMASH_HIPX(hipcub::DeviceScan::InclusiveScan(nullptr, sb, hd, st, hipcub::Max(), maxb));
    tb = std::max(tb, sb);
    void *temp = dalloc<uint8_t>(tb);
    for (uint32_t b = 0; b < nb; ++b) {
      const uint64_t n = bcnt[b], o = boff[b];
      if (!n) continue;
      k_make_keys<IdxT><<<grid_for(n, kBlock, 65536), kBlock, 0, s>>>(
          SA + o, n, T, cmap, 2, kchars, bits, k0, v0);
      hipcub::DoubleBuffer<uint64_t> kb(k0, k1);
      hipcub::DoubleBuffer<IdxT> vb(v0, v1);
      size_t t2 = tb;
      SMASH_HIPX(hipcub::DeviceRadixSort::SortPairs(temp, t2, kb, vb, n, 0, kchars * bits, s));
      k_bounds<<<grid_for(n, kBlock, 65536), kBlock, 0, s>>>(kb.Current(), n, hd);
      t2 = tb;
      SMASH_HIPX(hipcub::DeviceScan::InclusiveScan(temp, t2, hd, st, hipcub::Max(), n, s));
      k_bucket_finish<IdxT><<<grid_for(n, kBlock, 65536), kBlock, 0, s>>>(
          kb.Current(), vb.Current(), st, n, o, SA, rank, act);
    }
    SMASH_HIPX(hipStreamSynchronize(s));
    dfree(k0); dfree(k1); dfree(v0); dfree(v1); dfree(hd); dfree(st); dfree(temp);
    vlog("bucket sorts done (%llu chars/key)", t0, uint64_t(kchars));
  }

  // 3. prefix doubling over tied suffixes
  {
    uint64_t *d_nsel = dalloc<uint64_t>(1);
    // active list from act[] flags
    size_t sb = 0;
    hipcub::CountingInputIterator<IdxT> cit(0);
    SMASH_HIPX(hipcub::DeviceSelect::Flagged(nullptr, sb, cit, act, (IdxT *)nullptr, d_nsel, N));
    void *temp = dalloc<uint8_t>(sb);
    uint64_t cap = 0, n_a = 0;
    // first selection: need an upper bound for P -> count flags via select itself
    IdxT *P = nullptr;
    {
      // count active first (DeviceReduce sum of flags)
      uint64_t *d_sum = dalloc<uint64_t>(1);
      size_t rb = 0;
      hipcub::TransformInputIterator<uint64_t, hipcub::CastOp<uint64_t>, const uint8_t *> fit(act, hipcub::CastOp<uint64_t>());
      SMASH_HIPX(hipcub::DeviceReduce::Sum(nullptr, rb, fit, d_sum, N));
      void *rt = dalloc<uint8_t>(rb);
      SMASH_HIPX(hipcub::DeviceReduce::Sum(rt, rb, fit, d_sum, N, s));
      SMASH_HIPX(hipMemcpyAsync(&n_a, d_sum, 8, hipMemcpyDeviceToHost, s));
      SMASH_HIPX(hipStreamSynchronize(s));
      dfree(rt); dfree(d_sum);
      cap = n_a;
      P = dalloc<IdxT>(cap);
      SMASH_HIPX(hipcub::DeviceSelect::Flagged(temp, sb, cit, act, P, d_nsel, N, s));
    }
    dfree(temp);
    dfree(act);
    uint64_t h = 2 + uint64_t(kchars);
    if (n_a) {
      IdxT *ord = dalloc<IdxT>(cap), *isH = dalloc<IdxT>(cap);
      uint64_t *k0 = dalloc<uint64_t>(cap), *k1 = dalloc<uint64_t>(cap);
      IdxT *v0 = dalloc<IdxT>(cap), *v1 = dalloc<IdxT>(cap);
      uint64_t *bnd = dalloc<uint64_t>(cap), *head = dalloc<uint64_t>(cap);
      uint8_t *act2 = dalloc<uint8_t>(cap);
      IdxT *P2 = dalloc<IdxT>(cap);
      size_t tb = sort_temp_bytes<uint64_t, IdxT>(cap, 64), t3 = 0;
      SMASH_HIPX(hipcub::DeviceScan::InclusiveScan(nullptr, t3, bnd, head, hipcub::Max(), cap));
      tb = std::max(tb, t3);
      t3 = 0;
      SMASH_HIPX(hipcub::DeviceScan::InclusiveSum(nullptr, t3, isH, ord, cap));
      tb = std::max(tb, t3);
      t3 = 0;
      SMASH_HIPX(hipcub::DeviceSelect::Flagged(nullptr, t3, P, act2, P2, d_nsel, cap));
      tb = std::max(tb, t3);
      void *tmp = dalloc<uint8_t>(tb);
      int rounds = 0;
      while (n_a) {
        if (h >= N || ++rounds > 64) throw hip_failure{"suffix sort did not converge"};
        const unsigned g = grid_for(n_a, kBlock, 65536);
        k_round_head<IdxT><<<g, kBlock, 0, s>>>(P, n_a, SA, rank, isH);
        size_t t2 = tb;
        SMASH_HIPX(hipcub::DeviceScan::InclusiveSum(tmp, t2, isH, ord, n_a, s));
        uint64_t nseg = 0;
        SMASH_HIPX(hipMemcpyAsync(&nseg, ord + (n_a - 1), sizeof(IdxT) == 8 ? 8 : 4,
                                  hipMemcpyDeviceToHost, s));
        SMASH_HIPX(hipStreamSynchronize(s));
        if (sizeof(IdxT) == 4) nseg &= 0xFFFFFFFFull;
        const int bits_ord = int(ceil_log2(nseg + 1));
        if (bits_ord + bits_rank > 64) throw hip_failure{"doubling key exceeds 64 bits"};
        k_round_pack<IdxT><<<g, kBlock, 0, s>>>(P, ord, n_a, SA, rank, h, N, bits_rank, k0, v0);
        hipcub::DoubleBuffer<uint64_t> kb(k0, k1);
        hipcub::DoubleBuffer<IdxT> vb(v0, v1);
        t2 = tb;
        SMASH_HIPX(hipcub::DeviceRadixSort::SortPairs(tmp, t2, kb, vb, n_a, 0,
                                                      bits_ord + bits_rank, s));
        k_round_apply<IdxT><<<g, kBlock, 0, s>>>(kb.Current(), vb.Current(), P, n_a, SA, bnd);
        t2 = tb;
        SMASH_HIPX(hipcub::DeviceScan::InclusiveScan(tmp, t2, bnd, head, hipcub::Max(), n_a, s));
        k_round_rank<IdxT><<<g, kBlock, 0, s>>>(kb.Current(), vb.Current(), head, n_a, rank, act2);
        t2 = tb;
        SMASH_HIPX(hipcub::DeviceSelect::Flagged(tmp, t2, P, act2, P2, d_nsel, n_a, s));
        uint64_t nn = 0;
        SMASH_HIPX(hipMemcpyAsync(&nn, d_nsel, 8, hipMemcpyDeviceToHost, s));
        SMASH_HIPX(hipStreamSynchronize(s));
        std::swap(P, P2);
        vlog("doubling h=%llu: %llu suffixes still tied", t0, h, nn);
        n_a = nn;
        h *= 2;
      }
      dfree(ord); dfree(isH); dfree(k0); dfree(k1); dfree(v0); dfree(v1);
      dfree(bnd); dfree(head); dfree(act2); dfree(P2); dfree(tmp);
    }
    dfree(P);
    dfree(d_nsel);
  }
  dfree(d_cnt);
  ix->d_sa = SA;
  ix->d_isa = rank;   // every group is a singleton: rank == ISA
}

template <class IdxT>
uint32_t *build_lcp32_t(smash_index *ix, hipStream_t s) {
  const uint64_t N = ix->N;
  uint32_t *lcp = dalloc<uint32_t>(N);
  uint64_t chunk = N / 262144;
  chunk = std::min<uint64_t>(std::max<uint64_t>(chunk, 64), 65536);
  const uint64_t threads = (N + chunk - 1) / chunk;
  const double t0 = wall();
  const char *ke = getenv("SMASH_LCP_KASAI");   // 1: the rank-order Kasai form (A/B)
  if (ke && ke[0] == '1') {
    k_kasai<IdxT><<<unsigned((threads + 127) / 128), 128, 0, s>>>(
        ix->d_text, N, static_cast<const IdxT *>(ix->d_sa),
        static_cast<const IdxT *>(ix->d_isa), lcp, chunk);
  } else {
    uint32_t *plcp = dalloc<uint32_t>(N);
    const uint64_t pc = (chunk + 15) & ~uint64_t(15);   // (k_plcp: whole 16-position blocks)
    const uint64_t pt = (N + pc - 1) / pc;
    k_plcp<IdxT><<<unsigned((pt + 127) / 128), 128, 0, s>>>(
        ix->d_text, N, static_cast<const IdxT *>(ix->d_sa),
        static_cast<const IdxT *>(ix->d_isa), plcp, pc);
    k_lcp_gather<IdxT><<<grid_for(N, 256, 1u << 20), 256, 0, s>>>(
        static_cast<const IdxT *>(ix->d_sa), N, plcp, lcp);
    SMASH_HIPX(hipStreamSynchronize(s));
    dfree(plcp);
  }
  SMASH_HIPX(hipGetLastError());
  if (getenv("SMASH_VERBOSE")) {
    SMASH_HIPX(hipStreamSynchronize(s));
    vlog("LCP (Kasai, %llu-position chunks)", t0, chunk);
  }
  return lcp;
}

template <class IdxT>
void build_map_t(smash_index *ix, const uint32_t *lcp, hipStream_t s) {
  uint64_t total = 0;
  for (uint32_t c = 0; c < ix->n_seq; c += 2) total += ix->sizes[c];
  ix->map_bytes = 2 + 2 * total;
  if (!ix->d_map) ix->d_map = dalloc<uint8_t>(ix->map_bytes);
  // 2 junk bytes upstream (longSA.cpp:617 writes one byte of each of two
  // string-literal pointers); we write zeros.
  SMASH_HIPX(hipMemsetAsync(ix->d_map, 0, 2, s));
  uint64_t off = 2;
  for (uint32_t c = 0; c < ix->n_seq; c += 2) {
    const uint64_t sz = ix->sizes[c];
    if (sz)
      k_map<IdxT><<<grid_for(sz, kBlock, 65536), kBlock, 0, s>>>(
          static_cast<const IdxT *>(ix->d_isa), lcp, ix->N, ix->startpos[c], sz,
          off, ix->d_map);
    off += 2 * sz;
  }
  SMASH_HIPX(hipGetLastError());
}

}  // namespace

void build_sa_isa(smash_index *ix, hipStream_t s) {
  if (ix->idx_bytes == 4) build_sa_isa_t<uint32_t>(ix, s);
  else build_sa_isa_t<uint64_t>(ix, s);
}

uint32_t *build_lcp32(smash_index *ix, hipStream_t s) {
  return ix->idx_bytes == 4 ? build_lcp32_t<uint32_t>(ix, s)
                            : build_lcp32_t<uint64_t>(ix, s);
}

void finish_lcp(smash_index *ix, const uint32_t *lcp, hipStream_t s) {
  const uint64_t N = ix->N;
  if (!ix->d_lcp8) {   // + 64 zero bytes: 16-byte probes may start at the last entry
    ix->d_lcp8 = dalloc<uint8_t>(N + 64);
    SMASH_HIPX(hipMemsetAsync(ix->d_lcp8 + N, 0, 64, s));
  }
  uint8_t *flag = dalloc<uint8_t>(N);
  k_lcp8<<<grid_for(N, kBlock, 65536), kBlock, 0, s>>>(lcp, N, ix->d_lcp8, flag);
  uint64_t *d_nsel = dalloc<uint64_t>(1);
  size_t sb = 0;
  hipcub::CountingInputIterator<uint64_t> cit(0);
  // count first
  uint64_t n = 0;
  {
    hipcub::TransformInputIterator<uint64_t, hipcub::CastOp<uint64_t>, const uint8_t *> fit(flag, hipcub::CastOp<uint64_t>());
    size_t rb = 0;
    SMASH_HIPX(hipcub::DeviceReduce::Sum(nullptr, rb, fit, d_nsel, N));
    void *rt = dalloc<uint8_t>(rb);
    SMASH_HIPX(hipcub::DeviceReduce::Sum(rt, rb, fit, d_nsel, N, s));
    SMASH_HIPX(hipMemcpyAsync(&n, d_nsel, 8, hipMemcpyDeviceToHost, s));
    SMASH_HIPX(hipStreamSynchronize(s));
    dfree(rt);
  }
  ix->n_ovf = n;
  dfree(ix->d_ovf);
  ix->d_ovf = dalloc<uint64_t>(2 * (n ? n : 1));
  if (n) {
    uint64_t *idx = dalloc<uint64_t>(n);
    SMASH_HIPX(hipcub::DeviceSelect::Flagged(nullptr, sb, cit, flag, idx, d_nsel, N));
    void *temp = dalloc<uint8_t>(sb);
    SMASH_HIPX(hipcub::DeviceSelect::Flagged(temp, sb, cit, flag, idx, d_nsel, N, s));
    k_ovf_fill<<<grid_for(n, kBlock, 65536), kBlock, 0, s>>>(idx, n, lcp, ix->d_ovf);
    SMASH_HIPX(hipStreamSynchronize(s));
    dfree(temp);
    dfree(idx);
  }
  SMASH_HIPX(hipStreamSynchronize(s));
  dfree(flag);
  dfree(d_nsel);
}

void build_map(smash_index *ix, const uint32_t *lcp, hipStream_t s) {
  if (ix->idx_bytes == 4) build_map_t<uint32_t>(ix, lcp, s);
  else build_map_t<uint64_t>(ix, lcp, s);
  ix->map_own = true;
}

}  // namespace smash
