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
// Memory: per forward base two sequential 8-byte ISA reads (forward and
// reverse-complement strand, the latter walking down) and two random LCP
// reads (adjacent bytes, one 64-B line each) -> ~146 B per base, HBM-bound.
// Each block takes a tile of consecutive bases (coalesced ISA loads); the
// bin counts of a tile, which spans few bins, go through LDS.
#include "common.hpp"

namespace smash {
namespace {

constexpr int kMB = 256;          // threads per block
constexpr int kMItems = 16;       // bases per thread per tile
constexpr int kLdsBins = 32;      // bins of a tile counted in LDS

struct MapCtx {
  const uint8_t *L8;
  const uint64_t *ovf;
  uint64_t n_ovf, N;
  const int64_t *bins;
  uint32_t nbins, k;
};

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

__device__ __forceinline__ uint32_t bin_of(const MapCtx &c, int64_t a) {
  uint32_t lo = 0, hi = c.nbins;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a < c.bins[mid]) hi = mid;
    else lo = mid + 1;
  }
  return lo == 0 ? c.nbins - 1 : lo - 1;
}

// bases [i0, i1) of one contig (text start sp, size S); out: map.bin bytes of
// base i0 onwards (or null); abs0 = chrom_sizes offset of the contig (< 0:
// not binned)
template <class IdxT>
__global__ __launch_bounds__(kMB) void k_mapscan(MapCtx c, const IdxT *__restrict__ ISA,
                                                 uint64_t sp, uint64_t S, uint64_t i0, uint64_t i1,
                                                 uint8_t *__restrict__ out, int64_t abs0,
                                                 unsigned long long *bin_counts,
                                                 unsigned long long *contig_count) {
  __shared__ unsigned long long s_bin[kLdsBins];
  __shared__ unsigned long long s_tot;
  __shared__ uint32_t s_b0;
  const uint64_t tile = uint64_t(kMB) * kMItems;
  const uint64_t ntiles = (i1 - i0 + tile - 1) / tile;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint64_t t0 = i0 + t * tile;
    if (threadIdx.x < kLdsBins) s_bin[threadIdx.x] = 0;
    if (threadIdx.x == 0) {
      s_tot = 0;
      s_b0 = (abs0 >= 0 && c.nbins) ? bin_of(c, abs0 + int64_t(t0)) : 0;
    }
    __syncthreads();
    const uint32_t b0 = s_b0;
    unsigned long long mine = 0;
#pragma unroll 4
    for (int j = 0; j < kMItems; ++j) {
      const uint64_t i = t0 + uint64_t(j) * kMB + threadIdx.x;
      if (i >= i1) break;
      const uint64_t sapos = ISA[sp + i];
      const uint64_t rcsapos = ISA[sp + 2 * S - i];
      uint64_t right = min_len_at(c, sapos);
      uint64_t left = min_len_at(c, rcsapos);
      if (right + i >= S) right = 0;
      if (left >= i) left = 0;
      if (out) {
        const uint64_t o = 2 * (i - i0);
        out[o] = uint8_t(left < 255 ? left : 255);
        out[o + 1] = uint8_t(right < 255 ? right : 255);
      }
      const uint64_t rb = right < 255 ? right : 255;
      if (rb >= 1 && rb <= c.k) {
        ++mine;
        if (abs0 >= 0 && c.nbins) {
          const uint32_t b = bin_of(c, abs0 + int64_t(i));
          const uint32_t d = b - b0;
          if (d < uint32_t(kLdsBins)) atomicAdd(&s_bin[d], 1ull);
          else atomicAdd(&bin_counts[b], 1ull);
        }
      }
    }
    if (mine) atomicAdd(&s_tot, mine);
    __syncthreads();
    if (threadIdx.x < kLdsBins && s_bin[threadIdx.x] && c.nbins)
      atomicAdd(&bin_counts[(b0 + threadIdx.x) % c.nbins], s_bin[threadIdx.x]);
    if (threadIdx.x == 0 && s_tot && contig_count) atomicAdd(contig_count, s_tot);
    __syncthreads();
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
  uint64_t g = 0;   // forward-base coordinate of the contig's first base
  for (uint32_t q = 0; q < ix->n_seq; q += 2) {
    const uint64_t S = ix->sizes[q], sp = ix->startpos[q];
    const uint64_t a = begin > g ? begin - g : 0;
    const uint64_t b = end < g + S ? end - g : S;
    if (a < b && g < end) {
      const uint64_t n = b - a;
      const uint64_t tiles = (n + uint64_t(kMB) * kMItems - 1) / (uint64_t(kMB) * kMItems);
      const unsigned grid = unsigned(tiles < 65536 ? tiles : 65536);
      k_mapscan<IdxT><<<grid, kMB, 0, s>>>(
          c, static_cast<const IdxT *>(ix->d_isa), sp, S, a, b,
          out ? out + 2 * (g + a - begin) : nullptr, h_chrom_off ? h_chrom_off[q / 2] : -1,
          reinterpret_cast<unsigned long long *>(d_bin_counts),
          d_contig_counts ? reinterpret_cast<unsigned long long *>(d_contig_counts + q / 2)
                          : nullptr);
      SMASH_HIP(hipGetLastError());
    }
    g += S;
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
  uint64_t total = 0;
  for (uint32_t q = 0; q < ix->n_seq; q += 2) total += ix->sizes[q];
  if (end > total) {
    set_error("smash_mappability_scan: range past the last forward base");
    return SMASH_ERR_ARG;
  }
  if (begin == end) return SMASH_OK;
  SMASH_HIP(hipSetDevice(ix->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (ix->idx_bytes == 4)
    return scan_t<uint32_t>(ix, begin, end, k, d_map_out, h_chrom_off, d_bin_starts, nbins,
                            d_bin_counts, d_contig_counts, s);
  return scan_t<uint64_t>(ix, begin, end, k, d_map_out, h_chrom_off, d_bin_starts, nbins,
                          d_bin_counts, d_contig_counts, s);
}
