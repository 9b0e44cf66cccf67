// smash-paper_amd/csrc/aux_build.hip -- search accelerators derived from the
// index (results-preserving; see mam_device.hpp):
//
//  U[x]  (u8, one per text position) = min(255, max(LCP[ISA[x]], LCP[ISA[x]+1]))
//        (built from SA + L8 by uniq_build.hip)
//        The suffix at x is alone in its SA interval at depth d iff U[x] < d
//        (d <= 255).  This is what the reference's suffix-link chain
//        (longSA.cpp:523-534 + expand_link, longSA.h:158-174) tests one step
//        at a time with two random LCP loads; the device scans U[pos+1..]
//        sequentially instead.  Same quantity as map.bin's `right` before the
//        edge rules (longSA.cpp:628-641, 666).
//  KT[w] (16 bytes per ACGT k-mer w, 2 bits/char, first char most
//        significant; layout in common.hpp) = the SA interval of the
//        suffixes starting with w, or lo > hi when w does not occur.  It
//        replaces the first k narrowing steps of top_down_faster from the
//        root (longSA.cpp:322-380).  The same entry carries the presence of
//        the 48 (k+2)-mers that contain w (k_kfilter), which the (F) window
//        filter of mam_sm.hpp reads: a window of min_len = k + 4 bases holds
//        3 such B-mers, all contained in the k-mer two bases into it, so one
//        entry decides the window.
#include "common.hpp"

namespace smash {
namespace {

__device__ inline int acgt2(uint8_t c) {
  switch (c) {
    case 'a': return 0;
    case 'c': return 1;
    case 'g': return 2;
    case 't': return 3;
    default: return -1;
  }
}

template <class IdxT>
__global__ void k_kcode(const IdxT *__restrict__ SA, const uint8_t *__restrict__ T,
                        uint64_t N, int K, uint32_t *code) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < N; r += stride) {
    const uint64_t x = SA[r];
    uint32_t c = 0;
    bool ok = x + K <= N;
    // the k bytes as two 8-byte words (the text has 64 zero bytes of pad):
    // two requests per rank instead of one byte load each
    const uint64_t *w = reinterpret_cast<const uint64_t *>(T);
    const uint64_t q = x >> 3, sh = (x & 7) * 8;
    const uint64_t a0 = w[q], a1 = w[q + 1], a2 = w[q + 2];
    const uint64_t b0 = sh ? (a0 >> sh) | (a1 << (64 - sh)) : a0;
    const uint64_t b1 = sh ? (a1 >> sh) | (a2 << (64 - sh)) : a1;
    for (int k = 0; k < K; ++k) {
      const int v = acgt2(uint8_t((k < 8 ? b0 : b1) >> (8 * (k & 7))));
      ok = ok && v >= 0;
      c = (c << 2) | uint32_t(v & 3);
    }
    code[r] = ok ? c : 0xFFFFFFFFu;
  }
}

__global__ void k_kfill(uint64_t *kt, uint64_t n) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t w = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; w < n; w += stride) {
    kt[2 * w] = 1;       // empty: lo > hi
    kt[2 * w + 1] = 0;
  }
}

__global__ void k_kbounds(const uint32_t *__restrict__ code, uint64_t N, uint64_t *kt) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < N; r += stride) {
    const uint32_t c = code[r];
    if (c == 0xFFFFFFFFu) continue;
    if (r == 0 || code[r - 1] != c) kt[2 * uint64_t(c)] = r;
    if (r + 1 == N || code[r + 1] != c) kt[2 * uint64_t(c) + 1] = r;
  }
}

// the (k+2)-mer presence bits of the table (common.hpp): every ACGT
// (k+2)-mer b0 b1 .. b(k+1) of the text sets one bit in each of the entries
// of the three k-mers it contains: b0..b(k-1) (bit b(k)*4 + b(k+1)),
// b1..b(k) (bit 16 + b0*4 + b(k+1)) and b2..b(k+1) (bit 32 + b0*4 + b1);
// filter bit f lives at bit 40 + f % 24 of word f / 24 of the entry
__global__ void k_kfilter(const uint8_t *__restrict__ T, uint64_t N, int K,
                          unsigned long long *kt) {
  // one thread per k-mer position x: the bits its entry gets from the three
  // (k+2)-mers that contain it (at x, x - 1, x - 2), OR-ed into the entry's
  // two words with at most two atomics (was three atomics per (k+2)-mer, one
  // in each of three entries); the bytes T[x - 2 .. x + K + 2) from 8-byte
  // words (T has 64 zero bytes past N)
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  const uint64_t *tw = reinterpret_cast<const uint64_t *>(T);
  for (uint64_t x = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; x + K <= N; x += stride) {
    const uint64_t a = x >= 2 ? x - 2 : 0;   // first byte loaded
    const uint64_t q = a >> 3, sh = (a & 7) * 8;
    const uint64_t w0 = tw[q], w1 = tw[q + 1], w2 = tw[q + 2], w3 = tw[q + 3];
    const uint64_t b0 = sh ? (w0 >> sh) | (w1 << (64 - sh)) : w0;
    const uint64_t b1 = sh ? (w1 >> sh) | (w2 << (64 - sh)) : w1;
    const uint64_t b2 = sh ? (w2 >> sh) | (w3 << (64 - sh)) : w2;
    const uint32_t off = uint32_t(x - a);   // 2 (or 0 / 1 at the text's start)
    // code of byte t of [x - 2, x + K + 2) (t = 0..K+3), -1 if not ACGT
    auto code = [&](uint32_t t) -> int {
      const uint32_t i = t + off - 2;     // index into the loaded bytes
      const uint64_t wd = i < 8 ? b0 : i < 16 ? b1 : b2;
      return acgt2(uint8_t(wd >> (8 * (i & 7))));
    };
    uint64_t c = 0;
    bool ok = true;
    for (int k = 0; k < K; ++k) {
      const int v = code(2 + k);
      ok = ok && v >= 0;
      c = (c << 2) | uint64_t(v & 3);
    }
    if (!ok) continue;
    const int l2 = x >= 2 ? code(0) : -1, l1 = x >= 1 ? code(1) : -1;
    const int r1 = x + K < N ? code(2 + K) : -1, r2 = x + K + 1 < N ? code(3 + K) : -1;
    unsigned long long m0 = 0, m1 = 0;
    auto put = [&](uint32_t f) {
      if (f < 24) m0 |= 1ull << (40 + f);
      else m1 |= 1ull << (40 + f - 24);
    };
    if (r1 >= 0 && r2 >= 0) put(uint32_t(r1 * 4 + r2));            // the (k+2)-mer at x
    if (l1 >= 0 && r1 >= 0) put(16u + uint32_t(l1 * 4 + r1));      // at x - 1
    if (l2 >= 0 && l1 >= 0) put(32u + uint32_t(l2 * 4 + l1));      // at x - 2
    if (m0) atomicOr(&kt[2 * c], m0);
    if (m1) atomicOr(&kt[2 * c + 1], m1);
  }
}

__global__ void k_present(const uint8_t *__restrict__ T, uint64_t N, unsigned int *present) {
  __shared__ unsigned int h[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += stride)
    h[T[i]] = 1;
  __syncthreads();
  for (int i = threadIdx.x; i < 256; i += blockDim.x)
    if (h[i]) present[i] = 1;
}

template <class IdxT>
void build_aux_t(smash_index *ix, hipStream_t s) {
  const uint64_t N = ix->N;
  if (!ix->d_uniq) ix->d_uniq = dalloc<uint8_t>(N + 64);
  SMASH_HIPX(hipMemsetAsync(ix->d_uniq + N, 0, 64, s));
  build_uniq_range(ix, 0, N, s);   // from SA + L8 (uniq_build.hip)
  release_uniq_scratch(ix);        // (the index build's HBM is the pipelines' after it)
  // k: floor(log4 N) characters, <= 16 (about one suffix per k-mer: a root
  // descent lands on a singleton or a short run; hg19: 4^16 x 16 B = 69 GB)
  int K = 4;
  while (K < 16 && (1ull << (2 * (K + 1))) <= N) ++K;
  ix->kmer_k = uint32_t(K);
  const uint64_t nk = 1ull << (2 * K);
  if (!ix->d_kmer) ix->d_kmer = dalloc<uint64_t>(2 * nk);
  k_kfill<<<grid_for(nk, 256, 1u << 20), 256, 0, s>>>(ix->d_kmer, nk);
  uint32_t *code = dalloc<uint32_t>(N);
  k_kcode<IdxT><<<grid_for(N, 256, 1u << 20), 256, 0, s>>>(
      static_cast<const IdxT *>(ix->d_sa), ix->d_text, N, K, code);
  k_kbounds<<<grid_for(N, 256, 1u << 20), 256, 0, s>>>(code, N, ix->d_kmer);
  SMASH_HIPX(hipStreamSynchronize(s));
  dfree(code);
  // the (k+2)-mer presence bits, in the same entries (after k_kbounds, which
  // writes whole words)
  ix->bitmap_b = uint32_t(K + 2);
  k_kfilter<<<grid_for(N, 256, 1u << 20), 256, 0, s>>>(
      ix->d_text, N, K, reinterpret_cast<unsigned long long *>(ix->d_kmer));
  unsigned int *pres = dalloc<unsigned int>(256);
  SMASH_HIPX(hipMemsetAsync(pres, 0, 1024, s));
  k_present<<<grid_for(N, 256, 4096), 256, 0, s>>>(ix->d_text, N, pres);
  unsigned int hp[256];
  SMASH_HIPX(hipMemcpyAsync(hp, pres, 1024, hipMemcpyDeviceToHost, s));
  SMASH_HIPX(hipStreamSynchronize(s));
  dfree(pres);
  for (int i = 0; i < 4; ++i) ix->in_text[i] = 0;
  for (int c = 0; c < 256; ++c)
    if (hp[c]) ix->in_text[c >> 6] |= 1ull << (c & 63);
  SMASH_HIPX(hipGetLastError());
}

}  // namespace

void build_aux(smash_index *ix, hipStream_t s) {
  if (ix->idx_bytes == 4) build_aux_t<uint32_t>(ix, s);
  else build_aux_t<uint64_t>(ix, s);
}

}  // namespace smash
