// tests/csrc/index_check.hip -- TEST INFRASTRUCTURE: an independent device
// checker of a suffix-array index at full size (hg19: N = 6.2e9), used by
// tests/test_gpu_configs.py to pin the device-built index without a CPU
// suffix sort.  It shares no code with the product (smash-paper_amd/csrc).
//
// Properties checked (together they prove SA is THE suffix array of T and
// that the LCP array is exact wherever it is below 255):
//   perm   SA[i] < N and ISA[SA[i]] == i for every rank i (SA is a
//          permutation, ISA its inverse)
//   order  for every rank i >= 1, with a = SA[i-1], b = SA[i] and l the
//          exact LCP (L8[i], or the overflow table's value when L8 == 255):
//          T[a..a+min(l,255)) == T[b..b+min(l,255)) and T[a+l] < T[b+l]
//          (signed bytes, as the reference's top_down_faster compares);
//          rank 0 is the '$' suffix N-1 with LCP 0 (longSA.cpp:224-237)
//   ovf    the overflow table holds exactly the ranks with L8 == 255, in
//          increasing rank order, each with a value >= 255
//   full   for every `every`-th overflow entry, T[a+255..a+l) ==
//          T[b+255..b+l) compared in full (up to `cap` bytes per entry)
#include <hip/hip_runtime.h>

#include <cstdint>

struct ichk_result {
  unsigned long long perm_bad, perm_first;
  unsigned long long order_bad, order_first;
  unsigned long long ovf_bad, ovf_first;
  unsigned long long full_bad, full_first, full_checked, full_bytes;
  unsigned long long rank0_ok;
};

namespace {

template <class I>
__device__ __forceinline__ uint64_t at(const void *a, uint64_t k) {
  return uint64_t(static_cast<const I *>(a)[k]);
}

__device__ void note(unsigned long long *cnt, unsigned long long *first, uint64_t i) {
  atomicAdd(cnt, 1ull);
  atomicMin(first, (unsigned long long)i);
}

template <class I>
__global__ void k_perm(const void *SA, const void *ISA, uint64_t N, ichk_result *r) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += stride) {
    const uint64_t s = at<I>(SA, i);
    if (s >= N || at<I>(ISA, s) != i) note(&r->perm_bad, &r->perm_first, i);
  }
}

// exact LCP at rank i: L8, else lower_bound over the sorted overflow ranks
__device__ uint64_t lcp_at(const uint8_t *L8, const uint64_t *ovf, uint64_t n_ovf, uint64_t i,
                           bool *ok) {
  const uint64_t v = L8[i];
  if (v != 255) return v;
  uint64_t lo = 0, hi = n_ovf;
  while (lo < hi) {
    const uint64_t m = (lo + hi) >> 1;
    if (ovf[2 * m] < i) lo = m + 1; else hi = m;
  }
  if (lo >= n_ovf || ovf[2 * lo] != i) { *ok = false; return 0; }
  return ovf[2 * lo + 1];
}

template <class I>
__global__ void k_order(const uint8_t *T, uint64_t N, const void *SA, const uint8_t *L8,
                        const uint64_t *ovf, uint64_t n_ovf, ichk_result *r) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += stride) {
    if (i == 0) {
      if (at<I>(SA, 0) == N - 1 && L8[0] == 0 && T[N - 1] == '$') atomicAdd(&r->rank0_ok, 1ull);
      continue;
    }
    const uint64_t a = at<I>(SA, i - 1), b = at<I>(SA, i);
    bool ok = a < N && b < N;
    const uint64_t l = ok ? lcp_at(L8, ovf, n_ovf, i, &ok) : 0;
    if (ok) ok = a + l < N && b + l < N;
    if (ok) {
      const uint64_t m = l < 255 ? l : 255;
      for (uint64_t k = 0; k < m && ok; ++k) ok = T[a + k] == T[b + k];
      ok = ok && int8_t(T[a + l]) < int8_t(T[b + l]);
    }
    if (!ok) note(&r->order_bad, &r->order_first, i);
  }
}

__global__ void k_ovf(const uint8_t *L8, uint64_t N, const uint64_t *ovf, uint64_t n_ovf,
                      unsigned long long *n255, ichk_result *r) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  unsigned long long c = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < N; i += stride)
    c += L8[i] == 255;
  atomicAdd(n255, c);
  for (uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < n_ovf; j += stride) {
    const uint64_t k = ovf[2 * j];
    const bool ok = k < N && L8[k] == 255 && ovf[2 * j + 1] >= 255 &&
                    (j == 0 || ovf[2 * (j - 1)] < k);
    if (!ok) note(&r->ovf_bad, &r->ovf_first, j);
  }
}

template <class I>
__global__ void k_full(const uint8_t *T, uint64_t N, const void *SA, const uint64_t *ovf,
                       uint64_t n_ovf, uint64_t every, uint64_t cap, ichk_result *r) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; t * every < n_ovf;
       t += stride) {
    const uint64_t j = t * every, i = ovf[2 * j], l = ovf[2 * j + 1];
    if (i == 0 || i >= N) continue;
    const uint64_t a = at<I>(SA, i - 1), b = at<I>(SA, i);
    if (a >= N || b >= N || a + l >= N || b + l >= N) {
      note(&r->full_bad, &r->full_first, j);
      continue;
    }
    const uint64_t e = l < 255 + cap ? l : 255 + cap;
    bool ok = true;
    for (uint64_t k = 255; k < e && ok; ++k) ok = T[a + k] == T[b + k];
    if (!ok) note(&r->full_bad, &r->full_first, j);
    atomicAdd(&r->full_checked, 1ull);
    atomicAdd(&r->full_bytes, (unsigned long long)(e > 255 ? e - 255 : 0));
  }
}

}  // namespace

// Runs every check synchronously on the current device; returns 0 or a
// hipError_t.  `out` is host memory.
extern "C" int ichk_run(const uint8_t *T, uint64_t N, const void *SA, const void *ISA,
                        uint32_t idx_bytes, const uint8_t *L8, const uint64_t *ovf,
                        uint64_t n_ovf, uint64_t every, uint64_t cap, ichk_result *out,
                        unsigned long long *n255_out) {
  ichk_result h = {};
  h.perm_first = h.order_first = h.ovf_first = h.full_first = ~0ull;
  ichk_result *r = nullptr;
  unsigned long long *n255 = nullptr;
  hipError_t e = hipMalloc(&r, sizeof(h));
  if (e == hipSuccess) e = hipMalloc(&n255, 8);
  if (e == hipSuccess) e = hipMemcpy(r, &h, sizeof(h), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(n255, 0, 8);
  if (e != hipSuccess) return int(e);
  const unsigned G = 8192, B = 256;
  if (idx_bytes == 8) {
    k_perm<uint64_t><<<G, B>>>(SA, ISA, N, r);
    k_order<uint64_t><<<G, B>>>(T, N, SA, L8, ovf, n_ovf, r);
    if (every) k_full<uint64_t><<<G, B>>>(T, N, SA, ovf, n_ovf, every, cap, r);
  } else {
    k_perm<uint32_t><<<G, B>>>(SA, ISA, N, r);
    k_order<uint32_t><<<G, B>>>(T, N, SA, L8, ovf, n_ovf, r);
    if (every) k_full<uint32_t><<<G, B>>>(T, N, SA, ovf, n_ovf, every, cap, r);
  }
  k_ovf<<<G, B>>>(L8, N, ovf, n_ovf, n255, r);
  e = hipGetLastError();
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(out, r, sizeof(h), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(n255_out, n255, 8, hipMemcpyDeviceToHost);
  (void)hipFree(r);
  (void)hipFree(n255);
  return int(e);
}
