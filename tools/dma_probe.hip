// tools/dma_probe.hip -- what global_load_lds of 1, 2 and 4 bytes per lane
// does on gfx950 (measurement tool, not product): one wave copies a row of
// `len` bytes from a source at a 2-byte (ushort) / 1-byte (ubyte) aligned
// address into LDS with lane i moving bytes [i*size, (i+1)*size), waits,
// and writes the LDS row out; the host compares with the source.  Every
// source address is naturally aligned for its size (no unaligned DMA).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void glb_void_t;

template <int SIZE>
__global__ void k_probe(const uint8_t *src, uint32_t len, uint8_t *out) {
  __shared__ __attribute__((aligned(16))) uint8_t row[512];
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = lane; i < 512; i += 64) row[i] = 0xEE;
  __syncthreads();
  const uint32_t per = 64 * SIZE;   // bytes one instruction moves
  for (uint32_t b = 0; b < len; b += per) {
    const uint32_t n = (len - b + SIZE - 1) / SIZE < 64 ? (len - b + SIZE - 1) / SIZE : 64;
    if (lane < n) {
      glb_void_t *g = (glb_void_t *)(src + b + SIZE * lane);
      lds_void_t *l = (lds_void_t *)(row + b);
      if constexpr (SIZE == 1) __builtin_amdgcn_global_load_lds(g, l, 1, 0, 0);
      else if constexpr (SIZE == 2) __builtin_amdgcn_global_load_lds(g, l, 2, 0, 0);
      else __builtin_amdgcn_global_load_lds(g, l, 4, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (uint32_t i = lane; i < 512; i += 64) out[i] = row[i];
}

int main() {
  const uint32_t N = 1 << 16;
  std::vector<uint8_t> h(N);
  for (uint32_t i = 0; i < N; ++i) h[i] = uint8_t(i * 131 + 7);
  uint8_t *d = nullptr, *o = nullptr;
  if (hipMalloc(&d, N) || hipMalloc(&o, 512)) return 2;
  (void)hipMemcpy(d, h.data(), N, hipMemcpyHostToDevice);
  int bad = 0;
  struct Case { int size; uint32_t off, len; };
  const Case cs[] = {{2, 150, 150}, {2, 302, 150}, {2, 150 * 7, 100}, {1, 151, 101}, {1, 3, 150},
                     {4, 300, 148}};
  for (const Case &c : cs) {
    (void)hipMemset(o, 0, 512);
    if (c.size == 2) k_probe<2><<<1, 64>>>(d + c.off, c.len, o);
    else if (c.size == 1) k_probe<1><<<1, 64>>>(d + c.off, c.len, o);
    else k_probe<4><<<1, 64>>>(d + c.off, c.len, o);
    if (hipDeviceSynchronize() != hipSuccess) {
      std::printf("size %d off %u: launch failed\n", c.size, c.off);
      return 1;
    }
    std::vector<uint8_t> r(512);
    (void)hipMemcpy(r.data(), o, 512, hipMemcpyDeviceToHost);
    uint32_t mism = 0, first = ~0u, tail_ok = 1;
    for (uint32_t i = 0; i < c.len; ++i)
      if (r[i] != h[c.off + i]) { ++mism; if (first == ~0u) first = i; }
    const uint32_t moved = (c.len + c.size - 1) / c.size * c.size;
    for (uint32_t i = moved; i < 512; ++i) tail_ok &= r[i] == 0xEE;
    std::printf("size %d off %u len %u: %u mismatches (first %d), untouched tail %s\n", c.size, c.off,
                c.len, mism, int(first), tail_ok ? "yes" : "no");
    bad += mism != 0 || !tail_ok;
  }
  std::printf(bad ? "DMA_PROBE FAIL\n" : "DMA_PROBE OK\n");
  return bad ? 1 : 0;
}
