// tools/randbench.hip -- ceiling of dependent random 16-byte loads on MI355X
// as a function of the footprint (the access pattern of the MAM search:
// every lane follows its own chain of dependent probes into a ~144 GB index).
//
//   randbench <GiB list...>  |  randbench lines <GiB...>  |  randbench req  |  randbench calib
// For each footprint: lanes = waves_per_simd * 4 * CUs * 64 chains, each doing
// `steps` dependent 16-byte loads at hashed addresses; prints loads/s and the
// 64-B-line rate.  Also an "ilp" variant with 4 independent chains per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); std::exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

template <int ILP>
__global__ __launch_bounds__(256) void k_chase(const uint4 *buf, uint64_t n16, int steps,
                                               uint64_t *sink, uint64_t seed) {
  const uint64_t t = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
  uint64_t h[ILP];
#pragma unroll
  for (int k = 0; k < ILP; ++k) h[k] = mix(t * ILP + k + seed);
  uint64_t acc = 0;
  for (int s = 0; s < steps; ++s) {
    uint4 v[ILP];
#pragma unroll
    for (int k = 0; k < ILP; ++k) v[k] = buf[h[k] % n16];
#pragma unroll
    for (int k = 0; k < ILP; ++k) {
      acc += v[k].x;
      h[k] = mix(h[k] + v[k].x + 1);   // dependent on the loaded value
    }
  }
  if (acc == 0x123456789ull) sink[0] = acc;
}

// W 16-byte loads per step into ONE 64-byte line (W = 2: the kernel's
// addr/addr2 pairs; W = 4: the whole line): does a second request to a line
// cost at the random-request ceiling?
template <int W>
__global__ __launch_bounds__(256) void k_chase_line(const uint4 *buf, uint64_t n16, int steps,
                                                    uint64_t *sink, uint64_t seed) {
  const uint64_t t = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
  uint64_t h = mix(t + seed);
  uint64_t acc = 0;
  for (int s = 0; s < steps; ++s) {
    const uint64_t i = (h % n16) & ~uint64_t(3);
    uint4 v[W];
#pragma unroll
    for (int k = 0; k < W; ++k) v[k] = buf[i + k];
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) x += v[k].x ^ v[k].w;
    acc += x;
    h = mix(h + x + 1);
  }
  if (acc == 0x123456789ull) sink[0] = acc;
}

// one 16-byte load per step at a random byte offset inside a random 64-byte
// line (never crossing it): is an unaligned probe one request?
__global__ __launch_bounds__(256) void k_chase_ua(const uint8_t *buf, uint64_t n64, int steps,
                                                  uint64_t *sink, uint64_t seed) {
  const uint64_t t = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
  uint64_t h = mix(t + seed);
  uint64_t acc = 0;
  for (int s = 0; s < steps; ++s) {
    const uint64_t a = (h % n64) * 64 + (h >> 58) % 49;
    uint4 v;
    __builtin_memcpy(&v, buf + a, 16);
    const uint32_t x = v.x ^ v.w;
    acc += x;
    h = mix(h + x + 1);
  }
  if (acc == 0x123456789ull) sink[0] = acc;
}

// the request-rate ceilings without a modulo in the address math (power-of-
// two footprints, a multiply-shift hash): per step one 16-byte load at a
// random line (a miss beyond the caches) and W - 1 more 16-byte loads to the
// SAME line (requests that hit): the cost of a miss and of a hit request,
// the two kinds the MAM search issues (new lines; re-probes of a line it
// just touched, second blocks, prefetch elements)
template <int W, bool OFF = false>
__global__ __launch_bounds__(256) void k_req(const uint4 *buf, uint64_t mask16, int steps,
                                             uint64_t *sink, uint64_t seed) {
  const uint64_t t = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
  uint64_t h = mix(t + seed);
  uint32_t acc = 0;
  for (int s = 0; s < steps; ++s) {
    // OFF: the 16-byte block at a random offset in its 64-byte line (W = 1)
    const uint64_t i = ((h >> 17) & mask16) & (OFF ? ~uint64_t(0) : ~uint64_t(3));
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < W; ++k) {
      const uint4 v = buf[i + (k & 3)];
      x += v.x ^ v.w;
    }
    acc += x;
    h = (h + x + 1) * 0x9E3779B97F4A7C15ull;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char **argv) {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  if (argc > 1 && std::string(argv[1]) == "calib") {
    // FETCH_SIZE calibration for random 16-byte probes: one launch of a known
    // number of dependent random loads over 64 GiB (no line is reused)
    const uint64_t bytes = 64ull << 30, n16 = bytes / 16;
    void *buf = nullptr;
    uint64_t *sink;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 0, bytes));
    CK(hipMalloc(&sink, 8));
    const uint64_t threads = 4ull * 4 * cus * 64;
    const int steps = 64;
    k_chase<1><<<unsigned(threads / 256), 256>>>((const uint4 *)buf, n16, steps, sink, 7);
    CK(hipDeviceSynchronize());
    std::printf("calib: %llu random 16-byte loads (%llu threads x %d) over 64 GiB\n",
                (unsigned long long)(threads * steps), (unsigned long long)threads, steps);
    return 0;
  }
  if (argc > 1 && std::string(argv[1]) == "req") {
    uint64_t *sink;
    CK(hipMalloc(&sink, 8));
    std::vector<int> lgs = {-5, -2, 2, 6, 7};   // 32 MiB (L2-sized), 256 MiB (Infinity Cache), 4-128 GiB
    if (argc > 2) { lgs.clear(); for (int i = 2; i < argc; ++i) lgs.push_back(std::atoi(argv[i])); }
    for (int lg : lgs) {
      const uint64_t bytes = lg < 0 ? (1ull << 30) >> -lg : (1ull << 30) << lg;
      void *buf = nullptr;
      CK(hipMalloc(&buf, bytes));
      CK(hipMemset(buf, 0, bytes));
      for (int wps : {4, 8}) {
        for (int w : {1, 2, 3, 0}) {   // 0: one block at a random 16-byte offset
          const uint64_t threads = uint64_t(wps) * 4 * cus * 64;
          const int steps = 64;
          auto launch = [&](uint64_t seed) {
            if (w == 0) k_req<1, true><<<unsigned(threads / 256), 256>>>((const uint4 *)buf, bytes / 16 - 1, steps, sink, seed);
            else if (w == 1) k_req<1><<<unsigned(threads / 256), 256>>>((const uint4 *)buf, bytes / 16 - 1, steps, sink, seed);
            else if (w == 2) k_req<2><<<unsigned(threads / 256), 256>>>((const uint4 *)buf, bytes / 16 - 1, steps, sink, seed);
            else k_req<3><<<unsigned(threads / 256), 256>>>((const uint4 *)buf, bytes / 16 - 1, steps, sink, seed);
          };
          hipEvent_t a, b;
          CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
          launch(1);
          CK(hipDeviceSynchronize());
          CK(hipEventRecord(a));
          for (int r = 0; r < 3; ++r) launch(100 + r);
          CK(hipEventRecord(b));
          CK(hipEventSynchronize(b));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, a, b));
          const double lines = 3.0 * threads * steps;
          std::printf("req footprint %9.4f GiB  waves/SIMD %d  %s : %7.3f G lines/s  %7.3f G requests/s  %.3f ns per line\n",
                      double(bytes) / (1ull << 30), wps,
                      w == 0 ? "1 x 16 B, random offset  " : w == 1 ? "1 x 16 B per random line " :
                      w == 2 ? "2 x 16 B per random line " : "3 x 16 B per random line ",
                      lines / (ms * 1e-3) * 1e-9, (w ? w : 1) * lines / (ms * 1e-3) * 1e-9, ms * 1e6 / lines);
          std::fflush(stdout);
          CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
        }
      }
      CK(hipFree(buf));
    }
    return 0;
  }
  std::vector<double> gib;
  bool lines = false;   // "lines": W = 1, 2, 4 loads per 64-byte line
  for (int i = 1; i < argc; ++i) {
    if (std::string(argv[i]) == "lines") lines = true;
    else gib.push_back(std::atof(argv[i]));
  }
  if (gib.empty()) gib = {0.25, 4, 32, 128};
  uint64_t *sink;
  CK(hipMalloc(&sink, 8));
  for (double g : gib) {
    const uint64_t bytes = uint64_t(g * (1ull << 30)) & ~uint64_t(255);
    void *buf = nullptr;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 0, bytes));
    const uint64_t n16 = bytes / 16;
    if (lines) {
      const int wps = 4, steps = 64;
      const uint64_t threads = uint64_t(wps) * 4 * cus * 64;
      for (int w : {1, 2, 4, 0}) {   // 0: one unaligned 16-byte load inside the line
        hipEvent_t a, b;
        CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        auto launch = [&](uint64_t seed) {
          if (w == 0) k_chase_ua<<<unsigned(threads / 256), 256>>>((const uint8_t *)buf, n16 / 4, steps, sink, seed);
          else if (w == 1) k_chase_line<1><<<unsigned(threads / 256), 256>>>((const uint4 *)buf, n16, steps, sink, seed);
          else if (w == 2) k_chase_line<2><<<unsigned(threads / 256), 256>>>((const uint4 *)buf, n16, steps, sink, seed);
          else k_chase_line<4><<<unsigned(threads / 256), 256>>>((const uint4 *)buf, n16, steps, sink, seed);
        };
        launch(1);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < 3; ++r) launch(100 + r);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double ln = 3.0 * threads * steps;
        std::printf("footprint %8.3f GiB  waves/SIMD %d  %s : %.3f G lines/s  %.3f G loads/s\n",
                    g, wps, w == 0 ? "1 x 16 B unaligned" : w == 1 ? "1 x 16 B per line " :
                    w == 2 ? "2 x 16 B per line " : "4 x 16 B per line ",
                    ln / (ms * 1e-3) * 1e-9, (w ? w : 1) * ln / (ms * 1e-3) * 1e-9);
        std::fflush(stdout);
        CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
      }
      CK(hipFree(buf));
      continue;
    }
    for (int wps : {4, 8}) {
      for (int ilp : {1, 4}) {
        const uint64_t threads = uint64_t(wps) * 4 * cus * 64;
        const int steps = 64;
        hipEvent_t a, b;
        CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
        auto launch = [&](uint64_t seed) {
          if (ilp == 1) k_chase<1><<<unsigned(threads / 256), 256>>>((const uint4 *)buf, n16, steps, sink, seed);
          else k_chase<4><<<unsigned(threads / 256), 256>>>((const uint4 *)buf, n16, steps, sink, seed);
        };
        launch(1);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a));
        for (int r = 0; r < 3; ++r) launch(100 + r);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        const double loads = 3.0 * threads * steps * ilp;
        const double rate = loads / (ms * 1e-3);
        std::printf("footprint %8.2f GiB  waves/SIMD %d  ilp %d : %.3f G loads/s  (%.0f GB/s of 64-B lines)  avg latency %.2f us\n",
                    g, wps, ilp, rate * 1e-9, rate * 64e-9, (ms * 1e-3 / 3.0 / steps) * 1e6);
        std::fflush(stdout);
        CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
      }
    }
    CK(hipFree(buf));
  }
  return 0;
}
