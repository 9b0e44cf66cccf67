// tools/sm_emu/hip/hip_runtime.h -- a minimal stand-in for the HIP runtime
// header so that the device search code (smash-paper_amd/csrc/mam_sm.hpp)
// compiles as plain C++ for a single-lane host emulation (test tooling only:
// tools/sm_emu/sm_emu.cpp).  One "wave" = one lane: ballot is the predicate,
// shuffles are the identity, LDS is a host array.
#pragma once
#include <cstdint>
#include <cstring>

#define __host__
#define __device__
#define __global__
#define __shared__
#define __forceinline__ inline
#define __launch_bounds__(...)
#define __restrict__

typedef int hipError_t;
typedef void *hipStream_t;
typedef void *hipEvent_t;
static const hipError_t hipSuccess = 0;
inline const char *hipGetErrorString(hipError_t) { return "sm_emu: no HIP runtime"; }
inline hipError_t hipMalloc(void **, size_t) { return 1; }
inline hipError_t hipFree(void *) { return 0; }

struct dim3 { unsigned x = 0, y = 0, z = 0; };
extern thread_local dim3 threadIdx, blockIdx, blockDim;

struct uint4 { uint32_t x, y, z, w; };
inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return uint4{a, b, c, d}; }

inline void __syncthreads() {}
inline void __builtin_amdgcn_wave_barrier() {}
inline uint64_t __ballot(int p) { return p ? 1ull : 0ull; }
template <class T> inline T __shfl(T v, int, int = 64) { return v; }
inline int __popcll(unsigned long long v) { return __builtin_popcountll(v); }
inline unsigned long long atomicAdd(unsigned long long *p, unsigned long long v) {
  const unsigned long long o = *p; *p += v; return o;
}
