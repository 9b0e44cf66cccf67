// smash-paper_amd/csrc/mam_sm.hpp -- the v3 MAM search as a lane state
// machine: every loop iteration issues one 16-byte gather per lane (two for
// the states that own two independent probes), then each lane advances its
// state with ALU work only until it names its next address.
//
// Why: a direct per-lane implementation (mam_read_v3, mam_device.hpp) keeps
// the lanes of a wave in different phases; SIMT then issues each phase's
// load for its few lanes only and the wave waits one memory latency per
// phase present.  Here all lanes share one gather per iteration.  Because the
// wave executes the union of the state bodies present in an iteration, every
// body is kept small and branch-light:
//  * k_prep turns each read into a record (raw bytes, a 2-bit code stream,
//    and a "bad" mask = not ACGT or absent from the text) once, so the (F)
//    window filter, the B-mer and k-mer codes are O(1) bit extractions;
//  * states are grouped by what they load (an SA/ISA element, one text byte,
//    16 text bytes to compare, 16 U or LCP bytes to scan) and share the
//    decoding of the loaded block;
//  * 16-byte scans of U and LCP (singleton chains, expand_link) are unrolled
//    without branches.
//
// The algorithm, and therefore every emitted match, is mam_read_v3's: the
// same traverse / top_down_faster / (S) scan / (A) extension / (B) chain /
// suffix link / expand_link / (F) filter decisions, per lane, in order.
#pragma once
#include "mam_device.hpp"

// the 16-byte probe at byte address a (not necessarily aligned: gfx950's
// global loads take any byte address, and a block that stays inside one
// 64-byte line is one request).  The host emulation, tools/sm_emu,
// substitutes a checked, counted load here.
#ifndef PAD_KEEP
#define PAD_KEEP(x) asm volatile("" : "+v"(x))
#endif
// The search's policy knobs (binary-search prefetch, 32-byte U scans, linear
// L8 blocks before bisecting a run, the (F) filter policy, reads claimed per
// wave): compile-time defaults on the device, where their alternatives are
// dead code that still shapes the loop's registers and schedule; the host
// emulator (tools/sm_emu, SM_KNOB defined there) keeps them as runtime Ctx
// fields for its A/B tests of the policies.
#ifndef SM_KNOB
#define SM_KNOB(field, dflt) (dflt)
#endif
#ifndef SM_HOOK_BM
#define SM_HOOK_BM(mode, a1, a2)   // host emulation: filter outcomes (policies 0-2)
#endif
#ifndef SM_HOOK_F
#define SM_HOOK_F(j, bits)         // host emulation: filter outcomes (policy 3)
#endif
#ifndef SM_HOOK_BS
#define SM_HOOK_BS(size, depth)   // host emulation: interval statistics
#endif
// host emulation: where the binary-search compares start and stop (offsets
// from the probed suffix's start), and how far the L8 runs reach (kind 0:
// expand_link after ISA loads, 1: the traverse's final run around an SA rank)
#ifndef SM_HOOK_CMPBS
#define SM_HOOK_CMPBS(begin, sp, off)
#endif
#ifndef SM_HOOK_RUN
#define SM_HOOK_RUN(begin, kind, ext_l, ext_r)
#endif
#ifndef SM_HOOK_BYTE
#define SM_HOOK_BYTE(pos)
#endif
#ifndef SM_HOOK_PARK
#define SM_HOOK_PARK(a)           // host emulation: decide chains that park in S_ALU, by action
#endif
#ifndef SM_LOAD16
#define SM_LOAD16(a) ::smash::sm::load16u(a)
#endif
// the same load, told the lane state that issues it (the host emulation files
// the window filter's k-mer-table probes apart from the (C) descents')
#ifndef SM_LOAD16ST
#define SM_LOAD16ST(a, st) SM_LOAD16(a)
#endif
// speculative loads of a binary search's next SA elements (both children of
// the probe being compared; one of them is used): the emulation does not
// count them as probes, SM_HOOK_PF counts the one that is used
#ifndef SM_LOADPF16
#define SM_LOADPF16(a) ::smash::sm::load16u(a)
#endif
#ifndef SM_LOADIDX
#define SM_LOADIDX(p, i) uint64_t((p)[i])
#endif
#ifndef SM_HOOK_PF
#define SM_HOOK_PF(a)
#endif
// byte permute (v_perm_b32): byte i of the result is byte sel_i of the pair
// {s0 (bytes 4-7), s1 (bytes 0-3)} (8-11: the sign of byte 1/3/5/7 spread,
// 12: zero); the host emulation substitutes its own
#ifndef SM_PERM
#define SM_PERM(s0, s1, sel) __builtin_amdgcn_perm(s0, s1, sel)
#endif

// STATS builds: count the wave iterations in which a code region runs (any
// lane active in it), wave_stats[64 + k]; the regions' costs are paid per
// such iteration (tools/isa_regions.py gives their static VALU)
#define SM_REGION(k)                                                              \
  do {                                                                            \
    if (STATS) {                                                                  \
      const uint64_t am_ = __ballot(1);                                           \
      if (lane == uint32_t(__builtin_ctzll(am_))) atomicAdd(c.wave_stats + 64 + (k), 1ull); \
    }                                                                             \
  } while (0)

// n 16-byte record chunks from src into the LDS row dst, asynchronously
// (LDS-DMA: lanes 0..n-1 each move one chunk; dst wave-uniform)
#ifndef SM_DMA_ROW
#define SM_DMA_ROW(dst, src, n, lane) ::smash::sm::dma_row(dst, src, n, lane)
#endif

namespace smash {
namespace sm {

__device__ __forceinline__ uint4 load16u(uint64_t a) {
  uint4 v;
  __builtin_memcpy(&v, reinterpret_cast<const uint8_t *>(a), 16);
  return v;
}

#ifndef SM_DMA_ROW_HOST
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void glb_void_t;
__device__ __forceinline__ void dma_row(uint32_t *dst, const uint4 *src, uint32_t n, uint32_t lane) {
  if (lane < n)
    __builtin_amdgcn_global_load_lds((glb_void_t *)(src + lane), (lds_void_t *)dst, 16, 0, 0);
}
#endif

// record / LDS row geometry for a launch (reads up to max_len bases)
struct Geom {
  uint32_t w_raw;    // read bytes + lds_load8 over-read, in words
  uint32_t w_row;    // LDS row words: w_raw rounded up to whole 16-byte chunks
                     // (the row is one LDS-DMA of the record's raw chunks; lanes
                     // read their rows at unrelated offsets, so no padding
                     // against bank conflicts)
  uint32_t c_bad;    // record chunks holding the bad mask (1 or 2)
  uint32_t chunks;   // 16-byte record chunks per read
};

// the LDS row words of make_geom(L), as a constant expression (GEO kernels)
__host__ __device__ constexpr uint32_t geo_row(uint32_t L) {
  return ((L + 11) / 4 + 3) / 4 * 4 < 8 ? 8u : ((L + 11) / 4 + 3) / 4 * 4;
}

inline Geom make_geom(uint32_t max_len) {
  Geom g;
  g.w_raw = (max_len + 11) / 4;      // lds_load8 at offset <= L-1 reads 3 words
  g.w_row = (g.w_raw + 3) & ~3u;
  if (g.w_row < 8) g.w_row = 8;      // codes_raw reads 6 words from q <= w_row - 6
  g.c_bad = max_len > 128 ? 2 : 1;
  g.chunks = g.c_bad + (g.w_row + 3) / 4;
  return g;
}


// Record of read r (g.chunks * 4 words), built by k_prep:
//   [0, 4*c_bad)          bad mask, bit i of word i/32: base i is not ACGT
//                         or does not occur in the text
//   [4*c_bad, +w_row)     the read bytes, zero padded (w_row = whole chunks)
// The 2-bit base codes the B-mer / k-mer lookups need are derived from the
// bytes where they are used (codes_raw), which keeps the LDS row at the
// read's bytes (occupancy: 4 waves per SIMD at 150 bp).
// One block of 256 threads per `per_block` reads: (1) the block copies the
// reads' bytes into LDS with word loads and zeroes the records' LDS image,
// (2) one thread per (read, 32-base group) builds that group's bad-mask word
// and its 8 raw words from 9 LDS words (no per-thread byte loop over the
// whole read), (3) the block writes the records out with contiguous word
// stores.  All loops stride by blockDim.x (the host emulation runs one
// thread).
inline uint32_t prep_per_block(const Geom &g, uint64_t stride) {
  const uint64_t per = 24 * 1024 / (stride + 4 * (g.chunks * 4) + 8);
  return uint32_t(per < 1 ? 1 : per > 64 ? 64 : per);
}
__host__ __device__ inline uint32_t prep_in_words(uint64_t stride, uint32_t per) {
  // + the 9-word over-read of (2); a multiple of 4 words (the records' LDS
  // image after it takes 16-byte accesses)
  return (uint32_t((per * stride + 8 + 3) / 4 + 10) + 3) & ~3u;
}
inline size_t prep_lds_bytes(const Geom &g, uint64_t stride, uint32_t per) {
  return size_t(prep_in_words(stride, per)) * 4 + size_t(per) * (g.chunks * 4) * 4;
}

__global__ __launch_bounds__(256) void k_prep(const uint8_t *__restrict__ seqs, uint64_t stride,
                                              const uint16_t *__restrict__ lens, uint32_t len0,
                                              uint64_t n, uint64_t it0, uint64_t it1, uint64_t it2,
                                              uint64_t it3, Geom g, uint32_t per,
                                              uint32_t *__restrict__ rec) {
  extern __shared__ uint32_t prep_lds[];
  const uint32_t rw = g.chunks * 4;                    // record words
  const uint32_t G = 4 * g.c_bad;                      // 32-base groups (bad-mask words)
  const uint64_t r0 = uint64_t(blockIdx.x) * per;
  if (r0 >= n) return;
  const uint32_t nr = uint32_t(n - r0 < per ? n - r0 : per);
  // (1) input bytes [r0*stride, (r0+nr)*stride), word-aligned
  const uint64_t a0 = reinterpret_cast<uint64_t>(seqs + r0 * stride);
  const uint64_t a1 = reinterpret_cast<uint64_t>(seqs + (r0 + nr) * stride);
  const uint64_t w0 = a0 & ~uint64_t(3);
  const uint32_t nw = uint32_t(((a1 + 3) & ~uint64_t(3)) - w0) / 4;
  uint32_t *in = prep_lds;
  uint32_t *out = prep_lds + prep_in_words(stride, per);
  // 16-byte loads when the span starts on a 16-byte boundary (the usual
  // case: per * stride is a multiple of 16 for 150 bp and 100 bp reads),
  // else words; the records (rw words per read, a multiple of 4) and the
  // LDS images are always 16-byte aligned
  uint32_t k0 = 0;
  if ((w0 & 15) == 0) {
    const uint32_t n4 = nw / 4;
    for (uint32_t k = threadIdx.x; k < n4; k += blockDim.x)
      reinterpret_cast<uint4 *>(in)[k] = reinterpret_cast<const uint4 *>(w0)[k];
    k0 = 4 * n4;
  }
  for (uint32_t k = k0 + threadIdx.x; k < nw; k += blockDim.x)
    in[k] = reinterpret_cast<const uint32_t *>(w0)[k];
  for (uint32_t k = threadIdx.x; k < nr * rw / 4; k += blockDim.x)
    reinterpret_cast<uint4 *>(out)[k] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  // a/c/g/t occur in the text (anything else is always bad)
  auto itx = [&](uint32_t b) {
    const uint64_t w = b < 64 ? it0 : b < 128 ? it1 : b < 192 ? it2 : it3;
    return uint32_t((w >> (b & 63)) & 1ull);
  };
  const uint32_t ia = itx('a'), ic = itx('c'), ig = itx('g'), iu = itx('t');
  // (2) one (read, group) per thread
  for (uint32_t item = threadIdx.x; item < nr * G; item += blockDim.x) {
    const uint32_t t = item / G, gi = item - t * G;
    const uint32_t L = lens ? lens[r0 + t] : len0;
    if (32 * gi >= L) continue;
    const uint32_t boff = uint32_t(a0 - w0) + uint32_t(t * stride) + 32 * gi;
    const uint32_t wq = boff >> 2, sh = (boff & 3) * 8;
    uint32_t *o = out + t * rw;
    uint32_t bw = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      uint32_t w = in[wq + k];
      if (sh) w = (w >> sh) | (in[wq + k + 1] << (32 - sh));
      const uint32_t i0 = 32 * gi + 4 * k;             // base index of byte 0
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t b = (w >> (8 * j)) & 0xFF;
        const bool live = i0 + j < L;
        if (!live) w &= ~(0xFFu << (8 * j));
        const uint32_t good = (b == 'a' ? ia : 0u) | (b == 'c' ? ic : 0u) |
                              (b == 'g' ? ig : 0u) | (b == 't' ? iu : 0u);
        bw |= uint32_t(live && !good) << (4 * k + j);
      }
      if (8 * gi + k < g.w_raw) o[4 * g.c_bad + 8 * gi + k] = w;
    }
    o[gi] = bw;
  }
  __syncthreads();
  // (3) contiguous stores of the block's records
  uint4 *dst = reinterpret_cast<uint4 *>(rec + r0 * rw);
  for (uint32_t k = threadIdx.x; k < nr * rw / 4; k += blockDim.x)
    dst[k] = reinterpret_cast<const uint4 *>(out)[k];
}

// The same records without LDS: one thread per (read, 32-base group), ga =
// ceil(max_len / 32) groups per read, reads the group's bytes straight from
// HBM (the three aligned 16-byte blocks holding them) and writes the group's
// bad-mask word and its 8 raw words (two 16-byte stores); the read's last
// group also zeroes the bad-mask words and raw words past the groups.  Every
// record word is written, so the records equal k_prep's.  A kernel without
// LDS can share a CU with a running k_mam_sm (whose blocks hold all of it):
// the pipeline builds the next batch's records under the current batch's
// search instead of between the two searches.  Blocks are loaded only where
// they start before the end of the input (never past its last aligned
// block).  items = n * ga < 2^32 (host check).
__global__ __launch_bounds__(256) void k_prep_direct(const uint8_t *__restrict__ seqs,
                                                     uint64_t stride,
                                                     const uint16_t *__restrict__ lens,
                                                     uint32_t len0, uint32_t n, uint32_t ga,
                                                     uint64_t it0, uint64_t it1, uint64_t it2,
                                                     uint64_t it3, Geom g,
                                                     uint32_t *__restrict__ rec, uint32_t prio) {
#ifndef SM_DMA_ROW_HOST
  if (prio) __builtin_amdgcn_s_setprio(2);   // beside the search (pipeline.hip SMASH_BESIDE_SEARCH)
#endif
  const uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= n * ga) return;
  const uint32_t r = item / ga;
  const uint32_t gi = item - r * ga;
  const uint32_t L = lens ? lens[r] : len0;
  uint32_t *o = rec + uint64_t(r) * (g.chunks * 4);
  uint32_t w8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t bw = 0;
  if (32 * gi < L) {
    auto itx = [&](uint32_t b) {
      const uint64_t w = b < 64 ? it0 : b < 128 ? it1 : b < 192 ? it2 : it3;
      return uint32_t((w >> (b & 63)) & 1ull);
    };
    const uint32_t ia = itx('a'), ic = itx('c'), ig = itx('g'), iu = itx('t');
    const uint64_t end = reinterpret_cast<uint64_t>(seqs) + uint64_t(n) * stride;
    const uint64_t b0 = reinterpret_cast<uint64_t>(seqs) + uint64_t(r) * stride + 32 * gi;
    const uint64_t a16 = b0 & ~uint64_t(15);
    const uint32_t off = uint32_t(b0 & 15);
    uint32_t d[12];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
      const uint4 v = a16 + 16 * k < end && (k < 2 || off) ? reinterpret_cast<const uint4 *>(a16)[k]
                                                          : make_uint4(0, 0, 0, 0);
      d[4 * k] = v.x; d[4 * k + 1] = v.y; d[4 * k + 2] = v.z; d[4 * k + 3] = v.w;
    }
    const uint32_t q = off >> 2, sh = (off & 3) * 8;
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      // dwords k + q and k + q + 1 of the blocks, q in 0..3
      const uint32_t lo = q == 0 ? d[k] : q == 1 ? d[k + 1] : q == 2 ? d[k + 2] : d[k + 3];
      const uint32_t hi = q == 0 ? d[k + 1] : q == 1 ? d[k + 2] : q == 2 ? d[k + 3] : d[k + 4];
      uint32_t w = sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
      const uint32_t i0 = 32 * gi + 4 * k;
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t b = (w >> (8 * j)) & 0xFF;
        const bool live = i0 + j < L;
        if (!live) w &= ~(0xFFu << (8 * j));
        const uint32_t good = (b == 'a' ? ia : 0u) | (b == 'c' ? ic : 0u) |
                              (b == 'g' ? ig : 0u) | (b == 't' ? iu : 0u);
        bw |= uint32_t(live && !good) << (4 * k + j);
      }
      w8[k] = 8 * gi + k < g.w_raw ? w : 0u;
    }
  }
  o[gi] = bw;
  uint32_t *raw = o + 4 * g.c_bad;
  if (8 * gi + 8 <= g.w_row) {   // 16-byte aligned: records and their raw part are whole chunks
    reinterpret_cast<uint4 *>(raw + 8 * gi)[0] = make_uint4(w8[0], w8[1], w8[2], w8[3]);
    reinterpret_cast<uint4 *>(raw + 8 * gi)[1] = make_uint4(w8[4], w8[5], w8[6], w8[7]);
  } else {
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k)
      if (8 * gi + k < g.w_row) raw[8 * gi + k] = w8[k];
  }
  if (gi == ga - 1) {
    for (uint32_t k = ga; k < 4 * g.c_bad; ++k) o[k] = 0;
    for (uint32_t k = 8 * ga; k < g.w_row; ++k) raw[k] = 0;
  }
}

// groups per read of k_prep_direct
inline uint32_t prep_groups(uint32_t max_len) { return (max_len + 31) / 32; }

// lane states: S_COPY and above own a pending 16-byte probe at `addr`.
// S_BYTE and above probe byte arrays (text, U, L8) at the exact byte
// address (the block holds bytes [addr, addr + 16)); the states below
// probe aligned 16-byte blocks (records, bitmap words, k-mer entries,
// SA / ISA elements) and find their element at addr & 15.
enum : uint32_t { S_EXIT = 0, S_NEW, S_ALU, S_COPY, S_BM, S_KT, S_IDX, S_BYTE, S_CMP, S_USCAN,
                  S_EXL, S_EXR, S_EXB };
// S_IDX ops (an SA / ISA element arrived; *2: a second one in v2)
enum : uint32_t { O_SAPOS, O_SAPOS2, O_BS_SA, O_ISAJ, O_NS_SA2, O_NS_ISA2 };
// S_CMP ops (16-32 text bytes compared with the read)
enum : uint32_t { O_EXT = 0, O_BS };
// ALU continuations, in the order the decide chain runs them
enum : uint32_t { A_NONE = 0, A_BSP, A_BS, A_BS_DONE, A_XL_DONE, A_RUN_DONE, A_CHAIN_DONE,
                  A_EXPAND, A_AFTER, A_TOP, A_TRAV, A_DONE, A_EMIT, A_EXS };
// binary-search modes: 0 where P' sorts (traverse); 1 / 2 the left / right
// end of a run of suffixes sharing `cap` characters (from `cbase`) with P
enum : uint32_t { BS_INSERT = 0, BS_LEFT, BS_RIGHT };

__device__ __forceinline__ uint64_t lo64(const uint4 &v) { return uint64_t(v.x) | (uint64_t(v.y) << 32); }
__device__ __forceinline__ uint64_t hi64(const uint4 &v) { return uint64_t(v.z) | (uint64_t(v.w) << 32); }
__device__ __forceinline__ uint32_t dword_at(const uint4 &v, uint32_t i) {   // i = 0..3
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}
__device__ __forceinline__ uint32_t byte_at(const uint4 &v, uint32_t o) {
  return (dword_at(v, o >> 2) >> (8 * (o & 3))) & 0xFF;
}
// bytes [o, o+8) of the block (past 16: zero)
__device__ __forceinline__ uint64_t bytes8_at(const uint4 &v, uint32_t o) {
  const uint64_t lo = lo64(v), hi = hi64(v);
  if (o == 0) return lo;
  if (o < 8) return (lo >> (8 * o)) | (hi << (64 - 8 * o));
  if (o == 8) return hi;
  return hi >> (8 * (o - 8));
}
// agreeing bytes of block bytes [o, 16) with the read at P[poff ...], <= lim
__device__ __forceinline__ uint32_t agree_block(const uint4 &v, uint32_t o, const uint8_t *P,
                                                uint32_t poff, uint32_t lim) {
  uint32_t k = agree8(bytes8_at(v, o), lds_load8(P, poff), lim < 8 ? lim : 8u);
  if (k == 8 && lim > 8) k += agree8(bytes8_at(v, o + 8), lds_load8(P, poff + 8), lim - 8);
  return k;
}
// mask bit i (0..15): byte i of the block satisfies f
template <class F>
__device__ __forceinline__ uint32_t byte_mask(const uint4 &v, F f) {
  uint32_t m = 0;
#pragma unroll
  for (uint32_t i = 0; i < 16; ++i) {
    const uint32_t b = (dword_at(v, i >> 2) >> (8 * (i & 3))) & 0xFF;
    m |= uint32_t(f(b, i)) << i;
  }
  return m;
}

// packed 16-bit subtract (v_pk_sub_u16): both halves, no borrow between them
#ifndef SM_PK_SUB16
typedef unsigned short sm_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_sub16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_bit_cast(sm_u16x2, a) - __builtin_bit_cast(sm_u16x2, b));
}
#define SM_PK_SUB16(a, b) ::smash::sm::pk_sub16(a, b)
#endif

// 4-bit mask, bit j: (t_j - byte j of w) is negative, for 16-bit thresholds
// t_j in [-32768, 32767] given as packed halves te = (t0, t2), to = (t1, t3).
// The bytes go to 16-bit lanes by two byte permutes, two packed subtracts
// compare them, a third permute spreads the four sign bits to bytes (selectors
// 8-11) and one multiply gathers them: 9 VALU per 4 bytes instead of a
// compare and a select per byte.
__device__ __forceinline__ uint32_t gt4(uint32_t w, uint32_t te, uint32_t to) {
  const uint32_t e = SM_PERM(w, w, 0x0c020c00u), o = SM_PERM(w, w, 0x0c030c01u);
  const uint32_t r = SM_PERM(SM_PK_SUB16(to, o), SM_PK_SUB16(te, e), 0x0b090a08u);
  return ((r & 0x80808080u) * 0x00204081u) >> 28;
}
// mask bit i (0..15): byte i of the block > t_i, with t_i = base - i (desc)
// or base; thresholds below -32768 or above 32767 do not occur (base <= 271)
__device__ __forceinline__ uint32_t thr_mask(const uint4 &v, uint32_t base, bool desc) {
  const uint32_t bp = base * 0x00010001u, s4 = desc ? 0x00040004u : 0u;
  // (a lane below zero borrows from its upper neighbour, whose index is larger:
  // both lie past the bytes the callers keep)
  uint32_t te = bp - (desc ? 0x00020000u : 0u), to = bp - (desc ? 0x00030001u : 0u);
  uint32_t m = 0;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    m |= gt4(dword_at(v, k), te, to) << (4 * k);
    te -= s4;
    to -= s4;
  }
  return m;
}

// one bit of a lane's flag word, used like a bool
struct FlagRef {
  uint32_t &f;
  uint32_t b;
  __device__ __forceinline__ operator bool() const { return (f >> b) & 1u; }
  __device__ __forceinline__ FlagRef &operator=(bool x) {
    f = (f & ~(1u << b)) | (uint32_t(x) << b);
    return *this;
  }
  __device__ __forceinline__ FlagRef &operator=(const FlagRef &o) { return *this = bool(o); }
};

struct Bad {   // the read's bad mask (registers; named, never an array)
  uint32_t w0, w1, w2, w3, w4, w5, w6, w7;
  __device__ __forceinline__ uint32_t word(uint32_t i) const {
    uint32_t r = 0;
    r = i == 0 ? w0 : r; r = i == 1 ? w1 : r; r = i == 2 ? w2 : r; r = i == 3 ? w3 : r;
    r = i == 4 ? w4 : r; r = i == 5 ? w5 : r; r = i == 6 ? w6 : r; r = i == 7 ? w7 : r;
    return r;
  }
  // bits [a, a+n) as the low bits, n <= 32
  __device__ __forceinline__ uint32_t bits(uint32_t a, uint32_t n) const {
    const uint32_t q = a >> 5, s = a & 31;
    const uint64_t x = (uint64_t(word(q + 1)) << 32) | word(q);
    const uint32_t y = uint32_t(x >> s);
    return n >= 32 ? y : (y & ((1u << n) - 1));
  }
  // bits [a, a+64) as a 64-bit word (past the mask: zero)
  __device__ __forceinline__ uint64_t bits64(uint32_t a) const {
    const uint32_t q = a >> 5, s = a & 31;
    const uint64_t x = (uint64_t(word(q + 1)) << 32) | word(q);
    const uint64_t z = uint64_t(word(q + 2)) << 32;
    return (x >> s) | (s ? z << (32 - s) : 0ull);
  }
  // highest set bit in [a, a+n), or -1
  __device__ __forceinline__ int32_t last(uint32_t a, uint32_t n) const {
    uint32_t e = a + n;
    while (e > a) {
      const uint32_t k = e - a < 32 ? e - a : 32u;
      const uint32_t s = e - k;
      const uint32_t y = bits(s, k);
      if (y) return int32_t(s + 31 - __builtin_clz(y));
      e = s;
    }
    return -1;
  }
};

// 2-bit codes (a0 c1 g2 t3) of the 4 lowercase bytes of w, first byte most
// significant.  The low 3 bits of a c g t are 1 3 7 4, so one byte permute
// over an 8-entry table {1: 0, 3: 1, 7: 2, 4: 3} turns each byte into its
// code, and one multiply gathers the four 2-bit fields (no carries: the
// partial products land on disjoint bits).  Other bytes give garbage
// (callers check `bad`).
__device__ __forceinline__ uint32_t byte4_codes(uint32_t w) {
  const uint32_t cb = SM_PERM(0x02000003u, 0x01000000u, w & 0x07070707u);
  return (cb * 0x40100401u) >> 24;
}

// 2n code bits of bases [p, p+n) of the LDS row R of w_row words (first base
// most significant), n <= 21: always the 6 words from q (24 bases, no
// branches), q clamped so that they stay inside the row (p + n <= L <=
// 4 w_row - 8 keeps [p, p+n) inside them: sh + n <= 24)
__device__ __forceinline__ uint64_t codes_raw(const uint32_t *R, uint32_t w_row, uint32_t p,
                                              uint32_t n) {
  const uint32_t q0 = p >> 2, qm = w_row - 6;
  const uint32_t q = q0 < qm ? q0 : qm, sh = p - 4 * q;
  uint32_t hi = byte4_codes(R[q]);
  hi = (hi << 8) | byte4_codes(R[q + 1]);
  hi = (hi << 8) | byte4_codes(R[q + 2]);
  hi = (hi << 8) | byte4_codes(R[q + 3]);
  const uint32_t lo = (byte4_codes(R[q + 4]) << 8) | byte4_codes(R[q + 5]);
  const uint64_t x = (uint64_t(hi) << 16) | lo;
  return (x >> (48 - 2 * (sh + n))) & ((1ull << (2 * n)) - 1);
}

// the same over 7 words (28 bases): n <= 25 (the filter's pair of 20-base
// entry windows 3 bases apart), q clamped to w_row - 7 (p + n <= 4 w_row)
__device__ __forceinline__ uint64_t codes_raw7(const uint32_t *R, uint32_t w_row, uint32_t p,
                                               uint32_t n) {
  const uint32_t q0 = p >> 2, qm = w_row - 7;
  const uint32_t q = q0 < qm ? q0 : qm, sh = p - 4 * q;
  uint32_t hi = byte4_codes(R[q]);
  hi = (hi << 8) | byte4_codes(R[q + 1]);
  hi = (hi << 8) | byte4_codes(R[q + 2]);
  uint32_t lo = byte4_codes(R[q + 3]);
  lo = (lo << 8) | byte4_codes(R[q + 4]);
  lo = (lo << 8) | byte4_codes(R[q + 5]);
  lo = (lo << 8) | byte4_codes(R[q + 6]);
  const uint64_t x = (uint64_t(hi) << 32) | lo;   // 28 bases, the first most significant
  return (x >> (56 - 2 * (sh + n))) & ((1ull << (2 * n)) - 1);
}

template <class IdxT>
struct Ctx {
  // the index (DevIndex fields, flattened: every field is a live SGPR)
  const uint8_t *T;
  const IdxT *SA, *ISA;
  const uint8_t *L8, *U;
  const uint64_t *KT;     // k-mer table: {lo, hi} + (k+2)-mer presence bits (common.hpp)
  uint64_t N;
  uint32_t logN, K, B, min_len;
  // k_prep records and the LDS row geometry
  const uint4 *rec;
  uint32_t chunks, c_bad, w_row, w_raw;
  // direct rows (rows != null): the reads themselves, one 16-byte aligned,
  // zero-padded row of w_row words per mate (smash_read_stride): no
  // records; the row is DMA'd from its read and the bad mask computed from
  // it in LDS by the wave (row_bad); bad_tab: the 8-byte table of the
  // expected byte per low-3-bit code (a c g t if they occur in the text)
  const uint4 *rows;
  uint32_t direct;        // rows != null (0 / 1)
  uint32_t bad_tab_lo, bad_tab_hi;
  uint32_t lin_blocks;    // L8 blocks scanned per side of a run before bisecting (>= 1)
  uint32_t pad;           // experiment: dependent ALU ops added per iteration (0 = none)
  // (PK, the read -> bin-count pipeline) each emitted match word carries in
  // bits 40..47 the map.bin right byte m = max(LCP[r], LCP[r + 1]) + 1 of
  // its own SA row r when the word's L8 hints give it exactly (both < 127),
  // else 0 (csrc/pipeline.hip mate_fast)
  uint32_t mhint;
  uint32_t grab;          // reads a wave claims per atomic on `work` (>= 1)
  uint32_t bm_dual;       // (F) policy: 0 one B-mer per iteration, 1 last + first in one,
                          // 2 the cover policy (two B-mers per iteration chosen by mode),
                          // 3 (default) one k-mer entry = the window's B + 2 B-mers
  uint32_t pf;            // binary-search compares also load the children's SA elements
  uint32_t u32;           // (B) U scans load 32 bytes per iteration (else 16)
  uint32_t f2;            // (F) policy 3: a second k-mer entry (the next three B-mers)
                          // rides along with the first when they are unknown (1: always,
                          // 2: only after an entry showed an absent B-mer)
  const uint16_t *lens;
  uint32_t len0, cap;
  uint64_t n_reads;
  uint64_t *out;
  uint32_t *n_out;
  unsigned long long *work;
  // probe check: every probe address must lie in [lo, hi) (the span of the
  // index arrays and the records); a lane that names another address records
  // it in viol[1..9] (viol[0] counts) and retires instead of faulting
  uint64_t lo, hi;
  unsigned long long *viol;
  uint64_t in_text[4];    // bytes occurring in the text (copied to LDS)
  // STATS builds only: per-read loop iterations; per-kernel sums of wave
  // iterations and of active lanes over them
  uint32_t *iters;
  unsigned long long *wave_stats;   // [0] wave iterations [1] active lanes [2..] lane iterations per state
};

template <class IdxT>
__device__ __forceinline__ uint64_t ia(const IdxT *a, uint64_t i) {
  return reinterpret_cast<uint64_t>(a + i);
}
template <class IdxT>
__device__ __forceinline__ uint64_t idx_val(const uint4 &v, uint32_t ao) {
  if (sizeof(IdxT) == 8) return (ao & 8) ? hi64(v) : lo64(v);
  return dword_at(v, ao >> 2);
}

// packed-word hints (common.hpp): the 7-bit capped L8 byte at bit b of w is
// known to be < xd (a run stops there): exact below 127, and 127 only stands
// for >= 127
__device__ __forceinline__ bool pk_below(uint64_t w, uint32_t b, uint32_t xd) {
  const uint32_t c = uint32_t(w >> b) & 127u;
  return c < xd && c < 127u;
}
__device__ __forceinline__ bool pk_above(uint64_t w, uint32_t b, uint32_t xd) {
  return (uint32_t(w >> b) & 127u) >= xd;
}
// the lowercase base of 2-bit code q (a0 c1 g2 t3)
__device__ __forceinline__ uint32_t pk_char(uint32_t q) { return (0x74676361u >> (8 * q)) & 0xFFu; }
// the match word's map hint (Ctx::mhint) from its packed SA word w: m of the
// row from its two L8 bytes when both are below the 127 cap, else 0
__device__ __forceinline__ uint64_t pk_map_hint(uint64_t w) {
  const uint32_t a = uint32_t(w >> 36) & 127u, b = uint32_t(w >> 43) & 127u;
  return (a < 127u && b < 127u) ? uint64_t((a > b ? a : b) + 1u) << 40 : 0ull;
}
// the window's 7 bases as bytes 0..6 of a u64 (byte 7 zero): each 2-bit code
// spread to a byte selector, one permute of the a c g t table per 4 bytes
__device__ __forceinline__ uint64_t pk_window(uint64_t w) {
  const uint32_t c = uint32_t(w >> 50);   // 14 bits: base i at bits 2i
  const uint32_t s0 = (c & 3u) | ((c << 6) & 0x300u) | ((c << 12) & 0x30000u) | ((c << 18) & 0x3000000u);
  const uint32_t s1 = ((c >> 8) & 3u) | ((c >> 2) & 0x300u) | ((c << 4) & 0x30000u) | 0x0c000000u;
  return uint64_t(SM_PERM(0u, 0x74676361u, s0)) | (uint64_t(SM_PERM(0u, 0x74676361u, s1)) << 32);
}

// Direct rows: the bad-mask nibble of the 4 bytes of w (bit j: byte j is not
// a base that occurs in the text), bases at or past `live` (0..4) masked.
// One permute looks up the byte each low-3-bit code would have to be
// (tab_hi:tab_lo, a c g t where they occur in the text, else a byte that
// can never match), a xor marks the mismatching bytes, the zero-byte test
// gathers their high bits and one multiply packs them (as gt4).
__device__ __forceinline__ uint32_t bad_nibble(uint32_t w, uint32_t tab_lo, uint32_t tab_hi,
                                               uint32_t live) {
  const uint32_t expect = SM_PERM(tab_hi, tab_lo, w & 0x07070707u);
  const uint32_t z = expect ^ w;
  const uint32_t nz = (((z & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | z) & 0x80808080u;
  const uint32_t nib = (nz * 0x00204081u) >> 28;
  return live >= 4 ? nib : nib & ((1u << live) - 1u);
}

// the same mask for one row, one lane alone (the host emulation's form of
// the wave's computation in k_mam_sm)
__device__ inline Bad row_bad_mask(const uint32_t *row, uint32_t L, uint32_t tab_lo,
                                            uint32_t tab_hi) {
  uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (uint32_t k = 0; 4 * k < L && k < 64; ++k)
    m[k >> 3] |= bad_nibble(row[k], tab_lo, tab_hi, L - 4 * k) << (4 * (k & 7));
  return Bad{m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7]};
}

// the bad_nibble table from the bytes that occur in the text
inline void bad_table(const uint64_t in_text[4], uint32_t *lo, uint32_t *hi) {
  uint8_t t[8];
  for (uint32_t c = 0; c < 8; ++c) t[c] = uint8_t(0x80u | (c ^ 1u));   // never equal: low bits differ
  const uint8_t letters[4] = {'a', 'c', 'g', 't'};
  for (uint8_t b : letters)
    if ((in_text[b >> 6] >> (b & 63)) & 1ull) t[b & 7] = b;
  *lo = uint32_t(t[0]) | uint32_t(t[1]) << 8 | uint32_t(t[2]) << 16 | uint32_t(t[3]) << 24;
  *hi = uint32_t(t[4]) | uint32_t(t[5]) << 8 | uint32_t(t[6]) << 16 | uint32_t(t[7]) << 24;
}

// One lane = one read at a time.  Each iteration: (1) the lanes with a
// pending probe load 16 bytes (two blocks when need2); (2) "consume": the
// loaded block advances the lane's state; (3) "decide": a fixed chain of ALU
// continuations names the next probe.  The chain has no loops: the two rare
// transitions that go backwards in it (end of read inside traverse ->
// after-traverse; a window filter skip -> the next window) park the lane in
// S_ALU for one iteration.
//
// traverse (longSA.cpp:297-316) over an interval [start, end] whose suffixes
// share `depth` characters with P' = P[prefix..L): its result is the longest
// match  best = max_i lcp(P'[depth..], T[SA[i]+depth..])  and the suffixes
// reaching it.  top_down_faster finds it character by character; here a
// binary search with full comparisons (lcp skipping as in Manber-Myers) finds
// where P' sorts: the suffix with the longest match is next to that point and
// both neighbours are probed; the suffixes sharing `best` more characters
// form the run around it with L8 >= depth + best (found by the expand_link
// scanner, bounded by [start, end]).  Same final (depth, interval) as the
// reference's traverse; ~2.5 log2(interval) probes instead of 4 log2 per
// character.
// (occupancy experiments: the GEO kernels' minimum waves per SIMD)
#ifndef SM_GEO_WPS
#define SM_GEO_WPS 1
#endif
template <class IdxT, int BLOCK, bool CHECK, bool STATS, bool PK = false, int GEO = 0>
__global__ __launch_bounds__(BLOCK, GEO ? SM_GEO_WPS : 1) void k_mam_sm(const Ctx<IdxT> c) {
  // GEO = L (150 or 100): the launch geometry of L-base reads on an index
  // with a 16-mer table (K 16, min_len 20, B 18, geo_row(L)-word rows), as
  // constants: the shifts, masks and row offsets built from them fold, and
  // the loop keeps fewer SGPRs live (run_sm picks it only when the Ctx holds
  // exactly these)
  static_assert(GEO == 0 || (GEO >= 21 && GEO <= 255), "GEO is 0 or the read length");
  const uint32_t gK = GEO ? 16u : c.K, gMin = GEO ? 20u : c.min_len, gB = GEO ? 18u : c.B;
  const uint32_t gRow = GEO ? geo_row(GEO) : c.w_row, gLen0 = GEO ? uint32_t(GEO) : c.len0;
  // (and the pipeline's launch: direct rows, no length array, L - 19 match
  // slots, map hints on, a text of 2^32..2^33 characters, no SMASH_SM_PAD)
  const uint32_t gDirect = GEO ? 1u : c.direct, gPad = GEO ? 0u : c.pad, gMh = GEO ? 1u : c.mhint;
  const uint32_t gLogN = GEO ? 33u : c.logN, gCap = GEO ? uint32_t(GEO) - 19u : c.cap;
  const uint16_t *const gLens = GEO ? nullptr : c.lens;
  // PK: the SA / ISA words carry the packed hints (common.hpp; 8-byte
  // elements only): their position bits are PM, and the hint paths below
  // exist only in this instantiation
  static_assert(!PK || sizeof(IdxT) == 8, "packed words are 8-byte elements");
  constexpr uint64_t PM = PK ? kPkPosMask : ~0ull;
  extern __shared__ uint32_t ldsw[];
  // (the 256-bit in-text set stays in scalar registers: dynamic LDS is
  // exactly 16 blocks x 64 rows x 160 B = the CU's 160 KB at 150 bp)
  const uint64_t it0 = c.in_text[0], it1 = c.in_text[1], it2 = c.in_text[2], it3 = c.in_text[3];
  auto in_text = [&](uint32_t b) {
    const uint64_t w = b < 64 ? it0 : b < 128 ? it1 : b < 192 ? it2 : it3;
    return ((w >> (b & 63)) & 1ull) != 0;
  };
  const uint64_t N = c.N;
  uint32_t *row = ldsw + threadIdx.x * gRow;
  const uint8_t *P = reinterpret_cast<const uint8_t *>(row);
  const uint32_t lane = threadIdx.x & 63;
  // direct rows: the bytes of row word `lane` inside the read (0..4)
  const uint32_t row_live = 4 * lane < gLen0 ? (gLen0 - 4 * lane < 4 ? gLen0 - 4 * lane : 4u) : 0u;

  uint64_t q_next = 0, q_end = 0;   // this wave's claimed, unassigned reads
  uint32_t st = S_NEW, op = 0, pend = A_NONE;
  uint64_t addr = 0, addr2 = 0;
  // per-lane flags live as bits of ONE vector register: as `bool`s the
  // compiler keeps them as lane masks in SGPR pairs, which spill
  uint32_t fl = 0;
  FlagRef need2{fl, 0};
  uint64_t rd = 0;
  uint32_t L = 0, nem = 0;
  Bad bad{0, 0, 0, 0, 0, 0, 0, 0};
  // search state (longSA.h interval_t + prefix)
  uint32_t prefix = 0, depth = 0;
  uint64_t start = 0, end = 0, pos = 0;
  FlagRef have_pos{fl, 1};
  // phase registers, shared by phases that are never live together
  uint64_t lo = 0, hi = 0, bpos = 0, sp = 0, m = 0, bi = 0, es = 0, ee = 0;
  uint64_t &c0 = bpos, &c1 = sp;                                // (F) bitmap codes
  uint32_t lL = 0, lR = 0, best = 0, lc = 0, cbase = 0, cap = 0, bsm = 0, nblk = 0;
  FlagRef hit{fl, 2}, bm2{fl, 3}, skip_f{fl, 4}, xrun{fl, 5};
  FlagRef rdone{fl, 6};   // a run's right side was finished by S_EXB
  uint32_t fm = 0;        // (F) probe mode (bm_dual 2)
  // (F) policy 3: what the k-mer entries told about the read's B-mers, as
  // offsets from read position kp: fk bit i = the B-mer at kp + i is known,
  // bit 16 + i = it occurs; fj = the offset (from prefix) of the in-flight
  // probe's window; the last entry's interval {klo, khi} of the k-mer at kx
  // (its (C) descent needs no second probe)
  uint32_t fk = 0, kp = 0, fj = 0, kx = 0xFFFFFFFFu;
  uint64_t klo = 1, khi = 0;
  FlagRef fdead{fl, 11};    // the last entry showed an absent B-mer
  FlagRef ktr_set{fl, 7};   // a passed window's k-mer code is in m
  FlagRef clean{fl, 8};     // the read has no bad base (bad mask all zero)
  // binary-search prefetch: the S_CMP O_BS probe in flight also loads the SA
  // elements of its two children, SA[(lo+m)/2] (v2, when need2) and
  // SA[(m+1+hi)/2] (v3, when pfr), so the next probe's text compare issues
  // one iteration later instead of two
  FlagRef pf{fl, 9}, pfr{fl, 10};
  // PK: what the ISA words of an expand_link's ends told (set where they are
  // consumed, read by A_EXPAND in the same iteration): the left end stops at
  // start (- 1 with xl1), the right end at end (+ 1 with xr1)
  FlagRef xls{fl, 12}, xl1{fl, 13}, xrs{fl, 14}, xr1{fl, 15};
  FlagRef em{fl, 16};   // A_EMIT: the singleton at pos is a match to emit
  uint32_t dch = 0, j = 0, thresh = 0, xd = 0;
  uint32_t it = 0;
  uint64_t w_iters = 0, w_active = 0;
  // (B) from a singleton at (pos, d): scan U[pos+1 ...] for the chain's exit,
  // 32 bytes per iteration
  auto uscan_start = [&](uint64_t p, uint32_t d) {
    dch = d; j = 1;
    addr = reinterpret_cast<uint64_t>(c.U + p + 1);
    addr2 = addr + 16;
    need2 = SM_KNOB(u32, 1u) && d - 1 > 16;
    st = S_USCAN;
  };
  // a run [es, ee] grows within [lb, hb] while L8 >= xd: both sides' first
  // blocks in one iteration (S_EXB), or the one side with room; false: none
  // left blocks are the 16 bytes ENDING at es (from 0 when es < 15), right
  // blocks start at ee + 1
  // probe m decided: P' agrees with S_m on lc characters past cbase; ranout:
  // P' ran out (it is a prefix of S_m), else its next byte pb differs from
  // the text's tb (signed chars, like the reference)
  auto bs_decide = [&](bool ranout, uint32_t pb, uint32_t tb) {
    bool left;                                  // keep [lo, m) (else (m, hi))
    if (bsm == BS_INSERT) {
      left = ranout || int8_t(pb) < int8_t(tb);
      if (lc > best) { best = lc; bpos = sp; bi = m; }
    } else {                                    // in the run iff lcp reaches cap
      left = (lc >= cap) == (bsm == BS_LEFT);
    }
    if (left) { hi = m; lR = lc; }
    else { lo = m + 1; lL = lc; }
  };
  // compare P' with T[sp + cbase + lc ...] (sp = the SA word of probe m).
  // Packed words: the 7 bases T[x + K ...) in the word decide a compare that
  // starts and ends inside them without a text probe (true: decided, the
  // caller goes on at A_BS); a compare that agrees on all of them goes on in
  // the text after them
  auto bs_probe = [&]() -> bool {
    SM_HOOK_CMPBS(true, sp, cbase + lc);
    const uint32_t o = cbase + lc;
    if (PK && ((sp >> kPkPosBits) & 7u) != 5u && o - gK < kPkWindow) {
      const uint32_t rem = cap - lc, nav = gK + kPkWindow - o;
      const uint32_t lim = rem < nav ? rem : nav;
      const uint64_t win = pk_window(sp) >> (8 * (o - gK));
      const uint32_t k = agree8(win, lds_load8(P, prefix + o), lim);
      lc += k;
      if (k < lim || k == rem) {
        SM_HOOK_CMPBS(false, sp, cbase + lc);
        bs_decide(k == rem, k == rem ? 0u : uint32_t(P[prefix + o + k]),
                  uint32_t(win >> (8 * (k & 7))) & 0xFFu);
        pf = false; pfr = false; need2 = false;
        return true;
      }
    }
    addr = reinterpret_cast<uint64_t>(c.T + (sp & PM) + cbase + lc);
    addr2 = ia(c.SA, (lo + m) >> 1);
    need2 = SM_KNOB(pf, 1u) && lo < m;
    pfr = SM_KNOB(pf, 1u) && m + 1 < hi;
    pf = SM_KNOB(pf, 1u) != 0;
    st = S_CMP; op = O_BS;
    return false;
  };
  auto lblock = [&](uint64_t e) { return reinterpret_cast<uint64_t>(c.L8 + (e >= 15 ? e - 15 : 0)); };
  // (ls / rs: that side's end is known already, from packed-word L8 bytes)
  auto ex_start = [&](uint64_t lb, uint64_t hb, bool ls, bool rs) {
    const bool l = !ls && es > lb, r = !rs && ee < hb;
    nblk = 0;
    rdone = !r;
    addr = l ? lblock(es) : reinterpret_cast<uint64_t>(c.L8 + ee + 1);
    addr2 = reinterpret_cast<uint64_t>(c.L8 + ee + 1);
    need2 = l && r;
    st = l && r ? S_EXB : l ? S_EXL : S_EXR;
    return l || r;
  };

  // PK: expand_link's run around [start, end] at depth xd = the current
  // depth (both are set when the ISA words arrive): from the ISA word of
  // start, L8[start] and L8[start - 1]; from end's, L8[end + 1] and L8[end + 2]
  auto isa_hints = [&](uint64_t wl, uint64_t wr) {
    const uint32_t d = depth;
    xls = pk_below(wl, 40, d) || (pk_above(wl, 40, d) && pk_below(wl, 33, d));
    xl1 = !pk_below(wl, 40, d);
    xrs = pk_below(wr, 47, d) || (pk_above(wr, 47, d) && pk_below(wr, 54, d));
    xr1 = !pk_below(wr, 47, d);
  };

  for (;;) {
    // Work claiming: lanes that need a read take it from the wave's private
    // range [q_next, q_end); a wave refills it with ONE atomic on the global
    // counter for `grab` reads (or as many as its lanes need), so the
    // counter's single-address atomics stay far below what its L2 channel
    // serialises.  Reads past n_reads retire the lane as before.
    const uint64_t newm = __ballot(st == S_NEW);
    const uint32_t need = uint32_t(__popcll(newm));
    const uint64_t avail = q_end - q_next;
    unsigned long long base = 0;
    uint32_t take = 0;
    if (newm && avail < need) {
      take = need > SM_KNOB(grab, 16u) ? need : SM_KNOB(grab, 16u);
      if (lane == uint32_t(__builtin_ctzll(newm)))
        base = atomicAdd(c.work, (unsigned long long)take);
    }
    const uint64_t live = __ballot(st != S_EXIT);
    if (live == 0) break;
    if (STATS) { w_iters += 1; w_active += __popcll(live); }
    // direct rows: the rows DMA'd last iteration (the lanes still in S_COPY)
    // have landed -- waited for here, before this iteration's loads are
    // issued, where nothing else is outstanding; the bad mask of each, one
    // row word per lane, assembled only when a base is bad
    if (gDirect) {
      uint64_t cm = __ballot(st == S_COPY);
      if (cm) {
        SM_REGION(27);
#ifdef SM_HOST_LANE
        if (st == S_COPY) bad = row_bad_mask(row, L, c.bad_tab_lo, c.bad_tab_hi);
#else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        while (cm) {
          const uint32_t ln = uint32_t(__builtin_ctzll(cm));
          cm &= cm - 1;
          // (direct rows have one length, gLen0: row_live is this lane's
          // live bytes of word `lane`, 0 past the read)
          const uint32_t w = row_live ? ldsw[ln * gRow + lane] : 0u;
          const uint32_t nib = row_live ? bad_nibble(w, c.bad_tab_lo, c.bad_tab_hi, row_live) : 0u;
          if (__ballot(nib != 0)) {   // rare: a read with a bad base
            uint32_t x = nib << (4 * (lane & 7));
            x |= __shfl_xor(x, 1, 64);
            x |= __shfl_xor(x, 2, 64);
            x |= __shfl_xor(x, 4, 64);
            const uint32_t m0 = __shfl(x, 0, 64), m1 = __shfl(x, 8, 64), m2 = __shfl(x, 16, 64),
                           m3 = __shfl(x, 24, 64), m4 = __shfl(x, 32, 64), m5 = __shfl(x, 40, 64),
                           m6 = __shfl(x, 48, 64), m7 = __shfl(x, 56, 64);
            if (lane == ln) bad = Bad{m0, m1, m2, m3, m4, m5, m6, m7};
          }
        }
#endif
      }
    }
    const uint32_t st_ld = S_COPY + gDirect;   // the lowest state that loads
    if (CHECK && st >= st_ld &&
        (addr < c.lo || addr >= c.hi || (need2 && (addr2 < c.lo || addr2 >= c.hi)))) {
      if (atomicAdd(c.viol, 1ull) == 0) {
        c.viol[1] = st; c.viol[2] = op; c.viol[3] = addr; c.viol[4] = need2 ? addr2 : 0;
        c.viol[5] = prefix; c.viol[6] = depth; c.viol[7] = start; c.viol[8] = end; c.viol[9] = rd;
      }
      st = S_EXIT;
      need2 = false; pfr = false;
    }
    uint4 v = make_uint4(0, 0, 0, 0), v2 = make_uint4(0, 0, 0, 0);
    uint64_t v3 = 0;
    const uint64_t amask = st >= S_BYTE ? ~uint64_t(0) : ~uint64_t(15);
    if (st >= st_ld) v = SM_LOAD16ST(addr & amask, st);
    if (need2) {
      if (pf) v2 = SM_LOADPF16(addr2 & ~uint64_t(15));
      else v2 = SM_LOAD16ST(addr2 & amask, st);
    }
    if (pfr) v3 = SM_LOADIDX(c.SA, (m + 1 + hi) >> 1);
    bool fresh = false;   // assigned a read this iteration: its first chunk loads next
    if (newm) {
      if (take) base = __shfl(base, int(__builtin_ctzll(newm)), 64);
      if (st == S_NEW) {
        fresh = true;
        const uint32_t r = uint32_t(__popcll(newm & ((1ull << lane) - 1)));
        rd = r < avail ? q_next + r : base + (r - avail);
        if (rd >= c.n_reads) {
          st = S_EXIT;
        } else {
          L = gLens ? gLens[rd] : gLen0;
          // records: the lane loads the bad-mask chunks, the read's bytes go
          // to its LDS row by DMA (below); direct rows: the row is DMA'd
          // from the read and the wave computes the mask next iteration
          addr = reinterpret_cast<uint64_t>(c.rec + rd * c.chunks);
          addr2 = addr + 16;
          need2 = !gDirect && c.c_bad > 1;
          pf = false; pfr = false;
          bad = Bad{0, 0, 0, 0, 0, 0, 0, 0};
          st = S_COPY;
        }
      }
      if (take) { q_next = base + (need - avail); q_end = base + take; }
      else q_next += need;
      // LDS-DMA of the raw chunks of each newly assigned read into its row;
      // the lane's own loads of the next iteration (its bad mask) wait for
      // it (vmcnt retires in order) before any row read
      uint64_t fm_ = __ballot(fresh && st == S_COPY);
      if (fm_) SM_REGION(26);
      while (fm_) {
        const uint32_t ln = uint32_t(__builtin_ctzll(fm_));
        fm_ &= fm_ - 1;
        const uint64_t rl = __shfl(rd, int(ln), 64);
        if (gDirect)
          SM_DMA_ROW(ldsw + ln * gRow, c.rows + rl * (gRow >> 2), gRow >> 2, lane);
        else
          SM_DMA_ROW(ldsw + ln * gRow, c.rec + rl * c.chunks + c.c_bad, c.chunks - c.c_bad, lane);
      }
    }
    if (st < S_ALU || fresh) continue;
    if (STATS) {
      ++it;
      atomicAdd(c.wave_stats + 2 + (st == S_IDX ? 16 + op : st == S_CMP ? 40 + op : st), 1ull);
    }
#ifdef SM_TRACE
    if (st != S_COPY)
      printf("it %u st %u op %u prefix %u depth %u [%llu,%llu] pos %llu hp %d\n", it, st, op, prefix,
             depth, (unsigned long long)start, (unsigned long long)end, (unsigned long long)pos,
             int(have_pos));
#endif
    const uint32_t ao = st >= S_BYTE ? 0u : uint32_t(addr) & 15;   // element offset in v
    uint32_t a = A_NONE;
    SM_REGION(0);
    // the scan states' byte masks, one computation shared by all four (their
    // bodies would otherwise each pay for it): bit i of mv / mv2 is byte i of
    // v / v2 > t_i, t_i = D - 1 - i for the U scan (U[.+i] + i >= D, D =
    // dch - j; v2 continues at D - 16) and xd - 1 for L8 runs (the complement:
    // L8 < xd, a stop)
    uint32_t mv = 0, mv2 = 0;
    if (st >= S_USCAN) {
      const bool us = st == S_USCAN;
      const uint32_t base = us ? dch - j - 1 : xd - 1;
      mv = thr_mask(v, base, us);
      mv2 = thr_mask(v2, us ? base - 16 : base, us);
    }

    // ---------------- consume ----------------
    switch (st) {
      case S_ALU:
        SM_REGION(1);
        a = pend;
        break;
      case S_COPY: {                                 // bad-mask chunks 0 (v), 1 (v2)
        SM_REGION(2);
        if (!gDirect) {   // (direct rows: the wave set the mask above)
          bad.w0 = v.x; bad.w1 = v.y; bad.w2 = v.z; bad.w3 = v.w;
          bad.w4 = v2.x; bad.w5 = v2.y; bad.w6 = v2.z; bad.w7 = v2.w;   // (zero: c_bad 1)
        }
        need2 = false;
        prefix = 0; depth = 0; start = 0; end = N - 1; have_pos = false; nem = 0;
        skip_f = false; fm = 0; ktr_set = false;
        fk = 0; kp = 0; kx = 0xFFFFFFFFu; fdead = false;
        clean = (bad.w0 | bad.w1 | bad.w2 | bad.w3 | bad.w4 | bad.w5 | bad.w6 | bad.w7) == 0;
        a = A_TOP;
        break;
      }
      case S_BM: {                                   // (F) a k-mer table entry arrived
        SM_REGION(3);
        const bool two = need2;   // (policy 3: v2 holds the entry 3 bases on)
        need2 = false;
        if (SM_KNOB(bm_dual, 3u) == 3) {
          // the entry of the k-mer at x = kp + fj + 2; c0 = the 2-bit codes of
          // the k + 4 read bases [x - 2, x + k + 2), first most significant:
          // its presence bits give the B-mers at x - 2, x - 1, x (common.hpp).
          // two: v2 / c1 are the same for the k-mer at x + 3
          const uint32_t nb = 2 * (gK + 4);
          auto entry_bits = [&](const uint4 &e, uint64_t cc) {
            const uint64_t f48 = kt_filter(lo64(e), hi64(e));
            const uint32_t l1 = uint32_t(cc >> (nb - 2)) & 3, l0 = uint32_t(cc >> (nb - 4)) & 3;
            const uint32_t r1 = uint32_t(cc >> 2) & 3, r2 = uint32_t(cc) & 3;
            return (uint32_t(f48 >> (32 + 4 * l1 + l0)) & 1u) |
                   ((uint32_t(f48 >> (16 + 4 * l0 + r1)) & 1u) << 1) |
                   ((uint32_t(f48 >> (4 * r1 + r2)) & 1u) << 2);
          };
          const uint32_t bits = entry_bits(v, c0);
          SM_HOOK_F(fj, bits);
          fk |= (7u << fj) | (bits << (16 + fj));
          fdead = bits != 7u;
          if (two) {
            const uint32_t bits2 = entry_bits(v2, c1);
            SM_HOOK_F(fj + 3, bits2);
            fk |= (7u << (fj + 3)) | (bits2 << (19 + fj));
            fdead = fdead || bits2 != 7u;
          }
          kx = kp + fj + 2;
          klo = lo64(v) & kKtMask;
          khi = hi64(v) & kKtMask;
          a = A_TOP;
          break;
        }
        // The last B-mer [q1, q1+B) (q1 = prefix+min_len-B) is probed first:
        // absent, it lies inside every window starting in [prefix, q1], so
        // all of them are skipped at once; an absent first B-mer rules out
        // this window only.  (bm_dual: v2 holds the first B-mer's entry.)
        // A B-mer's presence is bit (code & 15) of its first k-mer's entry.
        const uint64_t cc = bm2 ? c0 : c1;
        const bool pa = (lo64(v) >> (40 + (cc & 15))) & 1ull;
        const bool pb = !SM_KNOB(bm_dual, 3u) || ((lo64(v2) >> (40 + (c0 & 15))) & 1ull);
        if (SM_KNOB(bm_dual, 3u) == 2) {
          // cover policy (bm_dual 2): the pair probed depends on the mode fm
          // (A_TOP); an absent B-mer at s rules out the windows [s-D, s]
          // (D = min_len - B), so the window advances past every window an
          // absent probe covers.  Modes: 0 {L(p), F(p)}, 1 {L(p), L(p+D+1)},
          // 2 {F(p), F(p+1)} with L(p) known present.
          const uint32_t D = gMin - gB;
          const uint32_t fm0 = fm;
          SM_HOOK_BM(fm, pa, pb);
          uint32_t adv = 0, nfm = 0;
          bool pass = false;
          if (fm == 0) {
            if (!pa) { adv = D + 1; nfm = 1; }
            else if (!pb) adv = 1;
            else pass = true;
          } else if (fm == 1) {
            if (!pa && !pb) { adv = 2 * D + 2; nfm = 1; }
            else if (!pa) { adv = D + 1; nfm = 2; }   // L of the new window = the 2nd probe
            else nfm = 2;                               // L(p) present: same window
          } else {
            if (!pb) adv = 2;
            else if (!pa) adv = 1;
            else pass = true;
          }
          if (pass) {
            skip_f = true; fm = 1;                      // window passed: go on at (C)
            m = (fm0 == 0 ? c0 : c1) >> (2 * (gB - gK));   // F(p) -> the k-mer code
            ktr_set = true;
          } else {
            fm = nfm;
            if (adv) { depth = 0; start = 0; end = N - 1; have_pos = false; prefix += adv; }
          }
          a = A_TOP;
        } else if (!pa && !bm2) {
          depth = 0; start = 0; end = N - 1; have_pos = false;
          prefix += gMin - gB + 1;
          a = A_TOP;
        } else if (!pa || !pb) {
          depth = 0; start = 0; end = N - 1; have_pos = false; ++prefix; a = A_TOP;
        } else if (!bm2 && !SM_KNOB(bm_dual, 3u)) {
          bm2 = true;
          addr = reinterpret_cast<uint64_t>(c.KT + 2 * (c0 >> 4));
        } else {
          skip_f = true;                              // window passed: go on at (C)
          a = A_TOP;
        }
        break;
      }
      case S_KT: {                                   // (C)
        SM_REGION(4);
        const uint64_t l0 = lo64(v) & kKtMask, h0 = hi64(v) & kKtMask;
        if (l0 <= h0) { depth = gK; start = l0; end = h0; have_pos = false; }
        a = A_TRAV;
        break;
      }
      case S_IDX: {
        SM_REGION(5);
        const uint64_t iv = idx_val<IdxT>(v, ao);
        const uint64_t iv2 = idx_val<IdxT>(v2, uint32_t(addr2) & 15);
        // (PK: the ISA words of an expand_link's ends -- one word for a
        // suffix link's target (O_ISAJ), two for a non-singleton's; one site)
        if (PK && (op == O_ISAJ || op == O_NS_ISA2)) isa_hints(iv, op == O_ISAJ ? iv : iv2);
        if (op == O_SAPOS || op == O_SAPOS2) {
          pos = iv; have_pos = true;
          a = op == O_SAPOS ? A_TRAV : A_AFTER;
        } else if (op == O_BS_SA) {                   // probe m: compare from lcp lc
          sp = iv;
          // 16 bytes first: a binary-search probe usually decides early
          a = A_BSP;
        } else if (op == O_ISAJ) {
          start = end = iv & PM; have_pos = false;
          a = A_EXPAND;
        } else if (op == O_NS_SA2) {                  // suffix link, both ends
          addr = ia(c.ISA, (iv & PM) + 1); addr2 = ia(c.ISA, (iv2 & PM) + 1);
          op = O_NS_ISA2;
        } else {                                      // O_NS_ISA2
          start = iv & PM; end = iv2 & PM; need2 = false;
          ++prefix; have_pos = false;
          if (depth == 0) { start = 0; end = N - 1; a = A_TOP; }
          else a = A_EXPAND;
        }
        break;
      }
      case S_BYTE: {                                 // is_leftmaximal: T[pos-1]
        SM_REGION(6);
        SM_HOOK_BYTE(pos & PM);
        em = P[prefix - 1] != uint8_t(byte_at(v, ao));
        a = A_EMIT;
        break;
      }
      case S_CMP: {                                  // (A) extension / traverse probe
        SM_REGION(7);
        // text bytes [addr, addr + 16) in v, then (tn2) the next 16 in v2
        // (pf: v2 / v3 hold the children's SA elements instead)
        const bool tn2 = need2 && !pf;
        const uint32_t off = prefix + (op == O_BS ? cbase : depth) + lc;
        const uint32_t rem = op == O_BS ? cap - lc : L - off;
        const uint32_t lim = rem < 16 ? rem : 16u;
        uint32_t k = agree_block(v, 0, P, off, lim);
        if (tn2 && k == lim && k < rem) {
          const uint32_t lim2 = rem - k < 16 ? rem - k : 16u;
          k += agree_block(v2, 0, P, off + k, lim2);
        }
        const uint32_t got = tn2 ? (rem < 32 ? rem : 32u) : lim;   // bytes available
        const bool had_pf = pf;
        pf = false; pfr = false;
        lc += k;
        if (k == got && k < rem) {                    // agreed on all loaded bytes: go on
          addr += k;
          addr2 = addr + 16;
          need2 = rem - k > 16;
        } else if (op == O_EXT) {
          need2 = false;
          depth += lc; lc = 0;
          a = A_AFTER;
        } else {                                      // O_BS: probe m decided
          SM_HOOK_CMPBS(false, sp, cbase + lc);
          need2 = false;
          // P' < S_m iff P' ran out (prefix of S_m) or the first differing
          // byte of P' is smaller
          const uint32_t tbyte = k < 16 ? byte_at(v, k) : byte_at(v2, k - 16);
          bs_decide(k == rem, k == rem ? 0u : uint32_t(P[off + k]), tbyte);
          const bool left = hi == m;
          if (had_pf && lo < hi) {                    // the next probe's SA element is here
            m = (lo + hi) >> 1;
            SM_HOOK_PF(ia(c.SA, m));
            sp = left ? idx_val<IdxT>(v2, uint32_t(m * sizeof(IdxT)) & 15) : v3;
            lc = lL < lR ? lL : lR;
            a = A_BSP;
          } else {
            a = A_BS;
          }
        }
        break;
      }
      case S_USCAN: {                                // (B) first j with U[pos+j] >= d-j
        SM_REGION(8);
        // U bytes [addr, addr + 16) in v, then (need2) the next 16 in v2
        bool fin = false;
#pragma unroll
        for (uint32_t h = 0; h < 2; ++h) {
          if (fin || (h == 1 && !need2)) break;
          const uint32_t D = dch - j;
          const uint32_t lim = D < 16 ? D : 16u;
          const uint32_t inr = (1u << lim) - 1;
          const uint32_t hm = (h ? mv2 : mv) & inr;   // U[.+i] + i >= D
          if (hm) {
            j += uint32_t(__builtin_ctz(hm)); hit = true; fin = true;
          } else {
            j += lim;
            if (j >= dch) { hit = false; fin = true; }
          }
        }
        if (fin) {
          need2 = false;
          a = A_CHAIN_DONE;
        } else {
          addr += need2 ? 32 : 16;
          addr2 = addr + 16;
          need2 = SM_KNOB(u32, 1u) && dch - j > 16;
        }
        break;
      }
      case S_EXL:                                    // L8 runs: expand_link (xrun = 0)
      case S_EXR:                                    // or the traverse's final run (1);
      case S_EXB: {                                  // S_EXB: both sides in one iteration
        SM_REGION(9);
        const uint64_t lb = xrun ? start : 0, hb = xrun ? end : N - 1;
        // run members before the stop in one block, walking down (left:
        // bytes (o-lim, o]) or up (right: bytes [o, o+lim)); *more: no stop
        // in the window and room beyond it
        auto side = [&](uint32_t mask, uint32_t o, bool left, bool &more) {
          const uint64_t room = left ? es - lb : hb - ee;
          const uint32_t w = left ? o + 1 : 16 - o;
          const uint32_t lim = room < uint64_t(w) ? uint32_t(room) : w;
          const uint32_t below = ~mask & 0xFFFFu;      // L8 < xd
          const uint32_t win = left ? (((1u << lim) - 1) << (o + 1 - lim)) : (((1u << lim) - 1) << o);
          const uint32_t sm = below & win;
          const uint32_t k = sm ? (left ? o - (31 - __builtin_clz(sm)) : uint32_t(__builtin_ctz(sm)) - o)
                                : lim;
          more = !sm && uint64_t(k) < room;
          return k;
        };
        bool moreL = false, moreR = false;
        // the left block ends at es (position es - its start), the right one
        // starts at ee + 1 (position 0)
        if (st != S_EXR)
          es -= side(mv, uint32_t(es - (addr - reinterpret_cast<uint64_t>(c.L8))), true, moreL);
        if (st != S_EXL) {
          const bool b2 = st == S_EXB;
          ee += side(b2 ? mv2 : mv, 0u, false, moreR);
          if (b2) rdone = !moreR;
        }
        need2 = false;
        const bool left = st != S_EXR;                // the side that continues here
        const bool more = left ? moreL : moreR;
        if (!more) {
          a = left ? A_XL_DONE : A_RUN_DONE;
        } else if (++nblk < SM_KNOB(lin_blocks, 8u)) {
          addr = left ? lblock(es) : reinterpret_cast<uint64_t>(c.L8 + ee + 1);
          st = left ? S_EXL : S_EXR;
        } else {                                      // long run: bisect for its end
          bsm = left ? BS_LEFT : BS_RIGHT;
          if (left) { lo = lb; hi = es; lL = 0; lR = cap; }
          else { lo = ee + 1; hi = hb + 1; lL = cap; lR = 0; }
          a = A_BS;
        }
        break;
      }
      default:
        break;
    }

    if (gPad) {                                    // issue-bound experiment (SMASH_SM_PAD)
      // gPad dependent v_add per lane; the empty asm keeps every one of them
      // (an earlier form let the compiler sink the chain under a rare branch)
      uint32_t x = uint32_t(addr);
      for (uint32_t k = 0; k < gPad; ++k) {
        x += k;
        PAD_KEEP(x);
      }
    }

    // ---------------- decide ----------------
    if (a == A_BSP) {                                 // probe m's SA word is in sp
      a = bs_probe() ? A_BS : A_NONE;
    }
    if (a == A_BS) {                                  // next probe of a binary search
      SM_REGION(10);
      if (lo < hi) {
        m = (lo + hi) >> 1;
        lc = lL < lR ? lL : lR;
        addr = ia(c.SA, m);
        st = S_IDX; op = O_BS_SA;
        a = A_NONE;
      } else {
        a = A_BS_DONE;
      }
    }
    if (a == A_BS_DONE) {
      SM_REGION(11);
      lc = 0;
      if (bsm == BS_LEFT) {
        es = lo;                                      // first suffix of the run
        a = A_XL_DONE;
      } else if (bsm == BS_RIGHT) {
        ee = lo - 1;                                  // last suffix of the run
        a = A_RUN_DONE;
      } else if (best == 0) {
        a = A_AFTER;                                  // no longer match: interval unchanged
      } else {                                        // the run of suffixes sharing best more
        xd = depth + best; xrun = true;
        cbase = depth; cap = best;
        es = bi; ee = bi;
        SM_HOOK_RUN(true, 1, 0, 0);
        // packed: the SA word of rank bi holds L8[bi] and L8[bi + 1], the
        // run's first stop on either side when it ends at bi
        xls = PK && pk_below(bpos, 36, xd); xrs = PK && pk_below(bpos, 43, xd);
        a = A_EXS;
      }
    }
    if (a == A_EXPAND) {                              // expand_link (longSA.h:158-174)
      SM_REGION(15);
      // the run around [start, end] with L8 >= depth = the suffixes sharing
      // P[prefix, prefix+depth); it fails iff it holds >= thresh more
      thresh = 2u * depth * gLogN;
      xd = depth; xrun = false;
      cbase = 0; cap = depth;
      es = start; ee = end;
      SM_HOOK_RUN(true, 0, 0, 0);
      // packed: the ISA words of start and end hold L8[start - 1 .. start]
      // and L8[end + 1 .. end + 2]: a run that ends within one more suffix
      // on a side needs no L8 probe there
      if (PK) {
        if (xls && xl1) es = start - 1;
        if (xrs && xr1) ee = end + 1;
      }
      a = A_EXS;
    }
    if (a == A_EXS) {                                 // (one site: the two runs above)
      a = ex_start(xrun ? start : 0, xrun ? end : N - 1, xls, xrs) ? A_NONE : A_RUN_DONE;
    }
    if (a == A_XL_DONE) {                             // left end known: right side
      SM_REGION(12);
      const uint64_t hb = xrun ? end : N - 1;
      nblk = 0;
      if (!xrun && start - es >= thresh) {            // expand_link gives up (longSA.h:164)
        SM_HOOK_RUN(false, 0, start - es, 99);
        depth = 0; start = 0; end = N - 1; have_pos = false;
        a = A_TOP;
      } else if (ee < hb && !rdone) {
        addr = reinterpret_cast<uint64_t>(c.L8 + ee + 1);
        st = S_EXR;
        a = A_NONE;
      } else {
        a = A_RUN_DONE;
      }
    }
    if (a == A_RUN_DONE) {
      SM_REGION(13);
      SM_HOOK_RUN(false, xrun ? 1 : 0, xrun ? bi - es : start - es, xrun ? ee - bi : ee - end);
      if (xrun) {                                     // traverse result
        start = es; end = ee; depth = xd; pos = bpos; have_pos = start == end;
        a = A_AFTER;
      } else if ((start - es) + (ee - end) >= thresh) {
        depth = 0; start = 0; end = N - 1; have_pos = false;
        a = A_TOP;
      } else {                                        // expand_link succeeded
        start = es; end = ee;
        a = A_TOP;
      }
    }
    if (a == A_CHAIN_DONE) {
      SM_REGION(14);
      prefix += j;
      if (!hit) {
        depth = 0; start = 0; end = N - 1; have_pos = false;
        a = A_TOP;
      } else {
        depth = dch - j;
        addr = ia(c.ISA, (pos & PM) + j);
        st = S_IDX; op = O_ISAJ;
        a = A_NONE;
      }
    }
    if (a == A_TOP) {
      SM_REGION(17);
      uint32_t kpos = ~0u;                            // a k-mer table probe's read window
      // the read's bad bits [prefix, prefix + 64) as this A_TOP starts: the
      // window tests below are shifts of them (prefix only grows here, by at
      // most 16, and a test spans at most 36 bits past that); clean reads
      // (almost all) skip the extraction
      const uint32_t bp0 = prefix;
      uint64_t bwin = 0;
      if (!clean) bwin = bad.bits64(prefix);
      auto badw = [&](uint32_t p, uint32_t n) {
        return uint32_t(bwin >> (p - bp0)) & ((1u << n) - 1u);
      };
      // (F) runs while the state is shallow, once per prefix (skip_f: this
      // prefix's window already passed the bitmap)
      bool proceed = skip_f || depth >= gMin;
      const bool ktr = skip_f && ktr_set;             // k-mer code of this window in m
      skip_f = false; ktr_set = false;
      if (prefix >= L || (!proceed && prefix + gMin > L)) {
        a = A_DONE;
      } else if (!proceed) {
        SM_REGION(24);
        // bad-mask work only for reads holding a bad base (clean: none)
        int32_t kb = -1;
        const uint32_t B = gB;
        const uint32_t D = gMin - B;
        if (!clean) {
          SM_REGION(20);
          kb = bad.last(prefix, gMin);
          while (kb >= 0 && in_text(P[kb]))
            kb = bad.last(prefix, uint32_t(kb) - prefix);
        }
        if (kb >= 0) {                                // absent byte: next window
          depth = 0; start = 0; end = N - 1; have_pos = false;
          prefix = uint32_t(kb) + 1;                  // (A_TOP again: parks in S_ALU)
          fm = 0;
        } else if (SM_KNOB(bm_dual, 3u) == 3) {
          // (F) policy 3.  Window [p, p + min_len) can start a match only if
          // its D + 1 B-mers (offsets 0..D from p) all occur; an absent
          // B-mer at offset s rules out the windows s - D .. s.  One k-mer
          // entry tells three consecutive B-mers (k_kfilter), so the window's
          // D + 1 = 3 (B = k + 2 = min_len - 2) take one probe, and inside a
          // run of absent B-mers the entry D + 2 bases in rules out D + 3
          // windows at once.  What is known is kept per read position (fk).
          if (B != gK + 2 || B > gMin || D + 3 > 16) {
            proceed = true;                           // no filter for this geometry
          } else {
            const uint32_t sh = prefix - kp;         // (prefix never decreases)
            uint32_t kn = sh < 16 ? (fk & 0xFFFFu) >> sh : 0u;
            uint32_t pr = sh < 16 ? (fk >> 16) >> sh : 0u;
            kp = prefix;
            const uint32_t A = kn & ~pr;              // known absent B-mers
            uint32_t kill = A;                        // windows they rule out
            for (uint32_t i = 1; i <= D; ++i) kill |= A >> i;
            const uint32_t adv = uint32_t(__builtin_ctz(~kill));
            if (adv) {
              prefix += adv; kp = prefix;
              kn >>= adv; pr >>= adv;
              depth = 0; start = 0; end = N - 1; have_pos = false;
            }
            fk = kn | (pr << 16);
            const uint32_t need = (2u << D) - 1;     // offsets 0..D
            if (prefix + gMin > L) {
              a = A_DONE;
            } else if ((kn & pr & need) == need) {
              proceed = true;                         // the window passes: (C)
            } else {
              const uint32_t W = gK + 4;             // read bases one entry needs
              const uint32_t u = uint32_t(__builtin_ctz(~kn & need));   // lowest unknown
              auto ok_at = [&](uint32_t jj) {
                return prefix + jj + W <= L && badw(prefix + jj, W) == 0;
              };
              // after an absent B-mer, bet on a run of them: offsets D..D+2;
              // else the entry whose three B-mers start at the lowest
              // unknown u (or end there: near the read end the entry's
              // context must stay inside the read) -- every probe learns u
              uint32_t jq = (fdead && ((kn & need) >> u) == 0) ? D : u;
              if (!ok_at(jq)) jq = u;
              if (!ok_at(jq) && u >= 1) jq = u - 1;
              if (!ok_at(jq) && u >= 2) jq = u - 2;
              if (!ok_at(jq)) {
                proceed = true;                       // a non-ACGT text byte: no verdict
              } else {
                SM_REGION(21);
                fj = jq;
                kpos = prefix + jq;                   // the entry's window: below
                // the next three B-mers' entry too, when some of them are
                // unknown and its window lies in the read: a run of absent
                // B-mers (a segment junction) is crossed twice as fast
                // (f2 2: only inside a run of absent B-mers, where it pays).
                // Its bits land at offsets jq + 3 .. jq + 5 of fk's 16-bit
                // halves, so only when jq + 6 <= 16 (D <= 10; min_len >= 29
                // at B 18 takes one entry per probe)
                need2 = SM_KNOB(f2, 2u) && (SM_KNOB(f2, 2u) == 1 || fdead) && jq + 6 <= 16 &&
                        ((kn >> (jq + 3)) & 7u) != 7u && ok_at(jq + 3);
                st = S_BM;
                a = A_NONE;
              }
            }
          }
        } else {
          // policies 0-2: two B-mers per probe pair
          const uint32_t sM = prefix + 2 * D + 1;   // mode 1's second B-mer
          bool okP = true, okQ = true;              // [p, p+B), [p+D, p+D+B): inside the read
          bool okP1 = prefix + 1 + B <= L, okM = sM + B <= L;
          if (!clean) {
            okP = bad.bits(prefix, B) == 0;
            okQ = bad.bits(prefix + D, B) == 0;
            okP1 = okP1 && bad.bits(prefix + 1, B) == 0;
            okM = okM && bad.bits(sM, B) == 0;
          }
          // probes: c1 <- B-mer at s1 (v), c0 <- B-mer at s2 (v2); mode 0 is
          // {last, first} of this window, 1 and 2 (bm_dual 2) see S_BM
          uint32_t s1 = prefix + D, s2 = prefix;
          bool ok = okQ && okP;
          if (SM_KNOB(bm_dual, 3u) == 2 && fm == 1 && okQ && okM) {
            s2 = sM; ok = true;
          } else if (SM_KNOB(bm_dual, 3u) == 2 && fm == 2 && okP && okP1) {
            s1 = prefix; s2 = prefix + 1; ok = true;
          } else {
            fm = 0;
          }
          if (B > 0 && B <= gMin && ok) {
            // both codes from one pass over the row when the span allows
            const uint32_t lo_s = s1 < s2 ? s1 : s2, hi_s = s1 < s2 ? s2 : s1;
            const uint32_t span = hi_s + B - lo_s;
            if (span <= 21) {
              SM_REGION(21);
              const uint64_t X = codes_raw(row, gRow, lo_s, span);
              const uint64_t mk = (1ull << (2 * B)) - 1;
              c1 = (X >> (2 * (lo_s + span - s1 - B))) & mk;
              c0 = (X >> (2 * (lo_s + span - s2 - B))) & mk;
            } else {
              SM_REGION(22);
              c0 = codes_raw(row, gRow, s2, B);
              c1 = codes_raw(row, gRow, s1, B);
            }
            // a B-mer's presence: its first k-mer's entry (B = k + 2)
            addr = reinterpret_cast<uint64_t>(c.KT + 2 * (c1 >> 4));
            st = S_BM; bm2 = false;
            if (SM_KNOB(bm_dual, 3u)) { addr2 = reinterpret_cast<uint64_t>(c.KT + 2 * (c0 >> 4)); need2 = true; }
            a = A_NONE;
          } else {
            proceed = true;                             // no bitmap verdict
            fm = 1;
          }
        }
      }
      if (a == A_TOP && proceed) {                     // (C) from the root
        if (depth == 0 && prefix + gK <= L && badw(prefix, gK) == 0) {
          if (kx == prefix) {
            // the filter loaded this k-mer's entry already (policy 3)
            SM_REGION(25);
            if (klo <= khi) { depth = gK; start = klo; end = khi; have_pos = false; }
            a = A_TRAV;
          } else {
            // the window's first B-mer code (gB >= gK) from the filter pass
            SM_REGION(23);
            if (ktr) addr = reinterpret_cast<uint64_t>(c.KT + 2 * m);
            else kpos = prefix;
            st = S_KT;
            a = A_NONE;
          }
        } else {
          a = A_TRAV;
        }
      }
      // one row read for both k-mer table probes: the filter's entry (S_BM,
      // the 20 bases from kpos: its k-mer is bases 2..K+1, c0 keeps them all)
      // and the root's k-mer (S_KT, bases 0..K-1 of the same span)
      if (kpos != ~0u) {
        // (23 bases: the second filter entry's window is the last 20)
        const uint64_t kmask = (1ull << (2 * gK)) - 1;
        const uint64_t cw = codes_raw7(row, gRow, kpos, gK + 7);
        const bool fb = st == S_BM;
        if (fb) {
          c0 = cw >> 6;
          c1 = cw & ((1ull << (2 * (gK + 4))) - 1);
          addr2 = reinterpret_cast<uint64_t>(c.KT + 2 * ((c1 >> 4) & kmask));
        }
        addr = reinterpret_cast<uint64_t>(c.KT + 2 * ((cw >> (fb ? 10 : 14)) & kmask));
      }
    }
    if (a == A_TRAV) {
      SM_REGION(18);
      if (depth >= L || prefix + depth >= L) {
        a = A_AFTER;                                  // (backwards: parks in S_ALU)
      } else {
        a = A_NONE;
        if (start == end) {                          // (A) singleton: extend
          if (!have_pos) {
            addr = ia(c.SA, start);
            st = S_IDX; op = O_SAPOS;
          } else {
            addr = reinterpret_cast<uint64_t>(c.T + (pos & PM) + depth);
            addr2 = addr + 16;
            need2 = L - prefix - depth > 16;
            st = S_CMP; op = O_EXT; lc = 0;
          }
        } else {                                     // search [start, end] for P'
          SM_HOOK_BS(end - start + 1, depth);
          lo = start; hi = end + 1; lL = 0; lR = 0; best = 0;
          bsm = BS_INSERT; cbase = depth; cap = L - prefix - depth;
          m = (lo + hi) >> 1;
          lc = 0;
          addr = ia(c.SA, m);
          st = S_IDX; op = O_BS_SA;
        }
      }
    }
    if (a == A_AFTER) {
      SM_REGION(16);
      if (depth <= 1) {
        depth = 0; start = 0; end = N - 1; have_pos = false; ++prefix;
        a = A_TOP;
      } else {
        a = A_NONE;
        if (start != end) {                          // non-singleton suffix link
          --depth;
          addr = ia(c.SA, start); addr2 = ia(c.SA, end); need2 = true;
          st = S_IDX; op = O_NS_SA2;
        } else if (!have_pos) {
          addr = ia(c.SA, start);
          st = S_IDX; op = O_SAPOS2;
        } else if (depth >= gMin && prefix != 0 && (pos & PM) != 0 &&
                   (!PK || ((pos >> kPkPosBits) & 7u) >= 4u)) {
          addr = reinterpret_cast<uint64_t>(c.T + (pos & PM) - 1);
          st = S_BYTE;
        } else {
          // (PK: is_leftmaximal from the BWT character in pos's SA word)
          em = depth >= gMin &&
               (!PK || prefix == 0 || (pos & PM) == 0 ||
                P[prefix - 1] != pk_char(uint32_t(pos >> kPkPosBits) & 3u));
          a = A_EMIT;
        }
      }
    }
    if (a == A_EMIT) {                                // (one site: S_BYTE and A_AFTER)
      if (em) {
        if (nem < gCap)
          c.out[rd * gCap + nem] =
              pack_match(pos & PM, prefix, depth) | (PK && gMh ? pk_map_hint(pos) : 0ull);
        ++nem;
      }
      uscan_start(pos & PM, depth);
      a = A_NONE;
    }
    if (a == A_DONE) {
      SM_REGION(19);
      c.n_out[rd] = nem;
      if (STATS && c.iters) c.iters[rd] = it;
      it = 0;
      st = S_NEW;
    } else if (a != A_NONE) {
      SM_HOOK_PARK(a);
      pend = a;
      st = S_ALU;
    }
  }
  if (STATS && lane == 0) {
    atomicAdd(c.wave_stats, (unsigned long long)w_iters);
    atomicAdd(c.wave_stats + 1, (unsigned long long)w_active);
  }
}

}  // namespace sm
}  // namespace smash
