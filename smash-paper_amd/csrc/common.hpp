// smash-paper_amd/csrc/common.hpp -- shared internals of libsmashgpu (gfx950).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/smash_gpu.h"

namespace smash {

void set_error(const std::string &msg);

// The k-mer table (aux_build.hip), one 16-byte entry per ACGT k-mer w (2 bits
// per base, first base most significant): two u64 words whose low 40 bits
// hold the SA interval {lo, hi} of the suffixes starting with w (lo > hi: w
// does not occur) and whose high 24 bits hold, together, 48 presence bits of
// the (k+2)-mers that contain w (the (F) window filter of mam_sm.hpp):
//   bit r1*4 + r2          w r1 r2   occurs (the (k+2)-mer starting AT w)
//   bit 16 + l*4 + r       l w r     occurs (starting one base before w)
//   bit 32 + l1*4 + l2     l1 l2 w   occurs (starting two bases before w)
constexpr uint64_t kKtMask = (1ull << 40) - 1;
__host__ __device__ inline uint64_t kt_filter(uint64_t w0, uint64_t w1) {
  return (w0 >> 40) | ((w1 >> 40) << 24);
}
// is the (k+2)-mer with code c (2k + 4 bits) in the text: bit c & 15 of its
// first k-mer's entry (the "w r1 r2" bits live in the first word)
__host__ __device__ inline bool kt_bmer_present(const uint64_t *KT, uint64_t c) {
  return (KT[2 * (c >> 4)] >> (40 + (c & 15))) & 1ull;
}

#define SMASH_HIP(call)                                                      \
  do {                                                                       \
    hipError_t e_ = (call);                                                  \
    if (e_ != hipSuccess) {                                                  \
      ::smash::set_error(std::string(#call) + ": " + hipGetErrorString(e_)); \
      return SMASH_ERR_HIP;                                                  \
    }                                                                        \
  } while (0)

// Throwing variant for internal helpers; converted to a status at the ABI.
struct hip_failure {
  std::string what;
};
#define SMASH_HIPX(call)                                                       \
  do {                                                                         \
    hipError_t e_ = (call);                                                    \
    if (e_ != hipSuccess)                                                      \
      throw ::smash::hip_failure{std::string(#call) + ": " +                   \
                                 hipGetErrorString(e_)};                       \
  } while (0)

template <class T>
T *dalloc(size_t n) {
  void *p = nullptr;
  if (n == 0) n = 1;
  hipError_t e = hipMalloc(&p, n * sizeof(T));
  if (e != hipSuccess)
    throw hip_failure{"hipMalloc(" + std::to_string(n * sizeof(T)) +
                      " B): " + hipGetErrorString(e)};
  return static_cast<T *>(p);
}
inline void dfree(void *p) {
  if (p) (void)hipFree(p);
}

inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap = 1u << 20) {
  uint64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<unsigned>(g);
}

inline uint64_t ceil_log2(uint64_t n) {
  uint64_t b = 0;
  while ((1ull << b) < n && b < 63) ++b;
  return b;
}

// Packed index words (round 5, pack_index.hip): a 64-bit SA / ISA element
// needs 33 bits at hg19 (N < 2^33); the search keeps hints for its next
// probes in the other 31, so they come with the element it loads anyway:
//   SA[r]  bits  0..32  the text position x = SA[r]
//                33..35 tag: 0..3 = T[x - 1] (a c g t, the BWT character, for
//                       is_leftmaximal) and the window below is exact;
//                       4 = T[x - 1] another byte (or x = 0), window exact;
//                       5 = the window holds a byte other than a c g t
//                36..42 min(L8[r], 127)       43..49 min(L8[r + 1], 127)
//                50..63 T[x + K .. x + K + 7), 2 bits per base (a0 c1 g2 t3,
//                       base i at bit 50 + 2i; K = the k-mer table's k)
//   ISA[x] bits  0..32  the rank r = ISA[x]
//                33..39 min(L8[r - 1], 127)   40..46 min(L8[r], 127)
//                47..53 min(L8[r + 1], 127)   54..60 min(L8[r + 2], 127)
// (L8 bytes outside [0, N) are 0).  A capped 127 compares exactly with any
// depth <= 127; every other reader masks the position bits (IdxArr).
constexpr uint32_t kPkPosBits = 33;
constexpr uint64_t kPkPosMask = (uint64_t(1) << kPkPosBits) - 1;
constexpr uint32_t kPkWindow = 7;   // bases in the SA word

// SA / ISA read through the position mask (~0 for a plain index)
template <class IdxT>
struct IdxArr {
  const IdxT *p;
  uint64_t mask;
  __host__ __device__ uint64_t operator[](uint64_t i) const { return uint64_t(p[i]) & mask; }
};

// Packed match (smash_gpu.h): ref 48 | qoff 8 | len 8
__host__ __device__ inline uint64_t pack_match(uint64_t ref, uint32_t q,
                                               uint32_t len) {
  return (ref & 0xFFFFFFFFFFFFull) | (uint64_t(q & 0xFF) << 48) |
         (uint64_t(len & 0xFF) << 56);
}

}  // namespace smash

// The device index (smash_gpu.h: smash_index).  SA/ISA width is 4 bytes when
// N < 2^32, else 8 (the reference's ANINT, size.h:24-38).
struct smash_index {
  int device = 0;
  uint64_t N = 0, logN = 0;
  uint32_t idx_bytes = 4;
  uint32_t n_seq = 0;
  bool rcref = true;             // text layout: -rcref (2 entries per contig) or forward only
  std::vector<uint64_t> startpos, sizes;
  std::vector<std::string> names;
  uint8_t *d_text = nullptr;     // N + 64 (zero pad)
  void *d_sa = nullptr;
  void *d_isa = nullptr;
  uint8_t *d_lcp8 = nullptr;     // min(LCP,255)
  uint64_t *d_ovf = nullptr;     // {idx,val} for LCP >= 255, sorted
  uint64_t n_ovf = 0;
  uint8_t *d_map = nullptr;
  uint64_t map_bytes = 0;
  // map.bin was computed here from this index (build_map), not read from a
  // file: the search's map hints (SearchWs::mhint) may stand in for its bytes
  bool map_own = false;
  uint64_t pos_mask = ~0ull;     // kPkPosMask when SA / ISA carry packed hints (pack_index.hip)
  uint8_t *d_uniq = nullptr;     // U[x] (aux_build.hip), N + 64
  mutable uint64_t *d_nsdir = nullptr;   // first U < 255 per 4096 positions (mappability.hip)
  uint8_t *d_uscratch = nullptr; // U's partition passes (uniq_build.hip), kept between
  uint64_t uscratch_bytes = 0;   // smash_mappability_prepare calls until released
  hipStream_t uaux = nullptr;    // the partition passes' second stream (chunks alternate)
  hipEvent_t uev[2] = {nullptr, nullptr};   // its start (after pass 1) and end events
  uint64_t *d_kmer = nullptr;    // per k-mer: {lo,hi} + (k+2)-mer presence bits (kt_filter)
  uint32_t kmer_k = 0;
  uint64_t *d_bitmap = nullptr;  // (none since round 3: the presence bits live in d_kmer)
  uint32_t bitmap_b = 0;         // B = k + 2, the filter's B-mer length
  uint64_t in_text[4] = {0, 0, 0, 0};   // bytes occurring in the text
  uint64_t *d_work = nullptr;    // k_mam work counter (stream-ordered use)
  // k_mam_sm read records (mam_sm.hpp k_prep), grown on demand by
  // smash_map_batch; like d_work, one batch in flight per index
  mutable uint32_t *d_rec = nullptr;
  mutable uint64_t rec_bytes = 0;
  // optional event pair recorded right around the k_mam_sm launch (set by
  // smash_pipeline profiling for the duration of one smash_map_batch call)
  mutable hipEvent_t kev[2] = {nullptr, nullptr};
  uint64_t *d_startpos = nullptr;
  uint64_t *d_sizes = nullptr;
  double build_seconds = 0;
  uint64_t device_bytes = 0;
};

namespace smash {
// sa_build.hip
void build_sa_isa(smash_index *ix, hipStream_t s);       // fills d_sa, d_isa
uint32_t *build_lcp32(smash_index *ix, hipStream_t s);   // exact LCP (u32, saturating)
void finish_lcp(smash_index *ix, const uint32_t *d_lcp32, hipStream_t s);  // lcp8 + ovf
void build_map(smash_index *ix, const uint32_t *d_lcp32, hipStream_t s);   // map.bin
void build_aux(smash_index *ix, hipStream_t s);   // U + k-mer table (aux_build.hip)
// the packed SA / ISA hints (pack_index.hip; after every build step that reads
// SA or ISA); pack = false: strip them (plain words)
void pack_index(smash_index *ix, bool pack, hipStream_t s);
// U for text positions [lo, hi) from SA + L8 (uniq_build.hip; lo rounded down to 64)
void build_uniq_range(smash_index *ix, uint64_t lo, uint64_t hi, hipStream_t s);
void release_uniq_scratch(smash_index *ix);   // the passes' scratch HBM
// mam.hip: smash_map_batch without the per-launch synchronisation of the
// probe check (sync_check = false: the caller runs probe_check later)
// caller-owned search workspace (the pipeline's double-buffered sets): the
// read records and the work counter of one k_mam_sm launch, so two launches
// on different streams can run at once; null: the index's own
struct SearchWs {
  uint8_t *rec = nullptr;
  uint64_t rec_bytes = 0;
  unsigned long long *work = nullptr;
  // waited on between the read records (k_prep) and the search: the match
  // buffers' previous reader, so the records of the next batch are built
  // while that reader still runs
  hipEvent_t gate = nullptr;
  // the pipeline's packed-index searches: match words carry the map hint
  // (sm::Ctx::mhint; bits 40..47, the post stage masks the reference to 40)
  bool mhint = false;
};
int map_batch_impl(const smash_index *ix, int mode, uint32_t min_len, const uint8_t *d_seqs,
                   uint64_t stride, const uint16_t *d_lens, uint32_t len, uint64_t n_reads,
                   uint64_t *d_out, uint32_t cap_per_read, uint32_t *d_n_out, void *stream,
                   bool sync_check, const SearchWs *ws = nullptr);
// record bytes of n reads of up to max_len bases (k_prep)
uint64_t search_rec_bytes(uint64_t n_reads, uint32_t max_len);
// the search takes these reads as direct rows (no records): native stride,
// 16-byte aligned (mam.hip; SMASH_DIRECT_ROWS=0 turns it off for A/B)
bool search_direct(const uint8_t *seqs, uint64_t stride, uint32_t len);
// grow the single-GPU key set before a batch of n_next pairs could overflow
// it (pipeline.hip; synchronous when it grows)
int ensure_keys(smash_pipeline *p, uint64_t n_next, hipStream_t s);
// one pipeline batch whose search waits for in_ev (null: for all earlier
// work on s) instead of for everything on s (pipeline.hip)
int count_batch_ev(smash_pipeline *p, const uint8_t *d_reads, uint64_t n_pairs,
                   uint64_t *d_counts, hipStream_t s, hipEvent_t in_ev);
int probe_check(const smash_index *ix);   // synchronous; SMASH_OK or the probe error
// mem.hip: smash_map_batch's MUM mode (MAM, then cleanMUMcand per read)
int map_batch_mum(const smash_index *ix, uint32_t min_len, const uint8_t *seqs, uint64_t stride,
                  const uint16_t *lens, uint32_t len, uint64_t n_reads, uint64_t *out, uint32_t cap,
                  uint32_t *n_out, hipStream_t s);
}  // namespace smash
