// smash-paper_amd/csrc/mam.hip -- per-read MAM search on gfx950.
//
// Replaces longSA::MAM (longSA.cpp:503-536) with traverse/top_down_faster
// (:297-380), the inline suffix link + expand_link (longSA.h:158-174) and
// is_leftmaximal (:540-546).  One read per lane; the read is staged in LDS;
// the SA interval lives in registers.  The work is chains of dependent
// random loads into the HBM-resident SA / ISA / text / LCP (no MFMA).
//
// Results are identical to the reference because the match set is a pure
// function of (read, index): the same probe sequence is executed.  LCP is
// read from the u8 array saturated at 255: expand_link only asks
// LCP >= depth with depth <= read length <= 255, for which
// min(LCP,255) >= depth <=> LCP >= depth, so the reference's overflow
// lower_bound (longSA.h:34-39) is never needed on this path.
#include "common.hpp"
#include "mam_device.hpp"
#include "mam_sm.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>

namespace smash {
namespace {

// Persistent grid sized to the resident capacity; each lane pulls the next
// read from a device work counter as soon as its previous read is done, so a
// slow read (repeats: large intervals) delays only its own lane instead of a
// whole block.  The read is copied into the lane's LDS row.
template <class IdxT, int BLOCK, bool PLAIN>
__global__ __launch_bounds__(BLOCK) void k_mam(
    DevIndex<IdxT> x, const uint8_t *__restrict__ seqs, uint64_t stride,
    const uint16_t *__restrict__ lens, uint32_t len0, uint64_t n_reads,
    uint32_t min_len, uint64_t *__restrict__ out, uint32_t cap,
    uint32_t *__restrict__ n_out, uint32_t row, unsigned long long *work) {
  extern __shared__ uint8_t lds[];
  uint8_t *P = lds + threadIdx.x * row;
  for (;;) {
    const uint64_t r = atomicAdd(work, 1ull);
    if (r >= n_reads) break;
    const uint32_t L = lens ? lens[r] : len0;
    // lane-private copy with aligned 4-byte global loads
    const uint8_t *src = seqs + r * stride;
    const uintptr_t a = reinterpret_cast<uintptr_t>(src);
    const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
    const uint32_t sh = uint32_t(a & 3);
    const uint32_t nw = (L + sh + 3) >> 2;
    for (uint32_t k = 0; k < nw; ++k) {
      const uint32_t v = w[k];
#pragma unroll
      for (uint32_t b = 0; b < 4; ++b) {
        const int32_t o = int32_t(4 * k + b) - int32_t(sh);
        if (o >= 0 && uint32_t(o) < L) P[o] = uint8_t(v >> (8 * b));
      }
    }
    MatchSink sink{out + r * cap, cap, 0};
    if (PLAIN) mam_read_plain(x, P, L, min_len, sink);
    else mam_read_v3(x, P, L, min_len, sink);
    n_out[r] = sink.n;
  }
}

// SMASH_MODE_MAM default: the state-machine kernel (mam_sm.hpp).  Setting
// SMASH_MAM_KERNEL=direct selects the direct per-lane v3 kernel instead (same
// results; kept for A/B measurement).
// 64-lane blocks: the LDS row of a lane is its read (40 words at 150 bp), so
// 16 blocks (4 waves per SIMD, the VGPR limit) fit the CU's 160 KB.
constexpr int kSmBlock = 64;

template <class IdxT, bool STATS, bool CHECK>
int run_sm(const smash_index *ix, const sm::Ctx<IdxT> &c0, uint64_t n_reads, size_t lds,
           hipStream_t s, bool sync_check) {
  constexpr int B = kSmBlock;
  // CHECK: every probe is checked against the span of the index arrays and
  // the records: a wild address retires its lane and fails the call instead
  // of faulting the GPU.
  // the packed-word instantiation for an index whose 8-byte SA / ISA words
  // carry the search's hints (pack_index.hip); the plain kernel reads whole
  // elements, so an A/B of the two runs over an unpacked index
  // (SMASH_PACK_IDX=0 or smash_index_pack) instead
  const bool pk = sizeof(IdxT) == 8 && ix->pos_mask == kPkPosMask;
  auto kern = pk ? sm::k_mam_sm<IdxT, B, CHECK, STATS, sizeof(IdxT) == 8>
                 : sm::k_mam_sm<IdxT, B, CHECK, STATS, false>;
  // the production geometries as compile-time constants (k_mam_sm GEO = L):
  // packed words, L-base direct rows (L = 150: C3 / C4; L = 100: C2), K 16 /
  // B 18 / min_len 20, L - 19 match slots, map hints, 2^32 < N <= 2^33
  // (every value the kernel folds)
  static const bool geo_env = [] {
    const char *e = std::getenv("SMASH_SM_GEO");
    return !(e && e[0] == '0');
  }();
  if (pk && !STATS && geo_env && c0.K == 16 && c0.B == 18 && c0.min_len == 20 &&
      c0.direct == 1 && c0.pad == 0 && !c0.lens && c0.mhint && c0.logN == 33 &&
      c0.cap == c0.len0 - 19 && c0.w_row == sm::geo_row(c0.len0)) {
    if (c0.len0 == 150) kern = sm::k_mam_sm<IdxT, B, CHECK, STATS, sizeof(IdxT) == 8, 150>;
    else if (c0.len0 == 100) kern = sm::k_mam_sm<IdxT, B, CHECK, STATS, sizeof(IdxT) == 8, 100>;
  }
  int per_cu = 0, cus = 0;
  SMASH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu, reinterpret_cast<const void *>(kern), B, lds));
  SMASH_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix->device));
  if (per_cu < 1) per_cu = 1;
  if (const char *e = std::getenv("SMASH_SM_BLOCKS_PER_CU")) {   // occupancy experiments
    const int cap = std::atoi(e);
    if (cap >= 1 && cap < per_cu) per_cu = cap;
  }
  uint64_t blocks = uint64_t(per_cu) * uint64_t(cus);
  const uint64_t want = (n_reads + B - 1) / B;
  if (blocks > want) blocks = want;
  sm::Ctx<IdxT> c = c0;
  std::vector<uint32_t> h_iters;
  if (STATS) {
    SMASH_HIP(hipMalloc(&c.iters, n_reads * sizeof(uint32_t)));
    SMASH_HIP(hipMalloc(&c.wave_stats, 128 * 8));
    SMASH_HIP(hipMemsetAsync(c.wave_stats, 0, 128 * 8, s));
  }
  // d_work[1..10]: sticky probe-check record (zeroed at index creation,
  // never reset): the pipeline reads it at stats time, so a batch does not
  // synchronise the stream (smash::probe_check)
  c.viol = reinterpret_cast<unsigned long long *>(ix->d_work) + 1;
  SMASH_HIP(hipMemsetAsync(c.work, 0, 8, s));
  if (ix->kev[0]) SMASH_HIP(hipEventRecord(ix->kev[0], s));
  kern<<<unsigned(blocks), B, lds, s>>>(c);
  SMASH_HIP(hipGetLastError());
  if (ix->kev[1]) SMASH_HIP(hipEventRecord(ix->kev[1], s));
  if (CHECK && sync_check) {
    SMASH_HIP(hipStreamSynchronize(s));
    if (int rc = probe_check(ix)) return rc;
  }
  if (STATS) {
    std::vector<uint32_t> hv(n_reads);
    unsigned long long ws[128];
    SMASH_HIP(hipMemcpy(hv.data(), c.iters, n_reads * 4, hipMemcpyDeviceToHost));
    SMASH_HIP(hipMemcpy(ws, c.wave_stats, 128 * 8, hipMemcpyDeviceToHost));
    SMASH_HIP(hipFree(c.iters));
    SMASH_HIP(hipFree(c.wave_stats));
    std::vector<uint32_t> srt(hv);
    std::sort(srt.begin(), srt.end());
    double sum = 0;
    for (uint32_t v : hv) sum += v;
    auto q = [&](double f) { return srt[std::min<size_t>(srt.size() - 1, size_t(f * srt.size()))]; };
    std::fprintf(stderr,
                 "[k_mam_sm] reads %llu blocks %llu (%d/CU) row %u words: lane-iterations/read mean %.1f "
                 "p50 %u p90 %u p99 %u p99.9 %u max %u; wave-iterations %llu, active lanes/iteration %.2f\n",
                 (unsigned long long)n_reads, (unsigned long long)blocks, per_cu, c.w_row, sum / n_reads,
                 q(0.5), q(0.9), q(0.99), q(0.999), srt.back(), ws[0],
                 double(ws[1]) / double(ws[0] ? ws[0] : 1));
    static const char *names[] = {"EXIT", "NEW", "ALU", "COPY", "BM", "KT", "IDX", "BYTE", "CMP",
                                  "USCAN", "EXL", "EXR", "EXB"};
    static const char *idx_ops[] = {"SAPOS", "SAPOS2", "SCAN_SA", "ISAJ", "NS_SA2", "NS_ISA2",
                                    "TD_SA2", "TD_SA"};
    static const char *byte_ops[] = {"TD_T2", "TD_T", "LM"};
    std::fprintf(stderr, "[k_mam_sm] lane-iterations per read by state:");
    for (int k = 0; k < 13; ++k)
      if (ws[2 + k]) std::fprintf(stderr, " %s %.1f", names[k], double(ws[2 + k]) / n_reads);
    for (int k = 0; k < 8; ++k)
      if (ws[18 + k]) std::fprintf(stderr, " IDX.%s %.1f", idx_ops[k], double(ws[18 + k]) / n_reads);
    for (int k = 0; k < 3; ++k)
      if (ws[34 + k]) std::fprintf(stderr, " BYTE.%s %.1f", byte_ops[k], double(ws[34 + k]) / n_reads);
    for (int k = 0; k < 2; ++k)
      if (ws[42 + k]) std::fprintf(stderr, " CMP.%s %.1f", k ? "SCAN" : "EXT", double(ws[42 + k]) / n_reads);
    std::fprintf(stderr, "\n");
    // SM_REGION counters: share of wave iterations each code region ran in
    static const char *regions[] = {
        "consume", "S_ALU", "S_COPY", "S_BM", "S_KT", "S_IDX", "S_BYTE", "S_CMP", "S_USCAN",
        "S_EX", "A_BS", "A_BS_DONE", "A_XL_DONE", "A_RUN_DONE", "A_CHAIN_DONE", "A_EXPAND",
        "A_AFTER", "A_TOP", "A_TRAV", "A_DONE", "TOP.!clean", "TOP.codes1", "TOP.codes2",
        "TOP.kt", "TOP.filter", "TOP.kcache", "dma", "rowbad"};
    std::fprintf(stderr, "[k_mam_sm] wave iterations running each region (%%):");
    for (int k = 0; k < 28; ++k)
      if (ws[64 + k])
        std::fprintf(stderr, " %s %.1f", regions[k], 100.0 * double(ws[64 + k]) / double(ws[0] ? ws[0] : 1));
    std::fprintf(stderr, "\n");
  }
  return SMASH_OK;
}

template <class IdxT>
int launch_sm(const smash_index *ix, uint32_t min_len, const uint8_t *seqs,
              uint64_t stride, const uint16_t *lens, uint32_t len,
              uint64_t n_reads, uint64_t *out, uint32_t cap, uint32_t *n_out,
              hipStream_t s, bool sync_check, const SearchWs *ws) {
  constexpr int B = kSmBlock;
  const sm::Geom g = sm::make_geom(lens ? 255 : len);
  // direct rows: the reads are the device's native rows (16-byte aligned,
  // 4 w_row bytes apart, zero padded: smash_read_stride) -- the search DMAs
  // each straight from its row and needs no records
  const bool direct = !lens && search_direct(seqs, stride, len);
  // read records (k_prep): the caller's workspace, else the index's buffer
  const uint64_t need = direct ? 0 : n_reads * g.chunks * 16;
  uint32_t *rec = ws ? reinterpret_cast<uint32_t *>(ws->rec) : nullptr;
  if (ws && need > ws->rec_bytes) {
    set_error("k_mam_sm: search workspace too small");
    return SMASH_ERR_ARG;
  }
  if (!ws && need > ix->rec_bytes) {
    SMASH_HIP(hipStreamSynchronize(s));
    if (ix->d_rec) SMASH_HIP(hipFree(ix->d_rec));
    ix->d_rec = nullptr;
    ix->rec_bytes = 0;
    const uint64_t bytes = need + need / 4;
    SMASH_HIP(hipMalloc(&ix->d_rec, bytes));
    ix->rec_bytes = bytes;
  }
  if (!ws) rec = ix->d_rec;
  const uint32_t ga = sm::prep_groups(lens ? 255 : len);
  // records (not for direct rows): k_prep (LDS-staged, the default:
  // profiles/r03/sched) or, with SMASH_PREP_LDS=0, k_prep_direct (no LDS: it
  // fits beside a running search but moves ~2x the bytes)
  const char *pl = std::getenv("SMASH_PREP_LDS");
  if (direct) {
  } else if (!(pl && pl[0] == '0') || n_reads * ga >= (1ull << 32)) {
    const uint32_t per = sm::prep_per_block(g, stride);
    const size_t plds = sm::prep_lds_bytes(g, stride, per);
    sm::k_prep<<<unsigned((n_reads + per - 1) / per), 256, plds, s>>>(
        seqs, stride, lens, len, n_reads, ix->in_text[0], ix->in_text[1], ix->in_text[2],
        ix->in_text[3], g, per, rec);
    SMASH_HIP(hipGetLastError());
  } else if (n_reads) {
    const uint64_t items = n_reads * ga;
    sm::k_prep_direct<<<unsigned((items + 255) / 256), 256, 0, s>>>(
        seqs, stride, lens, len, uint32_t(n_reads), ga, ix->in_text[0], ix->in_text[1],
        ix->in_text[2], ix->in_text[3], g, rec, 1u);   // raised priority beside a running search
    SMASH_HIP(hipGetLastError());
  }
  if (ws && ws->gate) SMASH_HIP(hipStreamWaitEvent(s, ws->gate, 0));
  sm::Ctx<IdxT> c;
  const DevIndex<IdxT> x = make_dev_index<IdxT>(ix);
  c.T = x.T; c.SA = x.SA.p; c.ISA = x.ISA.p; c.L8 = x.L8; c.U = x.U; c.KT = x.KT;
  c.N = x.N; c.logN = uint32_t(x.logN); c.K = uint32_t(x.K); c.B = uint32_t(x.B);
  c.min_len = min_len;
  c.rec = reinterpret_cast<const uint4 *>(rec);
  c.chunks = g.chunks; c.c_bad = g.c_bad; c.w_row = g.w_row; c.w_raw = g.w_raw;
  c.rows = direct ? reinterpret_cast<const uint4 *>(seqs) : nullptr;
  c.direct = direct ? 1u : 0u;
  sm::bad_table(ix->in_text, &c.bad_tab_lo, &c.bad_tab_hi);
  c.lin_blocks = 8;
  c.pad = 0;
  c.grab = 16;
  c.bm_dual = 3;
  c.pf = 1;
  c.u32 = 1;
  c.f2 = 2;
  // (pf, u32, bm_dual, grab and lin_blocks are the kernel's compile-time
  // defaults on the device, SM_KNOB in mam_sm.hpp: the fields above only
  // document them; tools/sm_emu varies them.  The environment variables that
  // set them in the emulator do nothing here: say so once.)
  static const bool knob_warned = [] {
    const char *names[] = {"SMASH_SM_BM_DUAL", "SMASH_SM_PF", "SMASH_SM_U32", "SMASH_SM_GRAB",
                           "SMASH_SM_LIN", "SMASH_SM_F2"};
    for (const char *n : names)
      if (std::getenv(n))
        std::fprintf(stderr, "smash: %s is an emulator knob (tools/sm_emu); the device kernel "
                             "uses its compile-time default\n", n);
    return true;
  }();
  (void)knob_warned;
  if (const char *e = std::getenv("SMASH_SM_PAD")) c.pad = uint32_t(std::atoi(e));
  c.mhint = ws && ws->mhint ? 1u : 0u;
  c.lens = lens; c.len0 = len; c.cap = cap; c.n_reads = n_reads;
  c.out = out; c.n_out = n_out;
  c.work = ws ? ws->work : reinterpret_cast<unsigned long long *>(ix->d_work);
  for (int k = 0; k < 4; ++k) c.in_text[k] = ix->in_text[k];
  c.iters = nullptr;
  c.wave_stats = nullptr;
  {
    const uint64_t N = ix->N, isz = ix->idx_bytes;
    const uint64_t spans[7][2] = {
        {reinterpret_cast<uint64_t>(ix->d_text), N + 64},
        {reinterpret_cast<uint64_t>(ix->d_sa), N * isz},
        {reinterpret_cast<uint64_t>(ix->d_isa), N * isz},
        {reinterpret_cast<uint64_t>(ix->d_lcp8), N + 64},
        {reinterpret_cast<uint64_t>(ix->d_uniq), N + 64},
        {reinterpret_cast<uint64_t>(ix->d_kmer), 16ull << (2 * ix->kmer_k)},
        {direct ? reinterpret_cast<uint64_t>(seqs) : reinterpret_cast<uint64_t>(rec),
         direct ? n_reads * stride : n_reads * g.chunks * 16}};
    c.lo = ~0ull; c.hi = 0;
    for (int k = 0; k < 7; ++k) {
      c.lo = std::min<uint64_t>(c.lo, spans[k][0]);
      c.hi = std::max<uint64_t>(c.hi, spans[k][0] + spans[k][1]);
    }
  }
  const size_t lds = size_t(B) * g.w_row * 4;
  if (std::getenv("SMASH_SM_STATS")) return run_sm<IdxT, true, true>(ix, c, n_reads, lds, s, true);
  const char *ck = std::getenv("SMASH_SM_CHECK");
  if (ck && ck[0] == '0') return run_sm<IdxT, false, false>(ix, c, n_reads, lds, s, sync_check);
  return run_sm<IdxT, false, true>(ix, c, n_reads, lds, s, sync_check);
}

bool use_direct() {
  const char *e = std::getenv("SMASH_MAM_KERNEL");
  return e && std::strcmp(e, "direct") == 0;
}

template <class IdxT, bool PLAIN>
int launch(const smash_index *ix, uint32_t min_len, const uint8_t *seqs,
           uint64_t stride, const uint16_t *lens, uint32_t len,
           uint64_t n_reads, uint64_t *out, uint32_t cap, uint32_t *n_out,
           hipStream_t s) {
  constexpr int B = 128;
  uint32_t maxL = lens ? 255 : len;
  uint32_t row = (maxL + 3) / 4 + 1;   // +1 word: lds_load8 over-read
  if ((row & 1) == 0) ++row;   // odd word stride: conflict-free LDS rows
  row *= 4;
  const size_t lds = size_t(B) * row + 16;
  int per_cu = 0, cus = 0;
  SMASH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu, reinterpret_cast<const void *>(k_mam<IdxT, B, PLAIN>), B, lds));
  SMASH_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix->device));
  if (per_cu < 1) per_cu = 1;
  uint64_t blocks = uint64_t(per_cu) * uint64_t(cus);
  const uint64_t need = (n_reads + B - 1) / B;
  if (blocks > need) blocks = need;
  DevIndex<IdxT> x = make_dev_index<IdxT>(ix);
  SMASH_HIP(hipMemsetAsync(ix->d_work, 0, 8, s));
  if (ix->kev[0]) SMASH_HIP(hipEventRecord(ix->kev[0], s));
  k_mam<IdxT, B, PLAIN><<<unsigned(blocks), B, lds, s>>>(
      x, seqs, stride, lens, len, n_reads, min_len, out, cap, n_out, row,
      reinterpret_cast<unsigned long long *>(ix->d_work));
  SMASH_HIP(hipGetLastError());
  if (ix->kev[1]) SMASH_HIP(hipEventRecord(ix->kev[1], s));
  return SMASH_OK;
}

}  // namespace
}  // namespace smash

namespace smash {

// The sticky probe-check record of k_mam_sm (d_work[1..10]); synchronous.
int probe_check(const smash_index *ix) {
  unsigned long long h[10];
  SMASH_HIP(hipMemcpy(h, ix->d_work + 1, sizeof(h), hipMemcpyDeviceToHost));
  if (!h[0]) return SMASH_OK;
  char msg[512];
  std::snprintf(msg, sizeof(msg),
                "k_mam_sm: %llu probes outside the index; first: state %llu op %llu addr %#llx "
                "addr2 %#llx prefix %llu depth %llu interval [%llu,%llu] read %llu",
                h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9]);
  std::fprintf(stderr, "%s\n", msg);
  set_error(msg);
  return SMASH_ERR_HIP;
}

bool search_direct(const uint8_t *seqs, uint64_t stride, uint32_t len) {
  static const bool off = std::getenv("SMASH_DIRECT_ROWS") && std::getenv("SMASH_DIRECT_ROWS")[0] == '0';
  return !off && len && stride == 4ull * sm::make_geom(len).w_row &&
         (reinterpret_cast<uint64_t>(seqs) & 15) == 0;
}

uint64_t search_rec_bytes(uint64_t n_reads, uint32_t max_len) {
  return n_reads * sm::make_geom(max_len).chunks * 16;
}

int map_batch_impl(const smash_index *ix, int mode, uint32_t min_len, const uint8_t *d_seqs,
                   uint64_t stride, const uint16_t *d_lens, uint32_t len, uint64_t n_reads,
                   uint64_t *d_out, uint32_t cap_per_read, uint32_t *d_n_out, void *stream,
                   bool sync_check, const SearchWs *ws) {
  if (!ix || !d_seqs || !d_out || !d_n_out || cap_per_read == 0) {
    set_error("smash_map_batch: bad arguments");
    return SMASH_ERR_ARG;
  }
  if (mode == SMASH_MODE_MEM) {
    set_error("smash_map_batch: MEM lengths can exceed the packed 8-bit field; use smash_match_batch");
    return SMASH_ERR_UNSUPPORTED;
  }
  if (mode != SMASH_MODE_MAM && mode != SMASH_MODE_MAM_PLAIN && mode != SMASH_MODE_MUM) {
    set_error("smash_map_batch: unknown mode");
    return SMASH_ERR_ARG;
  }
  if (mode != SMASH_MODE_MAM_PLAIN && (!ix->d_uniq || !ix->d_kmer)) {
    set_error("smash_map_batch: index lacks the search accelerators");
    return SMASH_ERR_ARG;
  }
  if (!d_lens && len > 255) {
    set_error("smash_map_batch: reads longer than 255 need the exact LCP path");
    return SMASH_ERR_UNSUPPORTED;
  }
  if (!d_lens && (len == 0 || len > 255)) {
    set_error("smash_map_batch: read length must be 1..255");
    return SMASH_ERR_ARG;
  }
  if (min_len < 2) {   // "NOTE: min_len must be > 1" (longSA.h:194)
    set_error("smash_map_batch: min_len must be > 1");
    return SMASH_ERR_ARG;
  }
  if (n_reads == 0) return SMASH_OK;
  SMASH_HIP(hipSetDevice(ix->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const bool plain = mode == SMASH_MODE_MAM_PLAIN;
  const bool sm_path = !plain && mode != SMASH_MODE_MUM && !use_direct();
  if (ws && ws->gate && !sm_path) SMASH_HIP(hipStreamWaitEvent(s, ws->gate, 0));   // (launch_sm: after k_prep)
  if (mode == SMASH_MODE_MUM)
    return map_batch_mum(ix, min_len, d_seqs, stride, d_lens, len, n_reads, d_out, cap_per_read,
                         d_n_out, s);
  if (sm_path) {
    if (ix->idx_bytes == 4)
      return launch_sm<uint32_t>(ix, min_len, d_seqs, stride, d_lens, len, n_reads, d_out,
                                 cap_per_read, d_n_out, s, sync_check, ws);
    return launch_sm<uint64_t>(ix, min_len, d_seqs, stride, d_lens, len, n_reads, d_out,
                               cap_per_read, d_n_out, s, sync_check, ws);
  }
  if (ix->idx_bytes == 4)
    return plain ? launch<uint32_t, true>(ix, min_len, d_seqs, stride, d_lens, len, n_reads,
                                          d_out, cap_per_read, d_n_out, s)
                 : launch<uint32_t, false>(ix, min_len, d_seqs, stride, d_lens, len, n_reads,
                                           d_out, cap_per_read, d_n_out, s);
  return plain ? launch<uint64_t, true>(ix, min_len, d_seqs, stride, d_lens, len, n_reads,
                                        d_out, cap_per_read, d_n_out, s)
               : launch<uint64_t, false>(ix, min_len, d_seqs, stride, d_lens, len, n_reads,
                                         d_out, cap_per_read, d_n_out, s);
}

}  // namespace smash

using namespace smash;

// Synchronous w.r.t. the probe check: a probe outside the index fails this
// call (the pipeline uses the asynchronous form and checks at stats time).
extern "C" uint32_t smash_read_stride(uint32_t read_len) {
  return read_len && read_len <= 255 ? 4 * sm::make_geom(read_len).w_row : 0;
}

extern "C" int smash_map_batch(const smash_index *ix, int mode, uint32_t min_len,
                               const uint8_t *d_seqs, uint64_t stride,
                               const uint16_t *d_lens, uint32_t len,
                               uint64_t n_reads, uint64_t *d_out,
                               uint32_t cap_per_read, uint32_t *d_n_out,
                               void *stream) {
  return map_batch_impl(ix, mode, min_len, d_seqs, stride, d_lens, len, n_reads, d_out,
                        cap_per_read, d_n_out, stream, true);
}
