// tools/sm_emu/sm_emu.cpp -- runs the device MAM state machine
// (smash-paper_amd/csrc/mam_sm.hpp: k_prep + k_mam_sm) on the host as a single
// lane, over host copies of the index arrays.  Test tooling only: it lets the
// CPU suite check the device kernel's control flow against the goldens and the
// oracle (tests/test_sm_emu.py), and it is the debugger for that kernel
// (rocgdb is not available on the GPU pool).  Not linked into the product.
#include "hip/hip_runtime.h"

// every probe must fall inside the array it targets (the device build checks
// only the span of all arrays)
// Access accounting for the roofline (bench.py): per array (T SA ISA L8 U KT
// BM records) the 16-byte probes and the distinct 64-byte line transitions
// (a probe whose line differs from that array's previous probe line), i.e.
// the algorithmic bytes of the kernel's own access sequence.
static const uint64_t *emu_spans;
static uint64_t emu_rec_lo, emu_rec_hi, emu_bad;
static uint64_t emu_probes[8], emu_lines[8], emu_last[8];
static unsigned long long emu_ws[64];   // the kernel's STATS counters of the last run
// every request the device issues: each 16-byte load (one per 64-byte line it
// touches), speculative ones included ([1] counts those), the row DMA one per
// line of its chunks
static uint64_t emu_req[2];
// requests by the issuing lane state and op (8 * st + op, set at each
// iteration's first load): [0] all, [1] to a line among the lane's last 8
// requested lines (a re-probe), [2] speculative, [3] the second line of a
// block that crosses a 64-byte line
static uint32_t emu_st;
static uint64_t emu_rq[128][4];
static uint64_t emu_ring[8];
static uint32_t emu_ring_i;
static void emu_reqs(uint64_t a, uint64_t n, bool spec) {
  const uint64_t k = ((a + n - 1) >> 6) - (a >> 6) + 1;
  emu_req[0] += k;
  if (spec) emu_req[1] += k;
  for (uint64_t line = a >> 6; line <= (a + n - 1) >> 6; ++line) {
    uint64_t *r = emu_rq[emu_st & 127];
    ++r[0];
    bool rep = false;
    for (uint32_t q = 0; q < 8; ++q) rep = rep || emu_ring[q] == line;
    r[1] += rep;
    r[2] += spec;
    r[3] += line != (a >> 6);
    emu_ring[emu_ring_i++ & 7] = line;
  }
}
// the 16 bytes at address a, exactly (the kernel aligns the blocks it wants
// aligned); a block crossing a 64-byte line is two requests and touches two
// lines
static int emu_array(uint64_t a) {
  int arr = -1;
  if (a >= emu_rec_lo && a < emu_rec_hi) arr = 7;
  for (int k = 0; k < 7 && arr < 0; ++k)
    if (a >= emu_spans[2 * k] && a < emu_spans[2 * k + 1]) arr = k;
  return arr;
}
static void emu_count(int arr, uint64_t a, uint64_t n) {
  for (uint64_t line = a >> 6; line <= (a + n - 1) >> 6; ++line) {
    ++emu_probes[arr];
    if (line != emu_last[arr]) { ++emu_lines[arr]; emu_last[arr] = line; }
  }
}
static uint4 emu_load16(uint64_t a, bool count = true) {
  const int arr = emu_array(a);
  if (arr != 7) emu_reqs(a, 16, !count);   // (record chunks: counted by the DMA / below)
  if (arr < 0) { ++emu_bad; return uint4{0, 0, 0, 0}; }
  if (count) emu_count(arr, a, 16);
  // the block may run past the array: copy the valid bytes
  const uint64_t hi = arr == 7 ? emu_rec_hi : emu_spans[2 * arr + 1];
  if (a + 16 <= hi) {
    uint4 r;
    std::memcpy(&r, reinterpret_cast<const void *>(a), 16);
    return r;
  }
  uint8_t buf[16] = {0};
  for (uint64_t k = 0; k < 16; ++k)
    if (a + k < hi) buf[k] = *reinterpret_cast<const uint8_t *>(a + k);
  uint4 r;
  std::memcpy(&r, buf, 16);
  return r;
}
#define SM_LOAD16(a) emu_load16(a)
// the window filter's k-mer-table probes (lane state S_BM) are filed under
// array 6 ("bitmap": the filter), the (C) descents' under 5 ("kmer")
static uint4 emu_load16st(uint64_t a, bool filter) {
  if (!filter || emu_array(a) != 5) return emu_load16(a);
  emu_reqs(a, 16, false);
  emu_count(6, a, 16);
  uint4 r;
  std::memcpy(&r, reinterpret_cast<const void *>(a), 16);
  return r;
}
#define SM_LOAD16ST(a, st) (emu_st = 8u * (st) + ((st) == 6u || (st) == 8u ? op : 0u), emu_load16st(a, (st) == 4u /* S_BM */))
// speculative SA prefetches: checked, not counted; the element the search
// goes on with is counted (one 8- or 4-byte probe) by SM_HOOK_PF
#define SM_LOADPF16(a) emu_load16(a, false)
template <class IdxT>
static uint64_t emu_loadidx(const IdxT *p, uint64_t i) {
  if (emu_array(reinterpret_cast<uint64_t>(p + i)) < 0) { ++emu_bad; return 0; }
  emu_reqs(reinterpret_cast<uint64_t>(p + i), sizeof(IdxT), true);
  return uint64_t(p[i]);
}
#define SM_LOADIDX(p, i) emu_loadidx(p, i)
static void emu_hook_pf(uint64_t a, uint64_t n) {
  const int arr = emu_array(a);
  if (arr < 0) ++emu_bad; else emu_count(arr, a, n);
}
#define SM_HOOK_PF(a) emu_hook_pf(a, sizeof(IdxT))
// the row DMA: every chunk a counted record probe; the lane's own load of
// the record's first chunks (next iteration) lies on the line the DMA's
// first chunk opened: the record's 192 bytes are 3 line transitions
static void emu_dma_row(uint32_t *dst, const uint4 *src, uint32_t n, const uint4 *rec0) {
  // one instruction: its lanes' chunks coalesce per line; the lane's own
  // bad-mask load next iteration is one more request per line it touches
  emu_req[0] += ((reinterpret_cast<uint64_t>(src + n) - 1) >> 6) - (reinterpret_cast<uint64_t>(src) >> 6) + 1;
  if (rec0 != src)   // (records: the lane's own load of the bad-mask chunks)
    emu_req[0] += ((reinterpret_cast<uint64_t>(src) - 1) >> 6) - (reinterpret_cast<uint64_t>(rec0) >> 6) + 1;
  for (uint32_t k = 0; k < n; ++k) {
    const uint4 v = emu_load16(reinterpret_cast<uint64_t>(src + k));
    std::memcpy(dst + 4 * k, &v, 16);
  }
  if (rec0 != src) emu_last[7] = reinterpret_cast<uint64_t>(rec0) >> 6;   // chunks 0, 1: the line chunk 2 opened
}
// (direct rows: the row is the read itself, no bad-mask chunks before it)
#define SM_DMA_ROW(dst, src, n, lane) emu_dma_row(dst, src, n, c.direct ? (src) : (src) - c.c_bad)
// direct rows: the bad mask from the lane's own row (the device computes it
// with the whole wave)
#define SM_HOST_LANE
#define SM_DMA_ROW_HOST
// the policy knobs stay runtime here (the device compiles their defaults)
#define SM_KNOB(field, dflt) (c.field)
#define PAD_KEEP(x) ((void)(x))
// v_perm_b32 on the host: byte i of the result from selector byte i (0-7 a
// byte of {s0:s1}, 8-11 the sign of byte 1/3/5/7 spread, 12 zero, 13+ 0xFF)
static uint32_t emu_perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  const uint64_t v = (uint64_t(s0) << 32) | s1;
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) {
    const uint32_t b = (sel >> (8 * i)) & 0xFF;
    uint32_t o = 0;
    if (b < 8) o = uint32_t(v >> (8 * b)) & 0xFF;
    else if (b < 12) o = ((v >> (16 * (b - 8) + 15)) & 1) ? 0xFF : 0;
    else if (b > 12) o = 0xFF;
    r |= o << (8 * i);
  }
  return r;
}
#define SM_PERM(s0, s1, sel) emu_perm(s0, s1, sel)
// v_pk_sub_u16 on the host: both 16-bit halves, no borrow between them
static uint32_t emu_pk_sub16(uint32_t a, uint32_t b) {
  return ((a - b) & 0xFFFFu) | (((a >> 16) - (b >> 16)) << 16);
}
#define SM_PK_SUB16(a, b) emu_pk_sub16(a, b)
// v_alignbyte_b32 on the host
static uint32_t emu_alignbyte(uint32_t hi, uint32_t lo, uint32_t s) {
  return uint32_t(((uint64_t(hi) << 32) | lo) >> (8 * (s & 3)));
}
#define SM_ALIGNBYTE(hi, lo, s) emu_alignbyte(hi, lo, s)
#define SM_CTZ64(x) ((x) ? __builtin_ctzll(x) : 64)
// traverse binary searches by interval size (1..63, 64 = larger) and start depth
static uint64_t emu_bs_size[65], emu_bs_depth[256], emu_bm[16], emu_f[16 * 8];
#define SM_HOOK_BM(mode, a1, a2) (++emu_bm[4 * (mode) + 2 * (a1) + (a2)])
// policy 3: probes by (offset j of the entry's first B-mer, 3 presence bits)
#define SM_HOOK_F(j, bits) (++emu_f[8 * ((j) < 16 ? (j) : 15) + (bits)])
#define SM_HOOK_BS(size, depth) \
  do { ++emu_bs_size[(size) < 64 ? (size) : 64]; ++emu_bs_depth[(depth) < 255 ? (depth) : 255]; } while (0)
// opportunity statistics (tools/emu_profile.py --opp): [off0][stop] of every
// binary-search compare, weighted by the text lines it cost; L8 runs by
// (kind, left extension, right extension), weighted by all lines they cost
static uint64_t emu_cmp_n[64 * 64], emu_cmp_lines[64 * 64], emu_cmp_off0, emu_cmp_l0;
static uint64_t emu_run_n[2 * 10 * 10], emu_run_lines[2 * 10 * 10], emu_run_l0[2];
static uint64_t emu_byte_n, emu_byte_other;
static const uint8_t *emu_T;
static uint64_t emu_lines_all() {
  uint64_t t = 0;
  for (int k = 0; k < 8; ++k) t += emu_lines[k];
  return t;
}
static void emu_hook_cmpbs(bool begin, uint64_t sp, uint64_t off) {
  (void)sp;
  if (begin) { emu_cmp_off0 = off; emu_cmp_l0 = emu_lines[0]; return; }
  const uint64_t a = emu_cmp_off0 < 63 ? emu_cmp_off0 : 63, b = off < 63 ? off : 63;
  emu_cmp_n[64 * a + b] += 1;
  emu_cmp_lines[64 * a + b] += emu_lines[0] - emu_cmp_l0;
}
static void emu_hook_run(bool begin, int kind, uint64_t el, uint64_t er) {
  if (begin) { emu_run_l0[kind] = emu_lines_all(); return; }
  const uint64_t a = el < 9 ? el : 9, b = er < 9 ? er : 9;
  emu_run_n[100 * kind + 10 * a + b] += 1;
  emu_run_lines[100 * kind + 10 * a + b] += emu_lines_all() - emu_run_l0[kind];
}
static void emu_hook_byte(uint64_t pos) {
  ++emu_byte_n;
  const uint8_t ch = emu_T[pos - 1];
  if (ch != 'a' && ch != 'c' && ch != 'g' && ch != 't') ++emu_byte_other;
}
#define SM_HOOK_CMPBS(begin, sp, off) emu_hook_cmpbs(begin, sp, off)
#define SM_HOOK_RUN(begin, kind, el, er) emu_hook_run(begin, kind, el, er)
#define SM_HOOK_BYTE(pos) emu_hook_byte(pos)
static uint64_t emu_park[16];
#define SM_HOOK_PARK(a) (++emu_park[(a) & 15])
#include "../../smash-paper_amd/csrc/mam_sm.hpp"

thread_local dim3 threadIdx, blockIdx, blockDim;
namespace smash { namespace sm { alignas(16) uint32_t ldsw[1 << 12]; alignas(16) uint32_t prep_lds[1 << 16]; } }

using namespace smash;

// the records of n reads, by k_prep (one lane per block, LDS image) or by
// k_prep_direct (every (read, group) item, 256-thread blocks), as the device
// default (mam.hip) does
static int prep_records(const uint8_t *reads, uint64_t stride, const uint16_t *lens, uint32_t L,
                        uint64_t n, const uint64_t *in_text, const sm::Geom &g, uint32_t *rec,
                        bool direct) {
  if (direct) {
    blockDim.x = 256;
    const uint32_t ga = sm::prep_groups(lens ? 255 : L);
    const uint64_t items = n * ga;
    for (uint64_t i = 0; i < items; ++i) {
      blockIdx.x = unsigned(i / 256);
      threadIdx.x = unsigned(i % 256);
      sm::k_prep_direct(reads, stride, lens, L, uint32_t(n), ga, in_text[0], in_text[1], in_text[2],
                        in_text[3], g, rec, 0u);
    }
  } else {
    const uint32_t per = sm::prep_per_block(g, stride);
    if (sm::prep_lds_bytes(g, stride, per) > sizeof(sm::prep_lds)) return -1;
    blockDim.x = 1;
    threadIdx.x = 0;
    for (uint64_t b = 0; b * per < n; ++b) {
      blockIdx.x = unsigned(b);
      sm::k_prep(reads, stride, lens, L, n, in_text[0], in_text[1], in_text[2], in_text[3], g, per,
                 rec);
    }
  }
  blockIdx.x = 0;
  threadIdx.x = 0;
  blockDim.x = 1;
  return 0;
}

// both record builders over the same reads (tests: k_prep_direct == k_prep,
// word for word); returns the record words per read, -1 on a geometry error
extern "C" int sm_emu_prep(const uint8_t *reads, uint64_t stride, const uint16_t *lens, uint32_t L,
                           uint64_t n, const uint64_t *in_text, uint32_t *out_lds,
                           uint32_t *out_direct) {
  const sm::Geom g = sm::make_geom(lens ? 255 : L);
  const uint64_t words = n * g.chunks * 4;
  for (uint64_t i = 0; i < words; ++i) out_lds[i] = out_direct[i] = 0xDEADBEEFu;   // all written?
  if (prep_records(reads, stride, lens, L, n, in_text, g, out_lds, false)) return -1;
  if (prep_records(reads, stride, lens, L, n, in_text, g, out_direct, true)) return -1;
  return int(g.chunks * 4);
}

template <class IdxT>
static int run(const uint8_t *T, const void *SA, const void *ISA, const uint8_t *L8,
               const uint8_t *U, const uint64_t *KT, int K, const uint64_t *BM, int B,
               const uint64_t *in_text, uint64_t N, uint64_t logN, const uint8_t *reads,
               uint64_t stride, uint32_t L, uint64_t n, uint32_t min_len, uint64_t *out,
               uint32_t cap, uint32_t *n_out, uint32_t *iters, const uint64_t *spans,
               uint64_t *viol, uint32_t lin_blocks, uint64_t *counters, int packed) {
  const sm::Geom g = sm::make_geom(L);
  if (g.w_row > sizeof(sm::ldsw) / 4) return -1;
  // direct rows (the device's path for native-row input, the default here as
  // in bench.py; SMASH_SM_DIRECT=0: records built by k_prep)
  const bool direct = !(std::getenv("SMASH_SM_DIRECT") && std::getenv("SMASH_SM_DIRECT")[0] == '0');
  const uint64_t rw = 4ull * g.w_row;   // native row bytes
  std::vector<uint4> rows_mem(direct ? n * rw / 16 + 4 : 0);
  uint8_t *rows_p = direct ? reinterpret_cast<uint8_t *>(rows_mem.data()) : nullptr;
  while (direct && (reinterpret_cast<uint64_t>(rows_p) & 63)) rows_p += 16;
  for (uint64_t q = 0; direct && q < n; ++q) {
    std::memset(rows_p + q * rw, 0, rw);
    std::memcpy(rows_p + q * rw, reads + q * stride, L);
  }
  // 64-byte aligned, as the device's allocation (records are whole lines)
  std::vector<uint4> rec_mem(n * g.chunks + 4);
  uint4 *rec_p = rec_mem.data();
  while (reinterpret_cast<uint64_t>(rec_p) & 63) ++rec_p;
  struct { uint4 *p; size_t n; uint4 *data() { return p; } size_t size() const { return n; } } rec{
      rec_p, size_t(n * g.chunks)};
  if (!direct &&
      prep_records(reads, stride, nullptr, L, n, in_text, g, reinterpret_cast<uint32_t *>(rec.data()),
                   !(std::getenv("SMASH_PREP_LDS") && std::getenv("SMASH_PREP_LDS")[0] == '1')))
    return -1;
  threadIdx.x = 0;
  sm::Ctx<IdxT> c;
  emu_T = T;
  c.T = T; c.SA = static_cast<const IdxT *>(SA); c.ISA = static_cast<const IdxT *>(ISA);
  c.L8 = L8; c.U = U; c.KT = KT;
  (void)BM;   // (round 3: the filter's presence bits live in KT)
  c.N = N; c.logN = uint32_t(logN); c.K = uint32_t(K); c.B = uint32_t(B); c.min_len = min_len;
  c.rec = rec.data(); c.chunks = g.chunks; c.c_bad = g.c_bad; c.w_row = g.w_row; c.w_raw = g.w_raw;
  c.rows = direct ? reinterpret_cast<const uint4 *>(rows_p) : nullptr;
  c.direct = direct ? 1u : 0u;
  sm::bad_table(in_text, &c.bad_tab_lo, &c.bad_tab_hi);
  c.lin_blocks = lin_blocks;
  c.pad = 0;
  c.mhint = 0;
  c.grab = 1;
  c.bm_dual = std::getenv("SMASH_SM_BM_DUAL") ? uint32_t(std::atoi(std::getenv("SMASH_SM_BM_DUAL"))) : 3;   // = the device default (mam.hip)
  c.pf = std::getenv("SMASH_SM_PF") ? uint32_t(std::atoi(std::getenv("SMASH_SM_PF"))) : 1;
  c.u32 = std::getenv("SMASH_SM_U32") ? uint32_t(std::atoi(std::getenv("SMASH_SM_U32"))) : 1;
  c.f2 = std::getenv("SMASH_SM_F2") ? uint32_t(std::atoi(std::getenv("SMASH_SM_F2"))) : 2;
  c.lens = nullptr; c.len0 = L; c.cap = cap; c.n_reads = n;
  c.out = out; c.n_out = n_out;
  unsigned long long work = 0;
  c.work = &work;
  for (int k = 0; k < 4; ++k) c.in_text[k] = in_text[k];
  unsigned long long ws[128] = {0};
  c.iters = iters; c.wave_stats = ws;
  // the emulator checks every probe against its own array (the device checks
  // the span of all of them)
  (void)spans;
  c.lo = 0; c.hi = ~0ull;
  unsigned long long v[10] = {0};
  c.viol = v;
  emu_spans = spans;
  emu_rec_lo = direct ? reinterpret_cast<uint64_t>(rows_p) : reinterpret_cast<uint64_t>(rec.data());
  emu_rec_hi = emu_rec_lo + (direct ? n * rw : rec.size() * sizeof(uint4));
  emu_bad = 0;
  for (int k = 0; k < 8; ++k) { emu_probes[k] = emu_lines[k] = 0; emu_last[k] = ~0ull; }
  emu_req[0] = emu_req[1] = 0;
  std::memset(emu_rq, 0, sizeof(emu_rq));
  std::memset(emu_ring, 0xFF, sizeof(emu_ring));
  // packed index words (common.hpp): the SA / ISA arrays given carry them
  if (packed && sizeof(IdxT) == 8) sm::k_mam_sm<IdxT, 1, true, true, sizeof(IdxT) == 8>(c);
  else sm::k_mam_sm<IdxT, 1, true, true, false>(c);
  for (int k = 0; k < 10; ++k) viol[k] = v[k];
  viol[0] += emu_bad;
  for (int k = 0; k < 8; ++k) { counters[k] = emu_probes[k]; counters[8 + k] = emu_lines[k]; }
  for (int k = 0; k < 64; ++k) emu_ws[k] = ws[k];
  return 0;
}

// lane iterations of the last sm_emu_map by state (k_mam_sm STATS layout:
// [2 + state], IDX ops at [18 + op], CMP ops at [42 + op])
extern "C" void sm_emu_ws(uint64_t *out) {
  for (int k = 0; k < 64; ++k) out[k] = emu_ws[k];
}

// device requests of the last sm_emu_map: [0] all, [1] speculative
extern "C" void sm_emu_requests(uint64_t *out) { out[0] = emu_req[0]; out[1] = emu_req[1]; }
extern "C" void sm_emu_req_by_state(uint64_t *out) { std::memcpy(out, emu_rq, sizeof(emu_rq)); }

// (F) policy-3 probe outcomes since the last reset: [8 * j + bits]
extern "C" void sm_emu_filter_hist(uint64_t *out, int reset) {
  for (int k = 0; k < 128; ++k) { out[k] = emu_f[k]; if (reset) emu_f[k] = 0; }
}

// binary-search start histograms since the last reset (size[65], depth[256])
extern "C" void sm_emu_bs_hist(uint64_t *size, uint64_t *depth, int reset) {
  for (int k = 0; k < 65; ++k) { size[k] = emu_bs_size[k]; if (reset) emu_bs_size[k] = 0; }
  for (int k = 0; k < 256; ++k) { depth[k] = emu_bs_depth[k]; if (reset) emu_bs_depth[k] = 0; }
  for (int k = 0; k < 12; ++k) { depth[244 + k] = emu_bm[k]; if (reset) emu_bm[k] = 0; }
}

// the opportunity statistics since the last reset: cmp_n[4096], cmp_lines[4096],
// run_n[200], run_lines[200], byte[2]
extern "C" void sm_emu_opp(uint64_t *cmp_n, uint64_t *cmp_lines, uint64_t *run_n,
                           uint64_t *run_lines, uint64_t *byte, int reset) {
  for (int k = 0; k < 4096; ++k) {
    cmp_n[k] = emu_cmp_n[k]; cmp_lines[k] = emu_cmp_lines[k];
    if (reset) emu_cmp_n[k] = emu_cmp_lines[k] = 0;
  }
  for (int k = 0; k < 200; ++k) {
    run_n[k] = emu_run_n[k]; run_lines[k] = emu_run_lines[k];
    if (reset) emu_run_n[k] = emu_run_lines[k] = 0;
  }
  byte[0] = emu_byte_n; byte[1] = emu_byte_other;
  if (reset) emu_byte_n = emu_byte_other = 0;
}

extern "C" int sm_emu_map(const uint8_t *T, const void *SA, const void *ISA, int idx_bytes,
                          const uint8_t *L8, const uint8_t *U, const uint64_t *KT, int K,
                          const uint64_t *BM, int B, const uint64_t *in_text, uint64_t N,
                          uint64_t logN, const uint8_t *reads, uint64_t stride, uint32_t L,
                          uint64_t n, uint32_t min_len, uint64_t *out, uint32_t cap,
                          uint32_t *n_out, uint32_t *iters, const uint64_t *spans,
                          uint64_t *viol, uint32_t lin_blocks, uint64_t *counters, int packed) {
  if (idx_bytes == 4)
    return run<uint32_t>(T, SA, ISA, L8, U, KT, K, BM, B, in_text, N, logN, reads, stride, L, n,
                         min_len, out, cap, n_out, iters, spans, viol, lin_blocks, counters, 0);
  return run<uint64_t>(T, SA, ISA, L8, U, KT, K, BM, B, in_text, N, logN, reads, stride, L, n,
                       min_len, out, cap, n_out, iters, spans, viol, lin_blocks, counters, packed);
}

// decide chains parked in S_ALU since the last reset, by pending action
extern "C" void sm_emu_park_hist(uint64_t *out, int reset) {
  for (int k = 0; k < 16; ++k) { out[k] = emu_park[k]; if (reset) emu_park[k] = 0; }
}
