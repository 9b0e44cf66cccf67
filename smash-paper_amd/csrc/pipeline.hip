// smash-paper_amd/csrc/pipeline.hip -- the read -> bin-count chain per batch.
//
//   k_mam        longSA::MAM per mate                        (mam_device.hpp)
//   k_post       per pair: Aligner::prepare_matches           query.cpp:231-306
//                + mappability_tag L/R                         mappability_tag.cpp:93-124
//                + smashMEM filters, key                       smashMEM.py:84-92,154-217
//   dedup        global first-wins pair key set               smashMEM.py:149,217-228
//   k_emit       awk/perl extraction of major-chromosome hits smash_mapping.sh:29
//   k_bin        varbin adjacent de-dup + bisect + count      varbin.py:52-92
//
// All per-pair state lives in HBM; the host only launches.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "common.hpp"
#include "mam_device.hpp"

namespace {
constexpr int kB = 256;
// k_post (the general per-pair body) keeps a mate's alignments and both
// mates' hit lists in a per-thread slice of a global workspace sized for the
// largest possible mate (slots = L - min_len + 1 matches), so no input is
// ever cut; it runs as a bounded grid-stride launch of kPostThreads threads.
constexpr unsigned kPostBlocks = 64;
constexpr unsigned kPostThreads = kPostBlocks * kB;
enum Stat { S_PAIRS, S_KEYPAIRS, S_DUPEPAIRS, S_POS, S_DUPS, S_KEPT, S_MATCHES, S_ERR, S_N };
// d_stats: kStatStripes rows of kStatStride words.  The post-stage kernels
// add their counters wave by wave into row (wave id % kStatStripes), so no
// single word takes every wave's atomic, and need no LDS for a block
// reduction (a kernel with LDS cannot share a CU with the search, whose
// blocks hold all of it); the host sums the rows.  S_ERR lives in row 0.
constexpr uint32_t kStatStride = 16, kStatStripes = 16, kStatWords = kStatStride * kStatStripes;
// the multi-GPU export's header per key (smash_phase_export): {hash hi, hash
// lo, nk << 40 | word offset in the owner's segment} = SMASH_EXPORT_HDR_WORDS
// (round 3 also sent the global pair index and kept nk and the offset in
// words of their own: 40 B per key, now 24)
constexpr uint32_t kHdrWords = 1;   // nk << 40 | word offset (round 5: the hashes are recomputed)
constexpr uint64_t kHdrOffMask = (uint64_t(1) << 40) - 1;
static_assert(kHdrWords == SMASH_EXPORT_HDR_WORDS, "smash_gpu.h's export header");
}  // namespace

// The post-stage kernels run beside the next batch's k_mam_sm (no LDS, so
// they fit next to its blocks), whose waves are older and always ready: at
// equal priority the SIMD's oldest-first issue leaves them a trickle and
// they finish only when the search drains.  Raised priority lets them
// through; the search absorbs their (small) share of the memory system.
// (Round 3 A/B, profiles/r03/sched: default priority 150.7 vs 150.2-151.9 ms
// per C3 step; the knob was a process-global symbol and is gone.)
#define SMASH_BESIDE_SEARCH() __builtin_amdgcn_s_setprio(2)

struct smash_pipeline {
  const smash_index *ix = nullptr;
  int device = 0;
  uint32_t read_len = 0, min_len = 20, slots = 0, n_contig = 0, nbins = 0;
  uint32_t stride = 0;   // bytes from one mate to the next in d_reads (cfg.read_stride)
  int32_t min_excess = 4;
  int64_t hit_window = 10000;
  uint64_t max_pairs = 0;
  uint32_t *d_tag_off = nullptr;
  uint8_t *d_small = nullptr;
  int64_t *d_chrom_off = nullptr;
  int64_t *d_bins = nullptr;
  // bin directory: cell c = [c << cshift, (c + 1) << cshift) of the absolute
  // position; d_cell[c] = bisect_right(bins, c << cshift), d_cell[ncell] =
  // nbins, so a position's bisect runs over [d_cell[c], d_cell[c + 1]) only
  uint32_t *d_cell = nullptr;
  uint32_t ncell = 0, cshift = 0;
  uint32_t *d_sp_cell = nullptr;  // contig directory (PostCfg::sp_cell)
  uint32_t sp_ncell = 0, sp_shift = 0;
  uint64_t *d_match = nullptr;    // the current search set's (below)
  uint32_t *d_nmatch = nullptr;
  // two search sets: the k_mam_sm launch of batch b + 1 runs on its own
  // stream under the tail of batch b's (the slowest reads of a launch leave
  // most CUs idle for ~1.6 ms); set k is free again once the post stage of
  // its last batch has read it (ev_free)
  uint64_t *d_match_s[2] = {nullptr, nullptr};
  uint32_t *d_nmatch_s[2] = {nullptr, nullptr};
  uint8_t *d_rec_s[2] = {nullptr, nullptr};
  unsigned long long *d_work_s[2] = {nullptr, nullptr};
  uint64_t rec_bytes = 0;
  hipStream_t xs[2] = {nullptr, nullptr};
  hipEvent_t ev_in = nullptr, ev_found[2] = {nullptr, nullptr}, ev_free[2] = {nullptr, nullptr};
  hipEvent_t ev_done = nullptr;   // recorded once at creation: "inputs already complete"
  bool set_used[2] = {false, false};
  // schedule (read at creation; A/B): SMASH_GATE_POST (default 1) ev_free
  // is recorded after the batch's whole post stage (single-GPU count path),
  // so a set's next search starts once that batch is binned: the post stage
  // of batch b shares the GPU with search b + 1 only, never with b + 2's
  // (=0: after k_post, the set's match buffers' last reader);
  // SMASH_GATE_PREP=1 the next search's k_prep also waits for ev_free;
  // SMASH_ONE_SEARCH=1 a search waits for the other set's (never two
  // k_mam_sm at once)
  bool gate_prep = false, gate_post = false, one_search = false;
  bool found_rec[2] = {false, false};
  bool defer_free = false;        // count_batch_ev under gate_post
  // a search already issued into a set (smash_phase_map_ahead): its reads
  const uint8_t *pref_reads[2] = {nullptr, nullptr};
  uint64_t pref_n[2] = {0, 0};
  bool searched[2] = {false, false};
  int set = 1;
  int32_t *d_nk = nullptr;
  uint32_t *d_nmajor = nullptr;
  uint64_t *d_hits = nullptr;     // [max_pairs][2 * slots]: full hit rows (HitRows)
  uint64_t *d_hhead = nullptr;    // [max_pairs][kHitHead]: dense head rows
  uint64_t *d_hash = nullptr;   // [2*max_pairs] hi, lo
  uint8_t *d_keep = nullptr;
  uint64_t *d_slot = nullptr;     // [max_pairs] k_dedup_claim -> k_dedup_decide
  uint8_t *d_contest = nullptr;   // [max_pairs] claims of an already-claimed key mark it
                                  // (kSlotIns; null: SMASH_CLAIM_FLAG=0, every decide reads)
  uint64_t *d_tsum = nullptr;     // [tiles] the LDS-free scans' tile aggregates / prefixes
  int64_t *d_tlast = nullptr;
  bool cnt_ready = false;         // k_dedup_decide wrote d_cnt / d_lp for this batch
  bool reads_resident = false;    // smash_pipeline_reads_resident: searches wait on no input event
  // multi-GPU export: per (owner, block) keys << 32 | words and their
  // exclusive scan (k_export_count / k_export_fill); the owner's claim slots
  uint64_t *d_bcnt = nullptr, *d_boff = nullptr;
  void *d_scan_temp = nullptr;
  size_t scan_temp_bytes = 0;
  uint64_t *d_oslot = nullptr;
  uint64_t oslot_cap = 0;
  void *d_temp = nullptr;
  size_t temp_bytes = 0;
  uint64_t *d_table = nullptr;   // {hash hi, arena ref + 1} slots, 0 = empty
  uint64_t table_mask = 0;
  uint64_t *d_arena = nullptr;   // canonical keys: [lo, nk, hit words...] per key
  uint64_t arena_cap = 0;        // words
  unsigned long long *d_arena_top = nullptr;
  // pairs de-duplicated since the last reset (single GPU): a bound on the
  // keys the set holds, on the host, for the file feed's growth (ensure_keys)
  uint64_t keys_bound = 0;
  uint64_t epoch = 0;             // launches of the set's insert kernels (ref tags)
  uint32_t *d_posoff = nullptr;   // [max_pairs + 1]
  uint32_t *d_cnt = nullptr;      // [max_pairs]
  int64_t *d_pos0 = nullptr, *d_abs = nullptr;
  int64_t *d_prev = nullptr;      // [2] carried {last pos0 or -1, -}
  // fused positions + varbin (k_emit_bin): per pair the pos0 of its last
  // emitted position (-1: none), and its inclusive "last valid" scan
  int64_t *d_lp = nullptr, *d_lps = nullptr;
  bool fused_bin = true;
  uint32_t bin_flush = 0x8000;    // k_emit_bin_lds's 16-bit counter flush threshold
  uint32_t *d_binpart = nullptr;  // [kBinBlocks][nbins]: k_emit_bin_lds's per-block counts
  uint32_t coop_copy = 7;         // wave-cooperative key-word copies, bit 0: export, 1: single-GPU
                                  // decide, 2: owner decide (SMASH_COOP_COPY=0: per lane)
  bool bin_lds = true;            // k_emit_bin_lds when the bins fit (SMASH_BIN_LDS=0: global
                                  // atomics; the LDS form runs in the gap SMASH_GATE_POST leaves)
  bool pos_dirty = false;         // the positions arrays are not materialised yet
  unsigned long long *d_stats = nullptr;
  uint32_t *d_fb = nullptr;       // [1 + max_pairs]: k_post_fast<16> -> k_post pair list
  uint32_t *d_l16 = nullptr;      // [1 + max_pairs]: k_post_fast<8> -> k_post_fast<16>
  uint8_t *d_post_ws = nullptr;   // k_post workspace: kPostThreads slices
  uint64_t hash_mask = ~0ull;
  bool post_fast = false;
  // the searches' match words carry map hints (SearchWs::mhint, PostCfg):
  // packed index words, map.bin built from this index, tag offsets equal to
  // its contig offsets (SMASH_MAP_HINT=0: off, A/B)
  bool mhint = false;
  uint32_t post_cap = 0;
  uint32_t *d_send_q = nullptr;   // exported slot -> pair
  unsigned long long *d_owner = nullptr;  // per owner: [0,64) keys [64,128) words (k_export_totals)
  uint64_t *d_send_hdr = nullptr; // [n_export][kHdrWords] {nk << 40 | word offset}
  uint64_t *d_send_words = nullptr;   // the exported keys' hit words, grouped by owner
  uint64_t send_words_cap = 0;
  uint64_t *d_recv_base = nullptr;    // [2 * 65] owner side: header / word prefix per source
  // pinned host images of d_owner (the per-owner totals) and d_recv_base
  // (its host-to-device copy stays asynchronous: the host rewrites the image
  // only after the event of its previous copy)
  unsigned long long *h_owner = nullptr;
  uint64_t *h_recv_base = nullptr;
  hipEvent_t ev_base = nullptr;
  uint64_t n_pairs = 0, n_export = 0;
  hipStream_t last = nullptr;
  // smash_count_fastq's pinned slots, device buffers and copy stream, kept
  // across calls (pinning GBs of host memory costs more than a batch)
  void *feed = nullptr;
  void (*feed_free)(void *) = nullptr;
  // profiling (smash_pipeline_profile)
  bool prof = false;
  std::vector<hipEvent_t> ev;     // pairs: [2i] before, [2i+1] after k_mam
  uint64_t n_ev = 0, prof_reads = 0;
};

namespace smash {
namespace {

struct PostCfg {
  const uint64_t *startpos, *sizes;
  uint32_t n_seq, L, slots;
  const uint32_t *tag_off;
  const uint8_t *small;
  const int64_t *chrom_off;
  const uint8_t *map;
  uint64_t map_bytes;
  int32_t min_excess;
  int64_t window;
  uint32_t fast_cap;   // k_post_fast: mates with more matches go to k_post
  uint64_t hash_mask;  // ~0; tests shorten the key hash (SMASH_KEY_HASH_BITS) so
                       // that the exact key comparison meets real collisions
  // contig directory (k_post_fast): cell c = text positions [c << sp_shift,
  // (c + 1) << sp_shift); sp_cell[c] = upper_bound(startpos, c << sp_shift),
  // sp_cell[sp_ncell] = n_seq, so a position's contig bisect runs over
  // [sp_cell[c], sp_cell[c + 1]] only
  const uint32_t *sp_cell;
  uint32_t sp_shift, sp_ncell;
  // the search's map hints (SearchWs::mhint): a forward match word carries
  // its right map.bin byte before the edge rule in bits 40..47 (0: none)
  bool mhint;
};

// the reference position of a match word: 48 bits (smash_gpu.h), 40 when
// the word may carry a map hint (N < 2^33 then)
constexpr uint64_t kRefMask = 0xFFFFFFFFFFull;

// A pair's kept hit words (its key, smashMEM.py:122-131): in a dense head row
// of kHitHead words when it has at most that many (C3: all but a few; 6.7 on
// average), else in its full row of 2 * slots words.  Every reader knows nk,
// so it picks the row without a flag.  Dense rows put 64 consecutive pairs in
// 8 KB: the post stage, the de-dup and the binning read them as streams
// instead of one random line 2 * slots words apart per pair.
constexpr uint32_t kHitHead = 16;
struct HitRows {
  uint64_t *head, *full;
  uint32_t slots;
  __device__ __forceinline__ uint64_t *row(uint64_t q, int32_t nk) const {
    return nk <= int32_t(kHitHead) ? head + q * kHitHead : full + q * 2 * uint64_t(slots);
  }
};

struct Aln {
  int64_t pos, qpos;
  uint32_t seq;
  uint16_t prefix, len, suffix;
  uint8_t rc, pad;
};

struct Hit {
  int64_t pos;
  uint32_t tid, qstart, qend;
  int32_t L0, R0;
  int64_t qkey;   // qpos for to_print
  uint8_t rc;
};

__device__ inline bool merge_less(const Aln &a, const Aln &b) {   // to_merge
  if (a.rc != b.rc) return a.rc < b.rc;
  if (a.seq != b.seq) return a.seq < b.seq;
  if (a.pos != b.pos) return a.pos < b.pos;
  return a.prefix < b.prefix;
}

__device__ inline unsigned mapb(const PostCfg &c, uint64_t at) {
  return at < c.map_bytes ? c.map[at] : 0u;
}

// resolve + merge + to_print order + tags for one mate; returns #hits
__device__ int mate_hits(const PostCfg &c, const uint64_t *m, uint32_t n,
                         Hit *hits, Aln *a, int32_t &err) {
  int na = 0;
  const uint32_t L = c.L;
  for (uint32_t k = 0; k < n; ++k) {
    const uint64_t w = m[k];
    const uint64_t ref = w & (c.mhint ? kRefMask : 0xFFFFFFFFFFFFull);
    const uint32_t q = uint32_t((w >> 48) & 0xFF), len = uint32_t(w >> 56);
    uint32_t lo = 0, hi = c.n_seq;          // upper_bound(startpos, ref)
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (c.startpos[mid] <= ref) lo = mid + 1; else hi = mid;
    }
    const uint32_t si = lo - 1;
    const uint64_t rcpos = ref - q;
    int64_t pos = int64_t(rcpos - c.startpos[si]);
    const uint32_t extra = L - len - q;
    Aln x;
    x.qpos = q;
    x.len = uint16_t(len);
    if (si & 1) {
      x.seq = si - 1;
      pos = int64_t(c.sizes[si - 1] - uint64_t(pos)) - int64_t(L);
      x.prefix = uint16_t(extra);
      x.suffix = uint16_t(q);
      x.rc = 1;
    } else {
      x.seq = si;
      x.prefix = uint16_t(q);
      x.suffix = uint16_t(extra);
      x.rc = 0;
    }
    x.pos = pos;
    if (pos >= 0) a[na++] = x;            // erase pos < 0 (query.cpp:239-246)
  }
  // insertion sort by to_merge (distinct keys: no ties)
  for (int i = 1; i < na; ++i) {
    Aln t = a[i];
    int j = i - 1;
    while (j >= 0 && merge_less(t, a[j])) { a[j + 1] = a[j]; --j; }
    a[j + 1] = t;
  }
  int nh = 0;
  int g0 = 0;
  for (int i = 0; i < na; ++i) {
    const bool endg = (i + 1 == na) || a[i + 1].pos != a[i].pos ||
                      a[i + 1].seq != a[i].seq || a[i + 1].rc != a[i].rc;
    if (!endg) continue;
    Hit h;
    h.tid = a[i].seq >> 1;
    h.rc = a[i].rc;
    h.pos = a[i].pos;
    h.qstart = a[g0].prefix;                 // leading S (query.cpp:260-263)
    h.qend = L - a[i].suffix;                // trailing S (:267-268)
    int64_t qmin = a[g0].qpos;
    for (int k = g0 + 1; k <= i; ++k) qmin = a[k].qpos < qmin ? a[k].qpos : qmin;
    h.qkey = qmin;
    // mappability_tag on every '=' block; block k starts at offset prefix_k
    const uint32_t abspos = c.tag_off[h.tid] + uint32_t(h.pos + 1);
    const bool small = c.small[h.tid] != 0;
    for (int k = g0; k <= i; ++k) {
      const uint32_t cnt = a[k].len;
      const uint32_t li = abspos + uint32_t(a[k].prefix) + cnt - 1;
      const uint32_t ri = abspos + uint32_t(a[k].prefix) - 1;
      const unsigned lm = mapb(c, 2 + uint64_t(li) * 2);
      const unsigned left = lm ? lm - 1 : 255;
      const unsigned rm = mapb(c, 2 + uint64_t(ri) * 2 + 1);
      const unsigned right = rm ? rm : 255;
      if (k == g0) { h.L0 = int32_t(left); h.R0 = int32_t(right); }
      if (!small && err == 0) {
        if (left > cnt) err = SMASH_ERR_TAG_LEFT;
        else if (right > cnt) err = SMASH_ERR_TAG_RIGHT;
      }
    }
    // to_print order: insert by (qpos, rc)
    int j = nh - 1;
    while (j >= 0 && (h.qkey < hits[j].qkey || (h.qkey == hits[j].qkey && h.rc < hits[j].rc))) {
      hits[j + 1] = hits[j];
      --j;
    }
    hits[j + 1] = h;
    ++nh;
    g0 = i + 1;
  }
  return nh;
}

__device__ inline uint64_t mix64(uint64_t z) {
  z ^= z >> 33; z *= 0xff51afd7ed558ccdull;
  z ^= z >> 33; z *= 0xc4ceb9fe1a85ec53ull;
  z ^= z >> 33;
  return z;
}

// the general per-pair body (any number of matches, per-thread arrays);
// k_post_fast hands it the pairs whose mates exceed its register capacity
// workspace slice of one k_post thread: slots Aln, then 2 * slots Hit
__host__ __device__ inline uint64_t post_ws_bytes(uint32_t slots) {
  return (uint64_t(slots) * sizeof(Aln) + 2ull * slots * sizeof(Hit) + 15) & ~uint64_t(15);
}

__device__ __noinline__ void post_pair(const PostCfg &c, const uint64_t *__restrict__ match,
                                       const uint32_t *__restrict__ nmatch, uint64_t q,
                                       int32_t *nk_out, uint32_t *nmajor_out,
                                       HitRows hits_out, uint64_t *hash_out, int32_t &err,
                                       unsigned long long &nm, uint8_t *ws) {
  {
    Aln *a = reinterpret_cast<Aln *>(ws);
    Hit *h1 = reinterpret_cast<Hit *>(ws + uint64_t(c.slots) * sizeof(Aln));
    Hit *h2 = h1 + c.slots;
    const uint32_t n1 = nmatch[2 * q], n2 = nmatch[2 * q + 1];
    nm = n1 + n2;
    const int k1 = mate_hits(c, match + (2 * q) * c.slots, n1 < c.slots ? n1 : c.slots, h1, a, err);
    const int k2 = mate_hits(c, match + (2 * q + 1) * c.slots, n2 < c.slots ? n2 : c.slots, h2, a, err);
    if (n1 > c.slots || n2 > c.slots) err = SMASH_ERR_UNSUPPORTED;
    // smashMEM excess-mappability filter (smashMEM.py:84-92)
    int m1 = 0, m2 = 0;
    for (int i = 0; i < k1; ++i) {
      const int mx = h1[i].L0 > h1[i].R0 ? h1[i].L0 : h1[i].R0;
      if (int(h1[i].qend) - int(h1[i].qstart) - mx >= c.min_excess) h1[m1++] = h1[i];
    }
    for (int i = 0; i < k2; ++i) {
      const int mx = h2[i].L0 > h2[i].R0 ? h2[i].L0 : h2[i].R0;
      if (int(h2[i].qend) - int(h2[i].qstart) - mx >= c.min_excess) h2[m2++] = h2[i];
    }
    uint64_t *ho = hits_out.full + q * (2 * uint64_t(c.slots));
    int32_t nk = -1;
    uint32_t nmaj = 0;
    uint64_t hh = 0x9E3779B97F4A7C15ull, hl = 0xD1B54A32D192ED03ull;
    if (m1 > 0 || m2 > 0) {                  // smashMEM.py:162
      nk = 0;
      auto put = [&](uint32_t tid, int64_t pos) {
        ho[nk++] = (uint64_t(tid) << 48) | (uint64_t(pos) & 0xFFFFFFFFFFFFull);
        const uint64_t w = (uint64_t(tid) << 48) ^ uint64_t(pos);
        hh = mix64(hh ^ w) + 0x632BE59BD9B4E019ull;
        hl = mix64(hl + w * 0x9E3779B97F4A7C15ull) ^ (hl >> 29);
        if (c.chrom_off[tid] >= 0) ++nmaj;
      };
      for (int i = 0; i < m1; ++i) put(h1[i].tid, h1[i].pos);
      for (int b = 0; b < m2; ++b) {         // hit window (smashMEM.py:193-200)
        bool close = false;
        for (int i = 0; i < m1; ++i) {
          int64_t d = h1[i].pos - h2[b].pos;
          d = d < 0 ? -d : d;
          if (h1[i].tid == h2[b].tid && d < c.window) { close = true; break; }
        }
        if (!close) put(h2[b].tid, h2[b].pos);
      }
      hh = (mix64(hh ^ uint64_t(nk)) & c.hash_mask) | 1;
      hl = (mix64(hl + uint64_t(nk)) & c.hash_mask) | 1;
      if (nk <= int32_t(kHitHead))           // (the readers look for it there)
        for (int32_t i = 0; i < nk; ++i) hits_out.head[q * kHitHead + i] = ho[i];
    }
    nk_out[q] = nk;
    nmajor_out[q] = nmaj;
    hash_out[2 * q] = hh;
    hash_out[2 * q + 1] = hl;
  }
}

// the wave's sum of v (every lane of the wave calls it)
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// the stats row of this wave (kStatStripes rows, see d_stats)
__device__ __forceinline__ unsigned long long *stat_row(unsigned long long *stats) {
  const uint32_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  return stats + kStatStride * (w % kStatStripes);
}

// the wave's sums of a and b added to counters ia and ib of its stats row
// (every lane of the wave calls it); err: the first data error, row 0
__device__ __forceinline__ void wave_stats(unsigned long long *stats, int ia,
                                           unsigned long long a, int ib, unsigned long long b,
                                           int32_t err) {
  a = wave_sum(a);
  b = wave_sum(b);
  unsigned long long *row = stat_row(stats);
  if ((threadIdx.x & 63) == 0) {
    if (a) atomicAdd(&row[ia], a);
    if (b) atomicAdd(&row[ib], b);
  }
  if (err) atomicCAS(&stats[S_ERR], 0ull, (unsigned long long)(unsigned)err);
}

// stats of the pairs this thread handled (no LDS: see d_stats)
__device__ __forceinline__ void post_stats(unsigned long long nm, unsigned long long np,
                                           int32_t err, unsigned long long *stats) {
  wave_stats(stats, S_MATCHES, nm, S_PAIRS, np, err);
}

// general path: every pair (list == nullptr), or the pairs listed by
// k_post_fast; grid-stride, kPostThreads threads, one workspace slice each
__global__ __launch_bounds__(kB) void k_post(PostCfg c, const uint64_t *__restrict__ match,
                                             const uint32_t *__restrict__ nmatch,
                                             uint64_t n_pairs, const uint32_t *list,
                                             const uint32_t *n_list, int32_t *nk_out,
                                             uint32_t *nmajor_out, HitRows hits_out,
                                             uint64_t *hash_out, unsigned long long *stats,
                                             uint8_t *ws) {
  SMASH_BESIDE_SEARCH();
  int32_t err = 0;
  unsigned long long nm = 0, np = 0;
  const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  uint8_t *my = ws + t * post_ws_bytes(c.slots);
  const uint64_t n = list ? *n_list : n_pairs;
  for (uint64_t i = t; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    unsigned long long m = 0;
    post_pair(c, match, nmatch, list ? list[i] : i, nk_out, nmajor_out, hits_out, hash_out, err,
              m, my);
    nm += m;
    ++np;
  }
  post_stats(nm, np, err, stats);
}

// ---------------------------------------------------------------------------
// k_post_fast: the same per-pair chain with every per-mate list in
// registers.  A mate's alignments and hits are single u64 words whose
// unsigned order is the order the reference sorts them in, so the two sorts
// of Aligner::prepare_matches (to_merge, query.cpp:286; to_print, :301) are
// fixed compare-exchange networks over FCAP words (invalid words are ~0 and
// sort last).  Mates with more than FCAP matches go to k_post.
//   alignment: rc:1 | tid:15 | pos:32 | prefix:8 | len:8   (to_merge order)
//   hit:       qmin:8 | rc:1 | pass:1 | - | tid:16 | pos:32 (to_print order)
// Valid when every contig is shorter than 2^31 and there are fewer than 2^15
// contigs (host check).
// ---------------------------------------------------------------------------
constexpr int FCAP = 16;

__device__ __forceinline__ void cx(uint64_t &a, uint64_t &b) {
  const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
  a = lo;
  b = hi;
}

// append v to list (counter *n) for the lanes with pred: one atomic per
// wave (all lanes of the wave call it)
__device__ __forceinline__ void wave_push(uint32_t *list, uint32_t *n, bool pred, uint32_t v) {
  const uint64_t b = __ballot(pred);
  if (!b) return;
  const uint32_t lane = threadIdx.x & 63, leader = uint32_t(__builtin_ctzll(b));
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(n, uint32_t(__popcll(b)));
  base = __shfl(base, int(leader), 64);
  if (pred) list[base + uint32_t(__popcll(b & ((1ull << lane) - 1)))] = v;
}

// the same network over (key, payload) pairs, ordered by key
template <int N>
__device__ __forceinline__ void sort_net2(uint64_t (&v)[N], uint32_t (&r)[N]) {
#pragma unroll
  for (int p = 1; p < N; p <<= 1)
#pragma unroll
    for (int k = p; k >= 1; k >>= 1)
#pragma unroll
      for (int j = k % p; j <= N - 1 - k; j += 2 * k)
#pragma unroll
        for (int i = 0; i < k; ++i)
          if (i + j + k < N && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
            const bool sw = v[i + j + k] < v[i + j];
            const uint64_t a = v[i + j], b = v[i + j + k];
            const uint32_t ra = r[i + j], rb = r[i + j + k];
            v[i + j] = sw ? b : a; v[i + j + k] = sw ? a : b;
            r[i + j] = sw ? rb : ra; r[i + j + k] = sw ? ra : rb;
          }
}

// Batcher odd-even merge sort, N a power of two (fully unrolled)
template <int N>
__device__ __forceinline__ void sort_net(uint64_t (&v)[N]) {
#pragma unroll
  for (int p = 1; p < N; p <<= 1)
#pragma unroll
    for (int k = p; k >= 1; k >>= 1)
#pragma unroll
      for (int j = k % p; j <= N - 1 - k; j += 2 * k)
#pragma unroll
        for (int i = 0; i < k; ++i)
          if (i + j + k < N && (i + j) / (2 * p) == (i + j + k) / (2 * p))
            cx(v[i + j], v[i + j + k]);
}

// One mate's matches -> its tagged, merged, to_print-ordered hits (H).  The
// loads are issued slot-parallel in five rounds: the match words, the contig
// directory cells, two contig starts per cell, the contig's start / sizes /
// tag offset / small flag, and the two map.bin bytes of every alignment.  A
// slot without a load to make (past n, invalid, or a map byte the search's
// hint already gave) reads a fixed address instead (c.map: one hot line), so
// no load waits on a branch and the rounds overlap their slots' latencies
// (each slot was a chain of ~4 dependent loads, one slot after the other).
template <int CAP>
__device__ __forceinline__ void mate_fast(const PostCfg &c, const uint64_t *__restrict__ sp,
                                          const uint64_t *m, uint32_t n, uint64_t (&H)[CAP],
                                          int32_t &err) {
  const uint32_t L = c.L;
  uint64_t A[CAP];
  uint32_t R[CAP];   // payload through the sort: left byte | right byte << 8 | small << 16
  uint64_t w[CAP];
#pragma unroll
  for (int k = 0; k < CAP; ++k) w[k] = uint32_t(k) < n ? m[k] : 0;
  const uint64_t rmask = c.mhint ? kRefMask : 0xFFFFFFFFFFFFull;
  // round 2: the directory cell of every slot (slots past n: ref 0, cell 0)
  uint32_t c0[CAP], c1[CAP];
#pragma unroll
  for (int k = 0; k < CAP; ++k) {
    uint64_t cl = (w[k] & rmask) >> c.sp_shift;
    cl = cl < c.sp_ncell ? cl : c.sp_ncell - 1;
    c0[k] = c.sp_cell[cl];
    c1[k] = c.sp_cell[cl + 1];
  }
  // round 3: upper_bound(startpos, ref) over [c0, c1): the range's first
  // start decides it when the range holds at most one (almost every cell;
  // the bisection otherwise, rare: several small contigs in one cell)
  uint32_t lo[CAP];
  {
    uint64_t s0[CAP];
#pragma unroll
    for (int k = 0; k < CAP; ++k) s0[k] = sp[c0[k] < c.n_seq ? c0[k] : c.n_seq - 1];
#pragma unroll
    for (int k = 0; k < CAP; ++k) {
      const uint64_t ref = w[k] & rmask;
      uint32_t l = c0[k], h = c1[k];
      if (h - l <= 1) {
        l += uint32_t(l < h && s0[k] <= ref);
      } else {
        while (l < h) {
          const uint32_t mid = (l + h) >> 1;
          if (sp[mid] <= ref) l = mid + 1; else h = mid;
        }
      }
      lo[k] = uint32_t(k) < n ? l : 0u;
    }
  }
  // round 4: the contig's start, its size (forward: the hint's edge rule) or
  // its mate's (reverse strand: the position), its tag offset and small flag
  uint64_t spi[CAP], sz[CAP];
  uint32_t toff[CAP], sml = 0;
#pragma unroll
  for (int k = 0; k < CAP; ++k) {
    const uint32_t si = lo[k] ? lo[k] - 1 : 0;
    spi[k] = sp[si];
    sz[k] = c.sizes[(si & 1) ? si - 1 : si];
    toff[k] = c.tag_off[si >> 1];
    sml |= uint32_t(c.small[si >> 1] != 0) << k;
  }
  // the alignments (Alignment::resolve) and the addresses of their two map
  // bytes: left at the base after the block's end, right at its first base
  // (mappability_tag.cpp:98-101), the right one from the search's hint for a
  // forward match (its own SA row's m, zeroed when m + b >= the contig size,
  // longSA.cpp:666)
  // (xl / xr: the bytes' map entries minus 2, halved; 0 = none to load)
  uint32_t hint[CAP], xl[CAP], xr[CAP];
#pragma unroll
  for (int k = 0; k < CAP; ++k) {
    const uint64_t ref = w[k] & rmask;
    const uint32_t q = uint32_t((w[k] >> 48) & 0xFF), len = uint32_t(w[k] >> 56);
    const uint32_t si = lo[k] ? lo[k] - 1 : 0;
    int64_t pos = int64_t(ref - q - spi[k]);
    const uint32_t extra = L - len - q;
    const uint32_t rc = si & 1;
    if (rc) pos = int64_t(sz[k] - uint64_t(pos)) - int64_t(L);
    const uint64_t prefix = rc ? extra : q;
    const bool ok = uint32_t(k) < n && lo[k] != 0 && pos >= 0;   // erase pos < 0
    A[k] = ok ? (uint64_t(rc) << 63) | (uint64_t(si >> 1) << 48) | (uint64_t(pos) << 16) |
                    (prefix << 8) | len
              : ~0ull;
    const uint32_t h = c.mhint && !rc ? uint32_t(w[k] >> 40) & 0xFFu : 0u;
    hint[k] = h ? 0x100u | (ref - spi[k] + h >= sz[k] ? 0u : h) : 0u;
    // (mapb: an entry past the map reads 0)
    const uint32_t abspos = toff[k] + uint32_t(pos) + 1;
    const uint32_t bl = abspos + uint32_t(prefix) + len - 1, br = abspos + uint32_t(prefix) - 1;
    xl[k] = ok && 2 + uint64_t(bl) * 2 < c.map_bytes ? bl + 1 : 0u;
    xr[k] = ok && !hint[k] && 2 + uint64_t(br) * 2 + 1 < c.map_bytes ? br + 1 : 0u;
  }
  // round 5: every map byte at once (entry 2 + 2 b (+ 1), b = x - 1; x = 0
  // reads the map's first byte, a hot line, and is dropped)
#pragma unroll
  for (int k = 0; k < CAP; ++k) {
    const uint32_t lb = c.map[xl[k] ? uint64_t(xl[k]) * 2 : 0];
    const uint32_t rb = c.map[xr[k] ? uint64_t(xr[k]) * 2 + 1 : 0];
    const bool ok = A[k] != ~0ull;
    const uint32_t lm = xl[k] ? lb : 0u;
    const uint32_t rm = !ok ? 0u : (hint[k] & 0x100u) ? (hint[k] & 0xFFu) : xr[k] ? rb : 0u;
    R[k] = lm | (rm << 8) | (((sml >> k) & 1u) << 16);
  }
  sort_net2(A, R);
  // merge runs on one diagonal (rc, tid, pos) into hits; tag every block
  uint32_t g_prefix = 0, g_qmin = 0;
  int32_t g_l0 = 0, g_r0 = 0;
#pragma unroll
  for (int i = 0; i < CAP; ++i) {
    const uint64_t a = A[i];
    const bool valid = a != ~0ull;
    const uint32_t rc = uint32_t(a >> 63), tid = valid ? uint32_t(a >> 48) & 0x7FFF : 0u;
    const uint32_t pos = uint32_t(a >> 16), prefix = uint32_t(a >> 8) & 0xFF, len = uint32_t(a) & 0xFF;
    const uint32_t qpos = rc ? L - len - prefix : prefix;
    const bool start = i == 0 || (A[i - 1] >> 16) != (a >> 16);
    const bool endg = i + 1 == CAP || (A[i + 1 < CAP ? i + 1 : i] >> 16) != (a >> 16);
    const uint32_t lm = R[i] & 0xFFu, rm = (R[i] >> 8) & 0xFFu;
    const int32_t left = lm ? int32_t(lm) - 1 : 255, right = rm ? int32_t(rm) : 255;
    if (start) {
      g_prefix = prefix; g_qmin = qpos; g_l0 = left; g_r0 = right;
    } else {
      g_qmin = qpos < g_qmin ? qpos : g_qmin;
    }
    if (valid && err == 0 && !((R[i] >> 16) & 1u)) {
      if (uint32_t(left) > len) err = SMASH_ERR_TAG_LEFT;
      else if (uint32_t(right) > len) err = SMASH_ERR_TAG_RIGHT;
    }
    const int32_t mx = g_l0 > g_r0 ? g_l0 : g_r0;
    const uint32_t pass = int32_t(prefix + len) - int32_t(g_prefix) - mx >= c.min_excess;
    H[i] = valid && endg ? (uint64_t(g_qmin) << 56) | (uint64_t(rc) << 55) |
                               (uint64_t(pass) << 54) | (uint64_t(tid) << 32) | pos
                         : ~0ull;
  }
  sort_net(H);
}

__device__ __forceinline__ bool hit_kept(uint64_t h) { return h != ~0ull && ((h >> 54) & 1); }

// CAP words per mate (8: the common case; a pair with a mate above `lim`
// goes to the `up` list, for k_post_fast<16> or, past 16, k_post).  Pairs:
// all n_pairs (list == nullptr) or the *n_list listed ones (grid-stride).
template <int CAP>
__global__ __launch_bounds__(kB) void k_post_fast(PostCfg c, const uint64_t *__restrict__ match,
                                                  const uint32_t *__restrict__ nmatch,
                                                  uint64_t n_pairs, const uint32_t *list,
                                                  const uint32_t *n_list, uint32_t lim,
                                                  uint32_t *up_list, uint32_t *up_n,
                                                  int32_t *nk_out, uint32_t *nmajor_out,
                                                  HitRows hits_out, uint64_t *hash_out,
                                                  unsigned long long *stats) {
  SMASH_BESIDE_SEARCH();
  const uint64_t *sp = c.startpos;
  const uint64_t n = list ? *n_list : n_pairs;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  const uint64_t t0 = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  int32_t err = 0;
  unsigned long long nm = 0, np = 0;
  // every lane runs the same trip count (wave_push is wave-wide)
  for (uint64_t base = t0 - threadIdx.x % 64; base < n; base += stride) {
    const uint64_t i = base + threadIdx.x % 64;
    const bool in = i < n;
    const uint64_t q = in ? (list ? list[i] : i) : 0;
    const uint32_t n1 = in ? nmatch[2 * q] : 0, n2 = in ? nmatch[2 * q + 1] : 0;
    const bool over = in && (n1 > lim || n2 > lim);
    wave_push(up_list, up_n, over, uint32_t(q));
    if (in && !over) {
      nm += n1 + n2;
      ++np;
      uint64_t H1[CAP], H2[CAP];
      mate_fast<CAP>(c, sp, match + (2 * q) * c.slots, n1, H1, err);
      mate_fast<CAP>(c, sp, match + (2 * q + 1) * c.slots, n2, H2, err);
      // (8 words per mate: at most 16 kept hits, the head row; 16 per mate:
      // the full row, copied to the head row below when they fit)
      uint64_t *ho = CAP <= 8 ? hits_out.head + q * kHitHead
                              : hits_out.full + q * (2 * uint64_t(c.slots));
      int32_t nk = -1;
      uint32_t nmaj = 0;
      uint64_t hh = 0x9E3779B97F4A7C15ull, hl = 0xD1B54A32D192ED03ull;
      bool any = false;
#pragma unroll
      for (int i = 0; i < CAP; ++i) any = any || hit_kept(H1[i]) || hit_kept(H2[i]);
      if (any) {                              // smashMEM.py:162
        nk = 0;
        auto put = [&](uint64_t h) {
          const uint32_t tid = uint32_t(h >> 32) & 0xFFFF;
          const int64_t pos = int64_t(uint32_t(h));
          ho[nk++] = (uint64_t(tid) << 48) | uint64_t(pos);
          const uint64_t x = (uint64_t(tid) << 48) ^ uint64_t(pos);
          hh = mix64(hh ^ x) + 0x632BE59BD9B4E019ull;
          hl = mix64(hl + x * 0x9E3779B97F4A7C15ull) ^ (hl >> 29);
          if (c.chrom_off[tid] >= 0) ++nmaj;
        };
#pragma unroll
        for (int i = 0; i < CAP; ++i)
          if (hit_kept(H1[i])) put(H1[i]);
#pragma unroll
        for (int b = 0; b < CAP; ++b) {      // hit window (smashMEM.py:193-200)
          if (!hit_kept(H2[b])) continue;
          bool close = false;
#pragma unroll
          for (int i = 0; i < CAP; ++i) {
            int64_t d = int64_t(uint32_t(H1[i])) - int64_t(uint32_t(H2[b]));
            d = d < 0 ? -d : d;
            close |= hit_kept(H1[i]) && ((H1[i] >> 32) & 0xFFFF) == ((H2[b] >> 32) & 0xFFFF) &&
                     d < c.window;
          }
          if (!close) put(H2[b]);
        }
        hh = (mix64(hh ^ uint64_t(nk)) & c.hash_mask) | 1;
        hl = (mix64(hl + uint64_t(nk)) & c.hash_mask) | 1;
        if (CAP > 8 && nk <= int32_t(kHitHead))
          for (int32_t i = 0; i < nk; ++i) hits_out.head[q * kHitHead + i] = ho[i];
      }
      nk_out[q] = nk;
      nmajor_out[q] = nmaj;
      hash_out[2 * q] = hh;
      hash_out[2 * q + 1] = hl;
    }
  }
  post_stats(nm, np, err, stats);
}

// The persistent pair-key set of smashMEM.py:149,217-228 (dupeSet), exact:
// a key is the pair's kept hit list (tid << 48 | pos0 per hit, r1 then r2 in
// HI order, smashMEM.py:122-131).  Open addressing on the 64-bit hash `hi`;
// slot = {hi, ref}, ref = epoch << 40 | (1 + arena offset of the key record
// [lo, nk, words]) (0: the inserting thread has not published it yet).  A
// hash match counts as the same key only when lo, nk and every hit word
// agree, so a hash collision is a different key (it goes on probing), never a
// false duplicate.
//
// Slot accesses are relaxed, with no per-key release / acquire (agent-scope
// fences write back / invalidate the XCD's L2 on gfx950 and made the round-2
// insert kernel 5 ms per 2 M pairs): a launch compares only against records
// of earlier launches, which are visible across the kernel boundary, and
// against this launch's claims through the claimers' own input rows (the
// claim / decide kernels below).  Epochs wrap after 2^24 launches.
constexpr int kRefShift = 40;
// a published ref (the key's record is in the arena) carries kRefPub; the
// in-batch claims of k_dedup_claim (pair index + 1, this epoch) do not
constexpr uint64_t kRefPub = 1ull << 39;
struct KeyRef {
  const uint64_t *w;   // the key's hit words
  uint32_t nk;
  uint64_t lo;
};

__device__ bool same_key(const uint64_t *rec, const KeyRef &k) {
  if (rec[0] != k.lo || rec[1] != k.nk) return false;
  for (uint32_t i = 0; i < k.nk; ++i)
    if (rec[2 + i] != k.w[i]) return false;
  return true;
}

__device__ bool same_key(const KeyRef &a, const KeyRef &b) {
  if (a.lo != b.lo || a.nk != b.nk) return false;
  for (uint32_t i = 0; i < a.nk; ++i)
    if (a.w[i] != b.w[i]) return false;
  return true;
}

// the wave's inclusive prefix of v (every lane calls it) and its total
__device__ __forceinline__ uint32_t wave_incl(uint32_t v, uint32_t &total) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(v, d, 64);
    if (lane >= uint32_t(d)) v += y;
  }
  total = __shfl(v, 63, 64);
  return v;
}

// the decide kernels take kDecGroups groups of 64 consecutive keys per wave
// per trip and reserve their arena space with ONE atomic: the arena top is a
// single address, and one atomic per 64 keys (~100 k per 6.25 M-pair batch)
// serialised on its L2 channel for ~1 ms
constexpr uint32_t kDecGroups = 4;

// The key records {hash lo, nk, hit words} of a wave's winners, written by
// the whole wave: the decide kernels give each group of 64 keys one
// contiguous arena range
// (lane l's record at off(l), incl = the inclusive prefix of the record
// sizes), so word t of the range belongs to the first lane l with
// incl(l) > t and consecutive lanes store consecutive words (a lane-per-record
// loop stores 64 words a record apart per instruction).  ok: the lane's
// record fits the arena; lo / m / src: its hash lo, word count and words.
// Every lane of the wave calls it (wave-uniform trip count).
__device__ __forceinline__ void wave_fill_records(uint64_t *arena, uint64_t off, uint32_t incl,
                                                  uint32_t total, bool ok, uint64_t lo, uint32_t m,
                                                  const uint64_t *src, bool coop) {
  if (!coop) {   // (SMASH_COOP_COPY=0: one record per lane, the round-3 form)
    if (ok) {
      uint64_t *rec = arena + off;
      rec[0] = lo;
      rec[1] = m;
      for (uint32_t j = 0; j < m; ++j) rec[2 + j] = src[j];
    }
    return;
  }
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t srcv = reinterpret_cast<uint64_t>(src);
  for (uint32_t t0 = 0; t0 < total; t0 += 64) {
    const uint32_t t = t0 + lane;
    uint32_t l = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1)
      if (uint32_t(__shfl(int(incl), int(l + step - 1), 64)) <= t) l += step;
    l = l < 63u ? l : 63u;
    // (the shuffle runs on every lane, outside the select: a cross-lane read
    // under a partial exec mask returns 0 from the lanes it excludes)
    const uint32_t prev = uint32_t(__shfl(int(incl), int((l + 63u) & 63u), 64));
    const uint32_t before = l ? prev : 0u;
    const uint32_t r = t - before;   // word r of lane l's record
    const bool lok = __shfl(int(ok), int(l), 64) != 0;
    const uint64_t loff = __shfl(off, int(l), 64), llo = __shfl(lo, int(l), 64);
    const uint32_t lm = uint32_t(__shfl(int(m), int(l), 64));
    const uint64_t *ls = reinterpret_cast<const uint64_t *>(__shfl(srcv, int(l), 64));
    if (t < total && lok) arena[loff + r] = r == 0 ? llo : r == 1 ? uint64_t(lm) : ls[r - 2];
  }
}

// ---------------------------------------------------------------------------
// Single-GPU de-dup without a sort (the pair-key set of smashMEM.py:149,
// 217-228, first occurrence in pair order wins): two kernels, no LDS, so they
// run beside the next batch's search.
//
// k_dedup_claim: every keyed pair q walks the probe sequence of its hash hi.
//   * an empty slot: CAS the hi in, then publish ref = epoch << 40 | (q + 1),
//     a claim of this batch;
//   * a slot holding hi whose ref is published (kRefPub, an earlier batch's
//     key): same key (record words compared) -> q is a duplicate of an
//     earlier batch; else go on probing (a hash collision);
//   * a slot holding hi claimed in this batch (this epoch, no kRefPub) by pair
//     q2: same key (q2's hit row compared) -> atomicMin the ref with
//     epoch << 40 | (q + 1): the slot ends up naming the smallest pair of the
//     batch with that key; else go on probing.
//   A slot's key never changes once claimed (every pair that lowers its ref
//   has the claimer's key), so a comparison against whichever pair the ref
//   names is a comparison against the claimer.  A claim's ref is stored right
//   after its CAS; a prober that sees the hi before the ref reads the slot
//   again on its next trip.
// k_dedup_decide: pair q is kept iff its slot's ref is still its own claim
//   (the smallest pair of its key in the batch, and the key is new); the
//   kept pair writes the key's record into the arena and publishes the ref
//   (kRefPub: never equal to a claim, so the other pairs of the slot, reading
//   it before or after, all lose).  Fused: k_count_last's per-pair count and
//   last position.
// slot_of[q]: the claimed slot, kSlotOld (a key of an earlier batch) or
// kSlotNone (no key, or the set is full: the error is raised).
// ---------------------------------------------------------------------------
constexpr uint64_t kSlotOld = ~0ull, kSlotNone = ~0ull - 1;
// (single GPU) slot_of flag: the pair's claim filled an empty slot.  Unless
// a later claim of the same key marked it (contest[q]), nobody else claimed
// that slot this batch, so the pair wins and k_dedup_decide skips re-reading
// the slot (one random table line per key).  Every later claimant marks the
// claim it finds (the slot's current minimum), and the first of them finds
// the filler, so a filler that lost is always marked.
constexpr uint64_t kSlotIns = 1ull << 62;

__device__ __forceinline__ KeyRef pair_key(const HitRows &hits, const int32_t *nk,
                                           const uint64_t *hash, uint64_t q) {
  const int32_t k = nk[q];
  return KeyRef{hits.row(q, k), uint32_t(k), hash[2 * q + 1]};
}

__global__ void k_dedup_claim(const int32_t *__restrict__ nk, const uint64_t *__restrict__ hash,
                              HitRows hits, uint64_t n,
                              uint64_t *table, uint64_t mask, const uint64_t *arena,
                              uint64_t epoch, uint64_t *slot_of, uint8_t *contest,
                              unsigned long long *stats) {
  SMASH_BESIDE_SEARCH();
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  int32_t err = 0;
  for (uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; q < n; q += stride) {
    if (nk[q] < 0) continue;
    const KeyRef me = pair_key(hits, nk, hash, q);
    const uint64_t hi = hash[2 * q];
    const unsigned long long mine = (epoch << kRefShift) | (q + 1);
    uint64_t res = kSlotNone;
    uint64_t i = (hi ^ (hi >> 31)) & mask;
    uint32_t waits = 0;
    for (uint64_t probe = 0; probe <= mask;) {
      unsigned long long *sh = reinterpret_cast<unsigned long long *>(&table[2 * i]);
      unsigned long long *sr = sh + 1;
      unsigned long long cur = __hip_atomic_load(sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == 0) {
        const unsigned long long prev = atomicCAS(sh, 0ull, (unsigned long long)hi);
        if (prev == 0) {
          __hip_atomic_store(sr, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          res = i | (contest ? kSlotIns : 0ull);
          break;
        }
        cur = prev;
      }
      if (cur == hi) {
        const unsigned long long ref =
            __hip_atomic_load(sr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ref == 0) {
          // the claimer is between its CAS and its ref store: read this slot
          // again next trip (no wait inside the trip: a claimer in this wave
          // may be laid out after this branch)
          if (++waits > (1u << 22)) {   // (not a reachable state)
            err = SMASH_ERR_UNSUPPORTED;
            break;
          }
          continue;
        }
        if (ref & kRefPub) {
          if ((ref >> kRefShift) != epoch &&
              same_key(arena + ((ref & (kRefPub - 1)) - 1), me)) {
            res = kSlotOld;
            break;
          }
        } else if ((ref >> kRefShift) == epoch) {
          const uint64_t q2 = (ref & (kRefPub - 1)) - 1;
          if (same_key(me, pair_key(hits, nk, hash, q2))) {
            if (contest) contest[q2] = 1;   // (see kSlotIns)
            atomicMin(sr, mine);
            res = i;
            break;
          }
        }
        // (an unpublished ref of an earlier epoch: its batch ran out of
        // arena, an error already raised; no record to compare)
      }
      ++probe;
      i = (i + 1) & mask;
    }
    if (res == kSlotNone && err == 0) err = SMASH_ERR_NOMEM;   // the set is full
    slot_of[q] = res;
  }
  if (err) atomicCAS(&stats[S_ERR], 0ull, (unsigned long long)(unsigned)err);
}

// one wave per kDecGroups x 64 consecutive pairs per trip (wave-wide scans)
__global__ void k_dedup_decide(const int32_t *__restrict__ nk, const uint64_t *__restrict__ hash,
                               HitRows hits,
                               const uint32_t *__restrict__ nmajor,
                               const int64_t *__restrict__ chrom_off, uint64_t n,
                               uint64_t *table, uint64_t *arena, uint64_t arena_cap,
                               unsigned long long *arena_top, uint64_t epoch,
                               const uint64_t *__restrict__ slot_of,
                               const uint8_t *__restrict__ contest, uint8_t *keep,
                               uint32_t *cnt, int64_t *lp, unsigned long long *stats, bool coop) {
  SMASH_BESIDE_SEARCH();
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  unsigned long long kp = 0, dp = 0;
  bool full = false;
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t b0 = (uint64_t(blockIdx.x) * blockDim.x + (threadIdx.x & ~63u)) * kDecGroups;
       b0 < n; b0 += stride * kDecGroups) {
    bool wins[kDecGroups];
    uint32_t needs[kDecGroups], incls[kDecGroups], tots[kDecGroups];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t g = 0; g < kDecGroups; ++g) {
      const uint64_t q = b0 + 64 * g + lane;
      const int32_t m = q < n ? nk[q] : -1;
      bool win = false;
      if (m >= 0) {
        const uint64_t sl = slot_of[q];
        if (sl < kSlotNone && (sl & kSlotIns) && !contest[q]) {
          win = true;                       // the slot's only claimant this batch
        } else if (sl < kSlotNone) {
          const unsigned long long ref = __hip_atomic_load(
              reinterpret_cast<unsigned long long *>(&table[2 * (sl & ~kSlotIns) + 1]),
              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          win = ref == ((epoch << kRefShift) | (q + 1));
        }
        ++kp;
        dp += win ? 0 : 1;
      }
      wins[g] = win;
      needs[g] = win ? 2u + uint32_t(m) : 0u;
      incls[g] = wave_incl(needs[g], tots[g]);
      sum += tots[g];
    }
    unsigned long long wbase = 0;
    if (lane == 63 && sum) wbase = atomicAdd(arena_top, (unsigned long long)sum);
    wbase = __shfl(wbase, 63, 64);
#pragma unroll
    for (uint32_t g = 0; g < kDecGroups; ++g) {
      const uint64_t q = b0 + 64 * g + lane;
      const bool in = q < n;
      const int32_t m = in ? nk[q] : -1;
      const bool win = wins[g];
      const uint32_t need = needs[g], incl = incls[g], total = tots[g];
      const uint64_t off = uint64_t(wbase) + incl - need;
      wbase += total;
      const bool ok = win && off + need <= arena_cap;
      wave_fill_records(arena, off, incl, total, ok, win ? hash[2 * q + 1] : 0ull,
                        win ? uint32_t(m) : 0u, hits.row(in ? q : 0, m), coop);
      if (win) {
        if (!ok) {
          full = true;   // the slot stays a claim: never matched (no kRefPub)
        } else {
          __hip_atomic_store(
              reinterpret_cast<unsigned long long *>(&table[2 * (slot_of[q] & ~kSlotIns) + 1]),
              (unsigned long long)((epoch << kRefShift) | kRefPub | (off + 1)), __ATOMIC_RELAXED,
              __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (in) {
        keep[q] = win ? 1 : 0;
        const uint32_t c = win ? nmajor[q] : 0;   // k_count_last
        cnt[q] = c;
        int64_t last = -1;
        if (c) {
          const uint64_t *h = hits.row(q, m);
          for (int32_t j = m - 1; j >= 0; --j)
            if (chrom_off[uint32_t(h[j] >> 48)] >= 0) {
              last = int64_t(h[j] & 0xFFFFFFFFFFFFull);
              break;
            }
        }
        lp[q] = last;
      }
    }
  }
  wave_stats(stats, S_KEYPAIRS, kp, S_DUPEPAIRS, dp, full ? SMASH_ERR_NOMEM : 0);
}

// ---------------------------------------------------------------------------
// The two scans of the fused positions path without LDS (hipcub's use LDS and
// a decoupled look-back): per pair cnt (u32, inclusive sum -> posoff[q + 1])
// and lp (i64, inclusive "last valid" -> lps[q]).  A wave owns a tile of
// kScanTile consecutive pairs, kScanPer per lane; (1) tile aggregates, (2)
// one wave scans the aggregates into tile prefixes, (3) every tile re-scans
// its pairs from its prefix.
// ---------------------------------------------------------------------------
constexpr uint32_t kScanPer = 16, kScanTile = 64 * kScanPer;

__device__ __forceinline__ int64_t last_valid(int64_t a, int64_t b) { return b >= 0 ? b : a; }

// inclusive scans over the wave of (s, l) (sum, last valid)
__device__ __forceinline__ void wave_scan(uint64_t &s, int64_t &l) {
  const uint32_t lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t ys = __shfl_up(s, d, 64);
    const int64_t yl = __shfl_up(l, d, 64);
    if (lane >= uint32_t(d)) {
      s += ys;
      l = last_valid(yl, l);
    }
  }
}

// a lane's kScanPer consecutive (cnt, lp): 16-byte loads when the run is
// whole (q0 is a multiple of 16, the arrays are 256-byte aligned), one
// element per load at the batch's end (4 + 8 loads per lane instead of 32:
// the lanes' runs are 64 / 128 bytes apart, so each element load of a wave
// touched 64 lines)
__device__ __forceinline__ void scan_run(const uint32_t *__restrict__ cnt,
                                         const int64_t *__restrict__ lp, uint64_t q0, uint64_t n,
                                         uint32_t (&c)[kScanPer], int64_t (&v)[kScanPer]) {
  if (q0 + kScanPer <= n) {
    const uint4 *cv = reinterpret_cast<const uint4 *>(cnt + q0);
    const longlong2 *lv = reinterpret_cast<const longlong2 *>(lp + q0);
#pragma unroll
    for (uint32_t k = 0; k < kScanPer / 4; ++k) {
      const uint4 x = cv[k];
      c[4 * k] = x.x; c[4 * k + 1] = x.y; c[4 * k + 2] = x.z; c[4 * k + 3] = x.w;
    }
#pragma unroll
    for (uint32_t k = 0; k < kScanPer / 2; ++k) {
      const longlong2 y = lv[k];
      v[2 * k] = y.x; v[2 * k + 1] = y.y;
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
      const bool ok = q0 + k < n;
      c[k] = ok ? cnt[q0 + k] : 0;
      v[k] = ok ? lp[q0 + k] : -1;
    }
  }
}

__global__ void k_scan_tiles(const uint32_t *__restrict__ cnt, const int64_t *__restrict__ lp,
                             uint64_t n, uint64_t *tsum, int64_t *tlast) {
  SMASH_BESIDE_SEARCH();
  const uint64_t t = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
  const uint64_t q0 = t * kScanTile + uint64_t(threadIdx.x & 63) * kScanPer;
  uint64_t s = 0;
  int64_t l = -1;
  if (t * kScanTile < n) {
    uint32_t c[kScanPer];
    int64_t v[kScanPer];
    scan_run(cnt, lp, q0, n, c, v);
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
      s += c[k];
      l = last_valid(l, v[k]);
    }
  }
  wave_scan(s, l);
  if ((threadIdx.x & 63) == 63 && t * kScanTile < n) {
    tsum[t] = s;
    tlast[t] = l;
  }
}

// one wave: the exclusive prefixes of the ntile aggregates, in place
__global__ void k_scan_top(uint64_t *tsum, int64_t *tlast, uint64_t ntile) {
  SMASH_BESIDE_SEARCH();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t per = (ntile + 63) / 64;
  const uint64_t a = lane * per, b = a + per < ntile ? a + per : ntile;
  uint64_t s = 0;
  int64_t l = -1;
  for (uint64_t t = a; t < b; ++t) {
    s += tsum[t];
    l = last_valid(l, tlast[t]);
  }
  uint64_t is = s;
  int64_t il = l;
  wave_scan(is, il);
  uint64_t es = __shfl_up(is, 1, 64);   // exclusive prefix of this lane's range
  int64_t el = __shfl_up(il, 1, 64);
  if (lane == 0) { es = 0; el = -1; }
  for (uint64_t t = a; t < b; ++t) {
    const uint64_t ts = tsum[t];
    const int64_t tl = tlast[t];
    tsum[t] = es;
    tlast[t] = el;
    es += ts;
    el = last_valid(el, tl);
  }
}

__global__ void k_scan_apply(const uint32_t *__restrict__ cnt, const int64_t *__restrict__ lp,
                             uint64_t n, const uint64_t *__restrict__ tsum,
                             const int64_t *__restrict__ tlast, uint32_t *posoff, int64_t *lps) {
  SMASH_BESIDE_SEARCH();
  const uint64_t t = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
  const uint64_t q0 = t * kScanTile + uint64_t(threadIdx.x & 63) * kScanPer;
  const bool live = t * kScanTile < n;
  uint32_t c[kScanPer];
  int64_t v[kScanPer];
  uint64_t s = 0;
  int64_t l = -1;
  scan_run(cnt, lp, q0, live ? n : 0, c, v);
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k) {
    s += c[k];
    l = last_valid(l, v[k]);
  }
  uint64_t is = s;
  int64_t il = l;
  wave_scan(is, il);
  uint64_t es = __shfl_up(is, 1, 64);
  int64_t el = __shfl_up(il, 1, 64);
  if ((threadIdx.x & 63) == 0) { es = 0; el = -1; }
  if (!live) return;
  es += tsum[t];
  el = last_valid(tlast[t], el);
  if (q0 + kScanPer <= n) {   // whole run: 16-byte stores (posoff's are 4 bytes off alignment)
    uint32_t po[kScanPer];
    int64_t lo[kScanPer];
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
      es += c[k];
      el = last_valid(el, v[k]);
      po[k] = uint32_t(es);
      lo[k] = el;
    }
    __builtin_memcpy(posoff + q0 + 1, po, sizeof(po));
    __builtin_memcpy(lps + q0, lo, sizeof(lo));
    return;
  }
#pragma unroll
  for (uint32_t k = 0; k < kScanPer; ++k) {
    if (q0 + k >= n) break;
    es += c[k];
    el = last_valid(el, v[k]);
    posoff[q0 + k + 1] = uint32_t(es);
    lps[q0 + k] = el;
  }
}

__global__ void k_count(const uint8_t *keep, const uint32_t *nmajor, uint64_t n,
                        uint32_t *cnt) {
  const uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (q < n) cnt[q] = keep[q] ? nmajor[q] : 0;
}

__global__ void k_emit(const uint8_t *keep, const int32_t *nk,
                       HitRows hits, const uint32_t *off, uint64_t n,
                       const int64_t *chrom_off, int64_t *pos0, int64_t *absp) {
  const uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (q >= n || !keep[q]) return;
  const uint64_t *h = hits.row(q, nk[q]);
  uint64_t o = off[q];
  for (int32_t i = 0; i < nk[q]; ++i) {
    const uint32_t tid = uint32_t(h[i] >> 48);
    const int64_t p = int64_t(h[i] & 0xFFFFFFFFFFFFull);
    const int64_t co = chrom_off[tid];
    if (co < 0) continue;
    pos0[o] = p;
    absp[o] = p + co;
    ++o;
  }
}

// the bin of absolute position a (varbin: bisect_right over the starts,
// wrapping to the last bin below the first start), the cell directory
// narrowing the bisect when present
__device__ __forceinline__ uint32_t bin_of(int64_t a, const int64_t *__restrict__ bins,
                                           uint32_t nbins, const uint32_t *__restrict__ cell,
                                           uint32_t ncell, uint32_t cshift) {
  uint32_t lo = 0, hi = nbins;
  if (cell) {
    uint64_t c = a < 0 ? 0 : uint64_t(a) >> cshift;
    c = c < ncell ? c : ncell - 1;
    lo = cell[c];
    hi = cell[c + 1];
  }
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (a < bins[mid]) hi = mid; else lo = mid + 1;
  }
  return lo == 0 ? nbins - 1 : lo - 1;
}

// "last valid" scan operator (associative): the right operand unless it is -1
struct LastValid {
  __host__ __device__ int64_t operator()(int64_t a, int64_t b) const { return b >= 0 ? b : a; }
};

// varbin: adjacent de-dup on the pos string (== pos0), bisect_right, count.
__global__ __launch_bounds__(kB) void k_bin(const int64_t *__restrict__ pos0,
                                            const int64_t *__restrict__ absp,
                                            const uint32_t *npos_p, const int64_t *prev_p,
                                            const int64_t *__restrict__ bins, uint32_t nbins,
                                            const uint32_t *__restrict__ cell, uint32_t ncell,
                                            uint32_t cshift, unsigned long long *counts,
                                            unsigned long long *stats) {
  const uint64_t n = *npos_p;
  const int64_t prev0 = *prev_p;
  unsigned long long d = 0, k = 0, t = 0;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t p = pos0[i];
    const int64_t pr = i ? pos0[i - 1] : prev0;
    ++t;
    if (pr >= 0 && pr == p) { ++d; continue; }
    atomicAdd(&counts[bin_of(absp[i], bins, nbins, cell, ncell, cshift)], 1ull);
    ++k;
  }
  __shared__ unsigned long long sd, sk, st;
  if (threadIdx.x == 0) { sd = 0; sk = 0; st = 0; }
  __syncthreads();
  if (t) { atomicAdd(&st, t); atomicAdd(&sd, d); atomicAdd(&sk, k); }
  __syncthreads();
  if (threadIdx.x == 0 && st) {
    atomicAdd(&stats[S_POS], st);
    atomicAdd(&stats[S_DUPS], sd);
    atomicAdd(&stats[S_KEPT], sk);
  }
}

// per pair: the count of positions it emits (kept pairs: their major hits)
// and the pos0 of the last one (-1: none), read from the end of its hit row
__global__ void k_count_last(const uint8_t *keep, const uint32_t *nmajor, const int32_t *nk,
                             HitRows hits, const int64_t *chrom_off,
                             uint64_t n, uint32_t *cnt, int64_t *lp) {
  const uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const uint32_t c = keep[q] ? nmajor[q] : 0;
  cnt[q] = c;
  int64_t last = -1;
  if (c) {
    const uint64_t *h = hits.row(q, nk[q]);
    for (int32_t i = nk[q] - 1; i >= 0; --i)
      if (chrom_off[uint32_t(h[i] >> 48)] >= 0) {
        last = int64_t(h[i] & 0xFFFFFFFFFFFFull);
        break;
      }
  }
  lp[q] = last;
}

// positions + varbin in one pass (smash_mapping.sh:29 then varbin.py:52-92):
// one thread per pair walks its kept major hits in emission order; the line
// before its first is the last position of the nearest earlier pair that
// emitted any (the "last valid" scan lps), else the carried one.  Same
// adjacent de-dup, bins and statistics as k_emit followed by k_bin, without
// writing and re-reading the positions.
__global__ __launch_bounds__(kB) void k_emit_bin(
    const uint8_t *__restrict__ keep, const int32_t *__restrict__ nk,
    HitRows hits, const int64_t *__restrict__ chrom_off,
    const int64_t *__restrict__ lps, uint64_t n, const int64_t *prev_p,
    const int64_t *__restrict__ bins, uint32_t nbins, const uint32_t *__restrict__ cell,
    uint32_t ncell, uint32_t cshift, unsigned long long *counts, unsigned long long *stats) {
  SMASH_BESIDE_SEARCH();
  const int64_t prev0 = *prev_p;
  unsigned long long d = 0, k = 0, t = 0;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; q < n; q += stride) {
    if (!keep[q]) continue;
    const int32_t m = nk[q];
    if (m <= 0) continue;
    int64_t prev = q ? lps[q - 1] : -1;
    if (prev < 0) prev = prev0;
    const uint64_t *h = hits.row(q, m);
    for (int32_t i = 0; i < m; ++i) {
      const uint64_t w = h[i];
      const int64_t co = chrom_off[uint32_t(w >> 48)];
      if (co < 0) continue;
      const int64_t p = int64_t(w & 0xFFFFFFFFFFFFull);
      ++t;
      if (prev >= 0 && prev == p) {
        ++d;
      } else {
        atomicAdd(&counts[bin_of(p + co, bins, nbins, cell, ncell, cshift)], 1ull);
        ++k;
      }
      prev = p;
    }
  }
  wave_stats(stats, S_POS, t, S_DUPS, d, 0);   // no LDS (d_stats)
  wave_stats(stats, S_KEPT, k, S_KEPT, 0, 0);
}

// k_emit_bin with the counts summed on chip: a global atomic per position
// (one lane per random bin, executed at the memory side) is the slow shape
// of an atomic (MI355X_MICROARCH.md, Global float atomics).  The bins are
// cut in parts of kBinPart LDS counters; block (x, part) walks the pairs
// of its x slice, bins every emitted position as k_emit_bin does, counts the
// ones in its part in LDS and adds the part to the global counts once, lane
// i -> bin i (whole contiguous rows).  Every part re-walks the pairs (the
// walk, a chain of dependent loads per pair at 16 waves per CU, is the
// kernel's cost); part 0 keeps the stats.
//
// Round 4: the counters are 16-bit, two to an LDS word, so one part holds
// 77 824 bins (C3's 50 000 in one walk instead of two).  A half never
// overflows: the increment that takes a half from flush - 1 to flush (the
// atomic's old value tells exactly one thread) subtracts flush from it and
// adds flush to the global count; at most 1023 other increments of the block
// land between the two, and flush + 1023 < 2^16 (flush <= 2^15).
constexpr uint32_t kBinPart = 77824;   // 16-bit counters: 152 KB, one 1024-thread block per CU
constexpr uint32_t kBinPartsMax = 4;   // above: k_emit_bin
constexpr uint32_t kBinBlocks = 256;   // k_emit_bin_lds blocks per part (one per CU)
// the parts balanced: ceil(nbins / parts) bins each (50 k bins: 2 x 25 000,
// not 24 576 + 24 576 + 848 -- every part re-walks all the pairs)
inline uint32_t bin_parts(uint32_t nbins) { return (nbins + kBinPart - 1) / kBinPart; }
inline uint32_t bin_part_size(uint32_t nbins) {
  const uint32_t np = bin_parts(nbins);
  return np ? (nbins + np - 1) / np : 1;
}
__global__ __launch_bounds__(1024) void k_emit_bin_lds(
    const uint8_t *__restrict__ keep, const int32_t *__restrict__ nk,
    HitRows hits, const int64_t *__restrict__ chrom_off,
    const int64_t *__restrict__ lps, uint64_t n, const int64_t *prev_p,
    const int64_t *__restrict__ bins, uint32_t nbins, const uint32_t *__restrict__ cell,
    uint32_t ncell, uint32_t cshift, unsigned long long *counts, unsigned long long *stats,
    uint32_t part, uint32_t flush, uint32_t *binpart) {
  __shared__ uint32_t hc[kBinPart / 2];   // bin b0 + i: half i & 1 of word i >> 1
  const uint32_t b0 = blockIdx.y * part;
  const uint32_t b1 = b0 + part < nbins ? b0 + part : nbins;
  for (uint32_t i = threadIdx.x; i < (part + 1) / 2; i += blockDim.x) hc[i] = 0;
  __syncthreads();
  const int64_t prev0 = *prev_p;
  unsigned long long d = 0, k = 0, t = 0;
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  // a pair's inputs are fetched one trip ahead (keep, nk, lps[q - 1] and its
  // first 4 hit words as one 32-byte row prefix): the walk is a chain of
  // dependent loads per pair, and the next pair's part of it now overlaps
  // this pair's bin lookups
  struct Ahead {
    uint32_t kp;
    int32_t m;
    int64_t lp;
    uint4 h0, h1;
  };
  auto fetch = [&](uint64_t x) {
    Ahead a{0u, 0, -1, make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
    if (x < n) {
      a.kp = keep[x];
      a.m = nk[x];
      a.lp = x ? lps[x - 1] : -1;
      // (the head row's first 4 words, fetched before nk is known: a pair
      // with more than kHitHead hits reads its full row below instead)
      const uint4 *r = reinterpret_cast<const uint4 *>(hits.head + x * kHitHead);
      a.h0 = r[0];
      a.h1 = r[1];
    }
    return a;
  };
  uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  Ahead cur = fetch(q);
  for (; q < n; q += stride) {
    const Ahead nxt = fetch(q + stride);
    const int32_t m = cur.kp ? cur.m : 0;
    int64_t prev = cur.lp < 0 ? prev0 : cur.lp;
    const uint64_t *h = hits.row(q, cur.m);
    const int32_t pre = cur.m <= int32_t(kHitHead) ? 4 : 0;   // words from the prefetch
    for (int32_t i = 0; i < m; ++i) {
      const uint4 &hv = i < 2 ? cur.h0 : cur.h1;
      const uint64_t w = i >= pre ? h[i]
                                : (i & 1) ? (uint64_t(hv.w) << 32 | hv.z) : (uint64_t(hv.y) << 32 | hv.x);
      const int64_t co = chrom_off[uint32_t(w >> 48)];
      if (co < 0) continue;
      const int64_t p = int64_t(w & 0xFFFFFFFFFFFFull);
      ++t;
      if (prev >= 0 && prev == p) {
        ++d;
      } else {
        const uint32_t b = bin_of(p + co, bins, nbins, cell, ncell, cshift);
        if (b >= b0 && b < b1) {
          const uint32_t sh = 16 * ((b - b0) & 1);
          const uint32_t old = atomicAdd(&hc[(b - b0) >> 1], 1u << sh);
          if (((old >> sh) & 0xFFFFu) == flush - 1) {
            atomicSub(&hc[(b - b0) >> 1], flush << sh);
            atomicAdd(&counts[b], (unsigned long long)flush);
          }
        }
        ++k;
      }
      prev = p;
    }
    cur = nxt;
  }
  __shared__ unsigned long long sd, sk, st;
  if (threadIdx.x == 0) { sd = 0; sk = 0; st = 0; }
  __syncthreads();
  if (blockIdx.y == 0 && t) { atomicAdd(&st, t); atomicAdd(&sd, d); atomicAdd(&sk, k); }
  __syncthreads();
  if (threadIdx.x == 0 && st) {
    atomicAdd(&stats[S_POS], st);
    atomicAdd(&stats[S_DUPS], sd);
    atomicAdd(&stats[S_KEPT], sk);
  }
  // the block's counts as plain coalesced stores, k_bin_reduce sums the
  // blocks (no global atomic per non-zero bin per block)
  uint32_t *out = binpart + uint64_t(blockIdx.x) * nbins;
  for (uint32_t i = threadIdx.x; b0 + i < b1; i += blockDim.x)
    out[b0 + i] = (hc[i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
}

// counts[b] += the blocks' partial counts of bin b (one thread per bin), as
// an atomic: the caller's counts may be shared with other pipelines or
// streams (at most nbins atomics per batch, none for an empty bin)
__global__ void k_bin_reduce(const uint32_t *__restrict__ binpart, uint32_t blocks, uint32_t nbins,
                             unsigned long long *counts) {
  for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < nbins; b += gridDim.x * blockDim.x) {
    unsigned long long t = 0;
    for (uint32_t k = 0; k < blocks; ++k) t += binpart[uint64_t(k) * nbins + b];
    if (t) atomicAdd(&counts[b], t);
  }
}

// the batch's tail {count, last position} (lps_last: lps[n - 1]; count 0:
// -1) and the carried line for the next batch
__global__ void k_tail_lps(const uint32_t *npos_p, const int64_t *lps_last, int64_t *prev,
                           int64_t *tail) {
  const uint32_t c = *npos_p;
  const int64_t last = c ? *lps_last : -1;
  if (tail) { tail[0] = int64_t(c); tail[1] = last; }
  if (prev && c) prev[0] = last;
}

__global__ void k_tail(const uint32_t *npos_p, const int64_t *pos0, int64_t *prev,
                       int64_t *tail) {
  const uint32_t n = *npos_p;
  const int64_t last = n ? pos0[n - 1] : -1;
  if (tail) { tail[0] = int64_t(n); tail[1] = last; }
  if (prev && n) prev[0] = last;
}

__global__ void k_reset_prev(int64_t *prev) {
  prev[0] = -1;
  prev[1] = -1;
}

hipError_t ensure_positions(smash_pipeline *p) {
  if (p->d_pos0 && p->d_abs) return hipSuccess;
  const uint64_t n = p->max_pairs * 2 * p->slots;
  hipError_t e = p->d_pos0 ? hipSuccess : hipMalloc(reinterpret_cast<void **>(&p->d_pos0), 8 * n);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&p->d_abs), 8 * n);
  if (e != hipSuccess) {   // all or nothing: a later call must not find half the arrays
    (void)hipFree(p->d_pos0);
    p->d_pos0 = nullptr;
    p->d_abs = nullptr;
  }
  return e;
}

int check_pipe(smash_pipeline *p, uint64_t n_pairs) {
  if (!p) { set_error("null pipeline"); return SMASH_ERR_ARG; }
  if (n_pairs > p->max_pairs) {
    set_error("batch larger than cfg.max_pairs");
    return SMASH_ERR_ARG;
  }
  return SMASH_OK;
}

PostCfg post_cfg(const smash_pipeline *p) {
  PostCfg c;
  c.startpos = p->ix->d_startpos;
  c.sizes = p->ix->d_sizes;
  c.n_seq = p->ix->n_seq;
  c.L = p->read_len;
  c.slots = p->slots;
  c.tag_off = p->d_tag_off;
  c.small = p->d_small;
  c.chrom_off = p->d_chrom_off;
  c.map = p->ix->d_map;
  c.map_bytes = p->ix->map_bytes;
  c.min_excess = p->min_excess;
  c.window = p->hit_window;
  c.fast_cap = p->post_cap;
  c.hash_mask = p->hash_mask;
  c.sp_cell = p->d_sp_cell;
  c.sp_shift = p->sp_shift;
  c.sp_ncell = p->sp_ncell;
  c.mhint = p->mhint;
  return c;
}

HitRows hit_rows(const smash_pipeline *p) { return HitRows{p->d_hhead, p->d_hits, p->slots}; }

}  // namespace
}  // namespace smash

using namespace smash;

// table slots and arena words for a key set of `keys` keys (at least the
// batch's max_pairs): 2x the keys in power-of-two slots, 16 words per key
static void key_set_geometry(uint64_t keys, uint64_t max_pairs, uint64_t *slots,
                             uint64_t *arena_words) {
  const uint64_t cap = 2 * std::max<uint64_t>(keys, max_pairs);
  uint64_t pw = 1;
  while (pw < cap) pw <<= 1;
  *slots = pw;
  *arena_words = std::min<uint64_t>(16 * std::max<uint64_t>(keys, max_pairs) + (1u << 20),
                                    kRefPub - 2);
}

extern "C" uint64_t smash_pipeline_max_batch(uint32_t read_len, uint32_t min_len) {
  if (read_len == 0 || read_len > 255 || min_len < 2 || read_len < min_len) return 0;
  const uint64_t slots = read_len - min_len + 1;
  return ((1ull << 32) - 1) / (2 * slots);
}

extern "C" int smash_pipeline_create(const smash_index *ix,
                                     const smash_pipeline_cfg *cfg,
                                     smash_pipeline **out) {
  if (!ix || !cfg || !out || cfg->read_len == 0 || cfg->read_len > 255 ||
      cfg->min_len < 2 || cfg->read_len < cfg->min_len || cfg->max_pairs == 0 ||
      cfg->max_pairs > smash_pipeline_max_batch(cfg->read_len, cfg->min_len) ||
      cfg->n_contig * 2 != ix->n_seq ||
      !cfg->h_tag_offsets || !cfg->h_small_chr || !cfg->h_chrom_off ||
      !cfg->h_bin_starts || cfg->nbins == 0) {
    set_error("smash_pipeline_create: bad configuration");
    return SMASH_ERR_ARG;
  }
  if (cfg->read_stride && cfg->read_stride != cfg->read_len &&
      cfg->read_stride != smash_read_stride(cfg->read_len)) {
    set_error("smash_pipeline_create: read_stride must be 0, read_len or smash_read_stride(read_len)");
    return SMASH_ERR_ARG;
  }
  if (!ix->rcref) {   // the SMASH chain maps with -rcref (smash_mapping.sh:19)
    set_error("smash_pipeline_create: the count chain needs the -rcref text layout");
    return SMASH_ERR_ARG;
  }
  if (!ix->d_map) {
    set_error("smash_pipeline_create: index has no map.bin");
    return SMASH_ERR_ARG;
  }
  auto *p = new smash_pipeline;
  try {
    SMASH_HIPX(hipSetDevice(ix->device));
    p->ix = ix;
    p->device = ix->device;
    p->read_len = cfg->read_len;
    p->stride = cfg->read_stride ? cfg->read_stride : cfg->read_len;
    p->min_len = cfg->min_len;
    p->slots = cfg->read_len - cfg->min_len + 1;
    p->n_contig = cfg->n_contig;
    p->nbins = cfg->nbins;
    p->min_excess = cfg->min_excess;
    p->hit_window = cfg->hit_window;
    p->max_pairs = cfg->max_pairs;
    const uint64_t P = cfg->max_pairs;
    p->d_tag_off = dalloc<uint32_t>(p->n_contig);
    p->d_small = dalloc<uint8_t>(p->n_contig);
    p->d_chrom_off = dalloc<int64_t>(p->n_contig);
    p->d_bins = dalloc<int64_t>(p->nbins);
    SMASH_HIPX(hipMemcpy(p->d_tag_off, cfg->h_tag_offsets, 4 * p->n_contig, hipMemcpyHostToDevice));
    {
      const char *mh = getenv("SMASH_MAP_HINT");
      bool ok = !(mh && mh[0] == '0') && ix->pos_mask == kPkPosMask && ix->rcref && ix->d_map &&
                ix->map_own;
      uint64_t off = 0;
      for (uint32_t t = 0; ok && t < p->n_contig; ++t) {
        ok = cfg->h_tag_offsets[t] == off;
        off += ix->sizes[2 * t];
      }
      p->mhint = ok;
    }
    SMASH_HIPX(hipMemcpy(p->d_small, cfg->h_small_chr, p->n_contig, hipMemcpyHostToDevice));
    SMASH_HIPX(hipMemcpy(p->d_chrom_off, cfg->h_chrom_off, 8 * p->n_contig, hipMemcpyHostToDevice));
    SMASH_HIPX(hipMemcpy(p->d_bins, cfg->h_bin_starts, 8 * p->nbins, hipMemcpyHostToDevice));
    {   // bin directory (k_bin): at most 2^18 cells; only for ascending, non-negative starts
      const int64_t *b = cfg->h_bin_starts;
      bool ok = b[0] >= 0;
      for (uint32_t k = 1; k < p->nbins && ok; ++k) ok = b[k] >= b[k - 1];
      if (ok) {
        const uint64_t top = uint64_t(b[p->nbins - 1]);
        uint32_t sh = 10;
        while ((top >> sh) + 2 > (1u << 18)) ++sh;
        p->cshift = sh;
        p->ncell = uint32_t((top >> sh) + 2);
        std::vector<uint32_t> cell(p->ncell + 1);
        uint32_t r = 0;
        for (uint32_t c = 0; c < p->ncell; ++c) {
          const int64_t x = int64_t(uint64_t(c) << sh);
          while (r < p->nbins && b[r] <= x) ++r;   // bisect_right(bins, x)
          cell[c] = r;
        }
        cell[p->ncell] = p->nbins;
        p->d_cell = dalloc<uint32_t>(p->ncell + 1);
        SMASH_HIPX(hipMemcpy(p->d_cell, cell.data(), 4 * (p->ncell + 1), hipMemcpyHostToDevice));
      }
    }
    {   // contig directory (PostCfg::sp_cell): at most 2^16 cells over the text
      const std::vector<uint64_t> &sp = ix->startpos;
      const uint64_t top = ix->N;
      uint32_t sh = 8;
      while ((top >> sh) + 2 > (1u << 16)) ++sh;
      p->sp_shift = sh;
      p->sp_ncell = uint32_t((top >> sh) + 2);
      std::vector<uint32_t> cell(p->sp_ncell + 1);
      uint32_t r = 0;
      for (uint32_t c = 0; c < p->sp_ncell; ++c) {
        const uint64_t x = uint64_t(c) << sh;
        while (r < sp.size() && sp[r] <= x) ++r;   // upper_bound(startpos, x)
        cell[c] = r;
      }
      cell[p->sp_ncell] = uint32_t(sp.size());
      p->d_sp_cell = dalloc<uint32_t>(p->sp_ncell + 1);
      SMASH_HIPX(hipMemcpy(p->d_sp_cell, cell.data(), 4 * (p->sp_ncell + 1), hipMemcpyHostToDevice));
    }
    p->rec_bytes = search_rec_bytes(2 * P, p->read_len);
    int search_prio = 0;
    if (const char *e = getenv("SMASH_SEARCH_PRIO")) {
      int least = 0, greatest = 0;
      SMASH_HIPX(hipDeviceGetStreamPriorityRange(&least, &greatest));
      if (!strcmp(e, "high")) search_prio = greatest;
      else if (!strcmp(e, "low")) search_prio = least;
    }
    for (int k = 0; k < 2; ++k) {
      p->d_match_s[k] = dalloc<uint64_t>(2 * P * p->slots);
      p->d_nmatch_s[k] = dalloc<uint32_t>(2 * P);
      // (the records: only for dense input, allocated by the first search that needs them)
      p->d_work_s[k] = dalloc<unsigned long long>(1);
      // SMASH_SEARCH_PRIO=high / low: the search streams at that priority.
      // HIP shares a process's hardware queues among its streams once it
      // has GPU_MAX_HW_QUEUES (4) of them, one pool per priority; with RCCL
      // and gloo streams in the process (the sharded step) a search stream
      // landed on the caller's stream's queue, so the next search waited
      // behind every exchange kernel queued before it.  A stream of its own
      // priority gets a queue from another pool.
      if (search_prio) {
        SMASH_HIPX(hipStreamCreateWithPriority(&p->xs[k], hipStreamNonBlocking, search_prio));
      } else {
        SMASH_HIPX(hipStreamCreateWithFlags(&p->xs[k], hipStreamNonBlocking));
      }
      SMASH_HIPX(hipEventCreateWithFlags(&p->ev_found[k], hipEventDisableTiming));
      SMASH_HIPX(hipEventCreateWithFlags(&p->ev_free[k], hipEventDisableTiming));
    }
    SMASH_HIPX(hipEventCreateWithFlags(&p->ev_in, hipEventDisableTiming));
    SMASH_HIPX(hipEventCreateWithFlags(&p->ev_done, hipEventDisableTiming));
    SMASH_HIPX(hipEventRecord(p->ev_done, nullptr));
    SMASH_HIPX(hipEventSynchronize(p->ev_done));
    p->d_match = p->d_match_s[0];
    p->d_nmatch = p->d_nmatch_s[0];
    p->d_nk = dalloc<int32_t>(P);
    p->d_nmajor = dalloc<uint32_t>(P);
    p->d_hits = dalloc<uint64_t>(P * 2 * p->slots);
    p->d_hhead = dalloc<uint64_t>(P * smash::kHitHead);
    p->d_hash = dalloc<uint64_t>(2 * P);
    p->d_keep = dalloc<uint8_t>(P);
    {   // the multi-GPU export's per-(owner, block) counts, up to 64 owners
      const uint64_t nb = 64 * ((P + kB - 1) / kB);
      p->d_bcnt = dalloc<uint64_t>(nb);
      p->d_boff = dalloc<uint64_t>(nb);
      SMASH_HIPX(hipcub::DeviceScan::ExclusiveSum(nullptr, p->scan_temp_bytes, p->d_bcnt,
                                                  p->d_boff, nb));
      p->d_scan_temp = dalloc<uint8_t>(p->scan_temp_bytes);
    }
    size_t b = 0;
    p->d_posoff = dalloc<uint32_t>(P + 1);
    p->d_cnt = dalloc<uint32_t>(P);
    SMASH_HIPX(hipcub::DeviceScan::InclusiveSum(nullptr, b, p->d_cnt, p->d_posoff + 1, P));
    size_t c3 = 0;
    SMASH_HIPX(hipcub::DeviceScan::InclusiveScan(nullptr, c3, static_cast<const int64_t *>(nullptr),
                                                 static_cast<int64_t *>(nullptr), LastValid(), P));
    p->temp_bytes = std::max(b, c3);
    p->d_temp = dalloc<uint8_t>(p->temp_bytes);
    // key records: 2 + nk words each; SMASH reads keep ~7 hits per pair, the
    // arena holds 16 words per key of the capacity (an exhausted arena is a
    // reported error, SMASH_ERR_NOMEM, never a silent cut; refs hold offset
    // + 1 below kRefPub)
    uint64_t pw = 0;
    key_set_geometry(cfg->dedup_capacity, P, &pw, &p->arena_cap);
    p->table_mask = pw - 1;
    p->d_table = dalloc<uint64_t>(2 * pw);
    SMASH_HIPX(hipMemset(p->d_table, 0, 16 * pw));
    p->d_arena = dalloc<uint64_t>(p->arena_cap);
    p->d_arena_top = dalloc<unsigned long long>(1);
    SMASH_HIPX(hipMemset(p->d_arena_top, 0, 8));
    p->d_prev = dalloc<int64_t>(2);
    p->d_lp = dalloc<int64_t>(P);
    p->d_lps = dalloc<int64_t>(P);
    {
      const char *e = getenv("SMASH_FUSED_BIN");   // 0: k_emit + k_bin (A/B)
      p->fused_bin = !(e && e[0] == '0');
      const char *l = getenv("SMASH_BIN_LDS");   // profiles/r03/binlds: 1.39 vs 2.18 ms
      // (k_emit_bin_lds only where its parts fit: above kBinPartsMax parts,
      // k_emit_bin with global atomics, and no per-block count buffer)
      p->bin_lds = !(l && l[0] == '0') && p->fused_bin && bin_parts(p->nbins) <= kBinPartsMax;
      if (p->bin_lds) p->d_binpart = dalloc<uint32_t>(uint64_t(kBinBlocks) * p->nbins);
      // SMASH_BIN_FLUSH (tests): k_emit_bin_lds's flush threshold, a power of
      // two in [2, 2^15] (default 2^15)
      const char *fl = getenv("SMASH_BIN_FLUSH");
      const unsigned long f = fl ? std::strtoul(fl, nullptr, 10) : 0;
      if (f >= 2 && f <= 0x8000 && !(f & (f - 1))) p->bin_flush = uint32_t(f);
      const char *cc = getenv("SMASH_COOP_COPY");
      if (cc) p->coop_copy = uint32_t(std::strtoul(cc, nullptr, 10)) & 7u;
      auto on = [](const char *v, bool dflt) {
        const char *x = getenv(v);
        return x && x[0] ? x[0] == '1' : dflt;
      };
      p->gate_prep = on("SMASH_GATE_PREP", false);
      p->gate_post = on("SMASH_GATE_POST", true);   // profiles/r03/sched: 150.9 vs 160.1 ms
      p->one_search = on("SMASH_ONE_SEARCH", false);
    }
    // the positions arrays (2 x 8 B x every hit slot: 26 GB at 6.25 M
    // pairs) only for the two-kernel path; the fused path writes them when
    // smash_pipeline_positions asks (ensure_positions)
    if (!p->fused_bin) SMASH_HIPX(ensure_positions(p));
    int64_t init[2] = {-1, -1};
    SMASH_HIPX(hipMemcpy(p->d_prev, init, 16, hipMemcpyHostToDevice));
    p->d_stats = dalloc<unsigned long long>(kStatWords);
    SMASH_HIPX(hipMemset(p->d_stats, 0, 8 * kStatWords));
    p->d_slot = dalloc<uint64_t>(P);
    {
      const char *cf = getenv("SMASH_CLAIM_FLAG");   // (A/B: 0 = every decide reads its slot)
      if (!(cf && cf[0] == '0')) p->d_contest = dalloc<uint8_t>(P);
    }
    p->d_tsum = dalloc<uint64_t>(P / kScanTile + 1);
    p->d_tlast = dalloc<int64_t>(P / kScanTile + 1);
    p->d_send_q = dalloc<uint32_t>(P);
    p->d_fb = dalloc<uint32_t>(P + 1);
    p->d_l16 = dalloc<uint32_t>(P + 1);
    p->d_post_ws = dalloc<uint8_t>(uint64_t(kPostThreads) * post_ws_bytes(p->slots));
    {
      bool ok = p->n_contig < 0x7FFF;
      for (uint64_t z : ix->sizes) ok = ok && z < (1ull << 31);
      const char *e = getenv("SMASH_POST_LEGACY");
      p->post_fast = ok && !(e && *e && *e != '0');
      // SMASH_POST_CAP < 16 routes more pairs to the general kernel (tests)
      const char *pc = getenv("SMASH_POST_CAP");
      const uint32_t cap = pc && *pc ? uint32_t(atoi(pc)) : uint32_t(FCAP);
      p->post_cap = std::min<uint32_t>({cap, uint32_t(FCAP), p->slots});
    }
    if (const char *hb = getenv("SMASH_KEY_HASH_BITS")) {   // tests: force collisions
      const int b = atoi(hb);
      if (b > 0 && b < 64) p->hash_mask = (1ull << b) - 1;
    }
    p->d_owner = dalloc<unsigned long long>(4 * 64);
    p->d_send_hdr = dalloc<uint64_t>(uint64_t(kHdrWords) * P);
    p->d_recv_base = dalloc<uint64_t>(2 * 65);
    SMASH_HIPX(hipHostMalloc(reinterpret_cast<void **>(&p->h_owner), 8 * 256, hipHostMallocDefault));
    SMASH_HIPX(hipHostMalloc(reinterpret_cast<void **>(&p->h_recv_base), 8 * 2 * 65,
                             hipHostMallocDefault));
    SMASH_HIPX(hipEventCreateWithFlags(&p->ev_base, hipEventDisableTiming));
    SMASH_HIPX(hipMemset(p->d_posoff, 0, 4));
  } catch (hip_failure &f) {
    set_error(f.what);
    smash_pipeline_free(p);
    return SMASH_ERR_NOMEM;
  }
  *out = p;
  return SMASH_OK;
}

namespace smash {
uint32_t pipe_read_len(const smash_pipeline *p) { return p->read_len; }
uint32_t pipe_stride(const smash_pipeline *p) { return p->stride; }
uint64_t pipe_max_pairs(const smash_pipeline *p) { return p->max_pairs; }
int pipe_device(const smash_pipeline *p) { return p->device; }
void *&pipe_feed(smash_pipeline *p, void (*freer)(void *)) {
  p->feed_free = freer;
  return p->feed;
}
}  // namespace smash

extern "C" void smash_pipeline_free(smash_pipeline *p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  if (p->feed && p->feed_free) p->feed_free(p->feed);
  for (hipEvent_t e : p->ev) (void)hipEventDestroy(e);
  for (int k = 0; k < 2; ++k) {
    if (p->xs[k]) {
      (void)hipStreamSynchronize(p->xs[k]);
      (void)hipStreamDestroy(p->xs[k]);
    }
    if (p->ev_found[k]) (void)hipEventDestroy(p->ev_found[k]);
    if (p->ev_free[k]) (void)hipEventDestroy(p->ev_free[k]);
    for (void *q : {(void *)p->d_match_s[k], (void *)p->d_nmatch_s[k], (void *)p->d_rec_s[k],
                    (void *)p->d_work_s[k]})
      dfree(q);
  }
  if (p->ev_in) (void)hipEventDestroy(p->ev_in);
  if (p->ev_done) (void)hipEventDestroy(p->ev_done);
  if (p->ev_base) (void)hipEventDestroy(p->ev_base);
  if (p->h_owner) (void)hipHostFree(p->h_owner);
  if (p->h_recv_base) (void)hipHostFree(p->h_recv_base);
  for (void *q : {(void *)p->d_tag_off, (void *)p->d_small, (void *)p->d_chrom_off,
                  (void *)p->d_bins, (void *)p->d_cell, (void *)p->d_sp_cell,
                  (void *)p->d_nk, (void *)p->d_nmajor, (void *)p->d_hits, (void *)p->d_hhead,
                  (void *)p->d_hash, (void *)p->d_keep, (void *)p->d_bcnt, (void *)p->d_boff,
                  p->d_scan_temp, (void *)p->d_oslot,
                  (void *)p->d_slot, (void *)p->d_contest, (void *)p->d_tsum, (void *)p->d_tlast,
                  p->d_temp, (void *)p->d_table,
                  (void *)p->d_posoff, (void *)p->d_cnt, (void *)p->d_pos0,
                  (void *)p->d_abs, (void *)p->d_prev, (void *)p->d_stats,
                  (void *)p->d_lp, (void *)p->d_lps, (void *)p->d_binpart,
                  (void *)p->d_send_q, (void *)p->d_owner, (void *)p->d_fb, (void *)p->d_l16,
                  (void *)p->d_post_ws, (void *)p->d_arena, (void *)p->d_arena_top,
                  (void *)p->d_send_hdr, (void *)p->d_send_words, (void *)p->d_recv_base})
    dfree(q);
  delete p;
}

// the search of n_pairs pairs into set k on its stream, after in_ev (the
// reads are ready) and after the post stage that last read the set
static int search_into(smash_pipeline *p, int k, const uint8_t *d_reads, uint64_t n_pairs,
                       hipEvent_t in_ev) {
  hipStream_t xs = p->xs[k];
  SMASH_HIP(hipStreamWaitEvent(xs, in_ev, 0));
  if (p->one_search && p->found_rec[k ^ 1]) SMASH_HIP(hipStreamWaitEvent(xs, p->ev_found[k ^ 1], 0));
  if (p->gate_prep && p->set_used[k]) SMASH_HIP(hipStreamWaitEvent(xs, p->ev_free[k], 0));
  // the set's records were last read by its previous search, earlier on xs;
  // its match buffers by that batch's post stage: k_prep runs now, the
  // search after ev_free (SearchWs::gate)
  if (p->prof) {
    if (2 * p->n_ev + 2 > p->ev.size()) {
      for (int q = 0; q < 64; ++q) {
        hipEvent_t e;
        SMASH_HIP(hipEventCreate(&e));
        p->ev.push_back(e);
      }
    }
    p->ix->kev[0] = p->ev[2 * p->n_ev];          // recorded around k_mam_sm itself
    p->ix->kev[1] = p->ev[2 * p->n_ev + 1];
  }
  if (!search_direct(d_reads, p->stride, p->read_len) && !p->d_rec_s[k]) {   // k_prep's records
    SMASH_HIP(hipStreamSynchronize(xs));
    SMASH_HIP(hipMalloc(reinterpret_cast<void **>(&p->d_rec_s[k]), p->rec_bytes));
  }
  const SearchWs ws{p->d_rec_s[k], p->d_rec_s[k] ? p->rec_bytes : 0, p->d_work_s[k],
                    p->set_used[k] && !p->gate_prep ? p->ev_free[k] : nullptr, p->mhint};
  const int rc = map_batch_impl(p->ix, SMASH_MODE_MAM, p->min_len, d_reads, p->stride, nullptr,
                                p->read_len, 2 * n_pairs, p->d_match_s[k], p->slots,
                                p->d_nmatch_s[k], xs, false, &ws);   // probe check at stats time
  p->ix->kev[0] = p->ix->kev[1] = nullptr;
  if (rc) return rc;
  if (p->prof) {
    ++p->n_ev;
    p->prof_reads += 2 * n_pairs;
  }
  SMASH_HIP(hipEventRecord(p->ev_found[k], xs));
  p->found_rec[k] = true;
  p->pref_reads[k] = d_reads;
  p->pref_n[k] = n_pairs;
  p->searched[k] = true;
  return SMASH_OK;
}

// map -> resolve/tag/filter/hash -> in-batch order.  The search runs on the
// next set's stream once `in_ev` (the reads are ready) and the set's previous
// post stage have completed (unless smash_phase_map_ahead already searched
// these reads into that set); the rest runs on s after the search.  in_ev
// null: recorded on s now (everything before this call on s).  d_next: the
// next batch's search is issued into the other set right after this one's,
// before this batch's post stage is queued, so it runs while the caller
// works on this batch.
static int phase_map_impl(smash_pipeline *p, const uint8_t *d_reads, uint64_t n_pairs,
                          hipStream_t s, hipEvent_t in_ev, const uint8_t *d_next = nullptr,
                          uint64_t n_next = 0) {
  int rc = check_pipe(p, n_pairs);
  if (rc) return rc;
  if (d_next && (rc = check_pipe(p, n_next))) return rc;
  p->last = s;
  p->n_pairs = n_pairs;
  if (!n_pairs) return SMASH_OK;
  SMASH_HIP(hipSetDevice(p->device));
  const int k = p->set ^= 1;
  p->d_match = p->d_match_s[k];
  p->d_nmatch = p->d_nmatch_s[k];
  const bool have = p->searched[k] && p->pref_reads[k] == d_reads && p->pref_n[k] == n_pairs;
  if (!in_ev && p->reads_resident) in_ev = p->ev_done;   // (complete since creation)
  if (!in_ev && (!have || (d_next && n_next))) {
    in_ev = p->ev_in;
    SMASH_HIP(hipEventRecord(in_ev, s));
  }
  if (!have && (rc = search_into(p, k, d_reads, n_pairs, in_ev))) return rc;
  p->searched[k] = false;   // consumed by this batch
  const bool next_have = p->searched[k ^ 1] && p->pref_reads[k ^ 1] == d_next &&
                         p->pref_n[k ^ 1] == n_next;   // (smash_phase_search_ahead)
  if (d_next && n_next && !next_have && (rc = search_into(p, k ^ 1, d_next, n_next, in_ev)))
    return rc;
  SMASH_HIP(hipStreamWaitEvent(s, p->ev_found[k], 0));
  if (p->post_fast) {
    // mates of <= 8 matches (most pairs) in 8-word networks, <= 16 in
    // 16-word ones, the rest in the general kernel
    SMASH_HIP(hipMemsetAsync(p->d_fb, 0, 4, s));
    SMASH_HIP(hipMemsetAsync(p->d_l16, 0, 4, s));
    const PostCfg pc = post_cfg(p);
    k_post_fast<8><<<grid_for(n_pairs, kB, 1u << 30), kB, 0, s>>>(
        pc, p->d_match, p->d_nmatch, n_pairs, nullptr, nullptr, std::min(8u, p->post_cap),
        p->d_l16 + 1, p->d_l16, p->d_nk, p->d_nmajor, hit_rows(p), p->d_hash, p->d_stats);
    SMASH_HIP(hipGetLastError());
    k_post_fast<FCAP><<<grid_for(n_pairs, kB, 1024), kB, 0, s>>>(
        pc, p->d_match, p->d_nmatch, n_pairs, p->d_l16 + 1, p->d_l16, p->post_cap,
        p->d_fb + 1, p->d_fb, p->d_nk, p->d_nmajor, hit_rows(p), p->d_hash, p->d_stats);
    SMASH_HIP(hipGetLastError());
    k_post<<<kPostBlocks, kB, 0, s>>>(post_cfg(p), p->d_match, p->d_nmatch, n_pairs,
                                      p->d_fb + 1, p->d_fb, p->d_nk, p->d_nmajor, hit_rows(p),
                                      p->d_hash, p->d_stats, p->d_post_ws);
  } else {
    k_post<<<kPostBlocks, kB, 0, s>>>(post_cfg(p), p->d_match, p->d_nmatch, n_pairs, nullptr,
                                      nullptr, p->d_nk, p->d_nmajor, hit_rows(p), p->d_hash,
                                      p->d_stats, p->d_post_ws);
  }
  SMASH_HIP(hipGetLastError());
  if (!p->defer_free)
    SMASH_HIP(hipEventRecord(p->ev_free[k], s));   // the set's matches are read
  p->set_used[k] = true;
  p->cnt_ready = false;
  return SMASH_OK;
}

extern "C" int smash_phase_map(smash_pipeline *p, const uint8_t *d_reads,
                               uint64_t n_pairs, void *stream) {
  return phase_map_impl(p, d_reads, n_pairs, static_cast<hipStream_t>(stream), nullptr);
}

extern "C" int smash_phase_map_ahead(smash_pipeline *p, const uint8_t *d_reads,
                                     uint64_t n_pairs, const uint8_t *d_next, uint64_t n_next,
                                     void *stream) {
  return phase_map_impl(p, d_reads, n_pairs, static_cast<hipStream_t>(stream), nullptr, d_next,
                        n_next);
}

// the search of the batch after the next one, into the set the current
// batch used: its post stage has read that set's matches once
// smash_phase_export has returned (the host synchronisation there), so the
// search is gated on nothing the caller still waits for; the next-but-one
// smash_phase_map[_ahead] with the same reads uses it
extern "C" int smash_phase_search_ahead(smash_pipeline *p, const uint8_t *d_reads,
                                        uint64_t n_pairs, void *stream) {
  int rc = check_pipe(p, n_pairs);
  if (rc) return rc;
  if (!n_pairs) return SMASH_OK;
  const int k = p->set;   // the set of the batch smash_phase_map last took
  if (p->searched[k]) {
    set_error("smash_phase_search_ahead: the set still holds an unconsumed search");
    return SMASH_ERR_ARG;
  }
  SMASH_HIP(hipSetDevice(p->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p->reads_resident) return search_into(p, k, d_reads, n_pairs, p->ev_done);
  SMASH_HIP(hipEventRecord(p->ev_in, s));   // the reads are ready after the caller's work
  return search_into(p, k, d_reads, n_pairs, p->ev_in);
}

// 1 .. 2^24 - 1, never 0 (an unpublished slot)
static uint64_t next_epoch(smash_pipeline *p) {
  p->epoch = p->epoch % ((1ull << (64 - smash::kRefShift)) - 1) + 1;
  return p->epoch;
}

// single GPU: the persistent set, first occurrence in pair order
// (k_dedup_claim, k_dedup_decide), and the positions' per-pair counts
static int dedup_local(smash_pipeline *p, hipStream_t s) {
  const uint64_t n = p->n_pairs;
  if (!n) return SMASH_OK;
  const uint64_t epoch = next_epoch(p);
  if (p->d_contest) SMASH_HIP(hipMemsetAsync(p->d_contest, 0, n, s));
  k_dedup_claim<<<grid_for(n, kB, 8192), kB, 0, s>>>(p->d_nk, p->d_hash, hit_rows(p), n,
                                                     p->d_table, p->table_mask, p->d_arena, epoch,
                                                     p->d_slot, p->d_contest, p->d_stats);
  SMASH_HIP(hipGetLastError());
  k_dedup_decide<<<grid_for((n + kDecGroups - 1) / kDecGroups, kB, 8192), kB, 0, s>>>(
      p->d_nk, p->d_hash, hit_rows(p), p->d_nmajor, p->d_chrom_off, n, p->d_table,
      p->d_arena, p->arena_cap, p->d_arena_top, epoch, p->d_slot, p->d_contest, p->d_keep,
      p->d_cnt, p->d_lp, p->d_stats, (p->coop_copy & 2u) != 0);
  SMASH_HIP(hipGetLastError());
  p->cnt_ready = true;
  return SMASH_OK;
}

extern "C" int smash_phase_positions(smash_pipeline *p, int64_t *d_tail, void *stream) {
  if (!p) return SMASH_ERR_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  p->last = s;
  const uint64_t n = p->n_pairs;
  if (p->fused_bin) {
    // counts, offsets and each pair's preceding line; the positions
    // themselves are only written if someone asks (smash_pipeline_positions)
    if (n) {
      if (!p->cnt_ready)   // (the multi-GPU path: keep came from the owners)
        k_count_last<<<grid_for(n, kB, 1u << 30), kB, 0, s>>>(p->d_keep, p->d_nmajor, p->d_nk,
                                                             hit_rows(p), p->d_chrom_off,
                                                             n, p->d_cnt, p->d_lp);
      // posoff (offsets) and lps ("last valid" position), no LDS
      const uint64_t ntile = (n + kScanTile - 1) / kScanTile;
      const unsigned g = unsigned((ntile * 64 + kB - 1) / kB);
      k_scan_tiles<<<g, kB, 0, s>>>(p->d_cnt, p->d_lp, n, p->d_tsum, p->d_tlast);
      k_scan_top<<<1, 64, 0, s>>>(p->d_tsum, p->d_tlast, ntile);
      k_scan_apply<<<g, kB, 0, s>>>(p->d_cnt, p->d_lp, n, p->d_tsum, p->d_tlast, p->d_posoff,
                                    p->d_lps);
      SMASH_HIP(hipGetLastError());
      p->pos_dirty = true;
    }
    k_tail_lps<<<1, 1, 0, s>>>(p->d_posoff + n, p->d_lps + (n ? n - 1 : 0), nullptr, d_tail);
    SMASH_HIP(hipGetLastError());
    return SMASH_OK;
  }
  if (n) {
    k_count<<<grid_for(n, kB, 1u << 30), kB, 0, s>>>(p->d_keep, p->d_nmajor, n, p->d_cnt);
    size_t tb = p->temp_bytes;
    SMASH_HIP(hipcub::DeviceScan::InclusiveSum(p->d_temp, tb, p->d_cnt, p->d_posoff + 1, n, s));
    k_emit<<<grid_for(n, kB, 1u << 30), kB, 0, s>>>(p->d_keep, p->d_nk, hit_rows(p),
                                                    p->d_posoff, n,
                                                    p->d_chrom_off, p->d_pos0, p->d_abs);
  }
  p->pos_dirty = false;
  k_tail<<<1, 1, 0, s>>>(p->d_posoff + n, p->d_pos0, nullptr, d_tail);
  SMASH_HIP(hipGetLastError());
  return SMASH_OK;
}

extern "C" int smash_phase_bin(smash_pipeline *p, const int64_t *d_prev,
                               uint64_t *d_counts, void *stream) {
  if (!p || !d_counts) return SMASH_ERR_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  p->last = s;
  const uint64_t n = p->n_pairs;
  const int64_t *prev = d_prev ? d_prev : p->d_prev;
  if (p->fused_bin) {
    const uint32_t parts = bin_parts(p->nbins);
    if (n && p->bin_lds) {   // (set only when parts <= kBinPartsMax)
      const uint32_t part = bin_part_size(p->nbins);
      const unsigned gx = unsigned(std::min<uint64_t>(kBinBlocks, (n + 1023) / 1024));
      const dim3 grid(gx, parts);
      k_emit_bin_lds<<<grid, 1024, 0, s>>>(
          p->d_keep, p->d_nk, hit_rows(p), p->d_chrom_off, p->d_lps, n, prev, p->d_bins,
          p->nbins, p->d_cell, p->ncell, p->cshift, reinterpret_cast<unsigned long long *>(d_counts),
          p->d_stats, part, p->bin_flush, p->d_binpart);
      k_bin_reduce<<<grid_for(p->nbins, kB, 1024), kB, 0, s>>>(
          p->d_binpart, gx, p->nbins, reinterpret_cast<unsigned long long *>(d_counts));
    } else if (n) {
      k_emit_bin<<<grid_for(n, kB, 8192), kB, 0, s>>>(
          p->d_keep, p->d_nk, hit_rows(p), p->d_chrom_off, p->d_lps, n, prev, p->d_bins,
          p->nbins, p->d_cell, p->ncell, p->cshift, reinterpret_cast<unsigned long long *>(d_counts),
          p->d_stats);
    }
    // carry the adjacent-dup state across batches (single-GPU use)
    k_tail_lps<<<1, 1, 0, s>>>(p->d_posoff + n, p->d_lps + (n ? n - 1 : 0), p->d_prev, nullptr);
    SMASH_HIP(hipGetLastError());
    return SMASH_OK;
  }
  k_bin<<<2048, kB, 0, s>>>(p->d_pos0, p->d_abs, p->d_posoff + n, prev, p->d_bins,
                            p->nbins, p->d_cell, p->ncell, p->cshift,
                            reinterpret_cast<unsigned long long *>(d_counts),
                            p->d_stats);
  // carry the adjacent-dup state across batches (single-GPU use)
  k_tail<<<1, 1, 0, s>>>(p->d_posoff + n, p->d_pos0, p->d_prev, nullptr);
  SMASH_HIP(hipGetLastError());
  return SMASH_OK;
}

namespace smash {
// one batch, its search after in_ev (null: after everything on s so far)
int count_batch_ev(smash_pipeline *p, const uint8_t *d_reads, uint64_t n_pairs,
                   uint64_t *d_counts, hipStream_t s, hipEvent_t in_ev) {
  p->defer_free = p->gate_post;
  p->keys_bound += n_pairs;
  int rc = phase_map_impl(p, d_reads, n_pairs, s, in_ev);
  p->defer_free = false;
  if (rc) return rc;
  rc = dedup_local(p, s);
  if (!rc) rc = smash_phase_positions(p, nullptr, s);
  if (!rc) rc = smash_phase_bin(p, nullptr, d_counts, s);
  // on every exit once the search is queued: the set's next search must
  // follow whatever of this batch's post stage was queued on s
  if (p->gate_post && n_pairs && hipEventRecord(p->ev_free[p->set], s) != hipSuccess && !rc) {
    set_error("hipEventRecord failed");
    rc = SMASH_ERR_HIP;
  }
  return rc;
}
}  // namespace smash

extern "C" int smash_count_batch(smash_pipeline *p, const uint8_t *d_reads,
                                 uint64_t n_pairs, uint64_t *d_counts, void *stream) {
  return smash::count_batch_ev(p, d_reads, n_pairs, d_counts, static_cast<hipStream_t>(stream),
                               nullptr);
}

// ready: the reads' input event (hipEvent_t); null with `resident`: none
static int count_batches_impl(smash_pipeline *p, const uint8_t *d_reads, uint64_t n_pairs,
                              uint64_t batch_pairs, uint64_t *d_counts, hipStream_t s,
                              hipEvent_t ready, bool resident) {
  if (!p || (n_pairs && !d_reads) || !d_counts || batch_pairs == 0 ||
      batch_pairs > p->max_pairs) {
    set_error("smash_count_batches: bad arguments");
    return SMASH_ERR_ARG;
  }
  SMASH_HIP(hipSetDevice(p->device));
  // one input event for all batches, so batch b + 1's search can start under
  // the tail of batch b's: the caller's, an event already complete (resident
  // reads), or every batch's reads are ready once the work before this call
  // on s is
  hipEvent_t in_ev = ready ? ready : resident ? p->ev_done : nullptr;
  const bool own = !in_ev;
  int rc = SMASH_OK;
  if (own) {
    SMASH_HIP(hipEventCreateWithFlags(&in_ev, hipEventDisableTiming));
    rc = hipEventRecord(in_ev, s) == hipSuccess ? SMASH_OK : SMASH_ERR_HIP;
  }
  const uint64_t L2 = 2 * uint64_t(p->stride);
  for (uint64_t b0 = 0; rc == SMASH_OK && b0 < n_pairs; b0 += batch_pairs) {
    const uint64_t n = std::min(batch_pairs, n_pairs - b0);
    rc = smash::count_batch_ev(p, d_reads + b0 * L2, n, d_counts, s, in_ev);
  }
  if (own) (void)hipEventDestroy(in_ev);   // released once the waits on it have completed
  return rc;
}

extern "C" int smash_count_batches(smash_pipeline *p, const uint8_t *d_reads, uint64_t n_pairs,
                                   uint64_t batch_pairs, uint64_t *d_counts, void *stream) {
  return count_batches_impl(p, d_reads, n_pairs, batch_pairs, d_counts,
                            static_cast<hipStream_t>(stream), nullptr, false);
}

extern "C" int smash_count_batches_ready(smash_pipeline *p, const uint8_t *d_reads,
                                         uint64_t n_pairs, uint64_t batch_pairs,
                                         uint64_t *d_counts, void *stream, void *ready) {
  return count_batches_impl(p, d_reads, n_pairs, batch_pairs, d_counts,
                            static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(ready),
                            true);
}

// ---- multi-GPU de-dup exchange ------------------------------------------------
// Each rank exports its keyed pairs to owner = (hash hi >> 1) % world: a
// 3-word header {hi, lo, nk << 40 | word offset} per key and the
// key's nk hit words (hash + canonical key bytes + index).
// The owner decides first-wins over the exact keys and answers one byte per
// header.
namespace smash {
namespace {
// the owner rank of a key: its hash hi without bit 0, which is always set
// (0 marks an empty slot of the key set), so hi % world would leave every
// even rank of an even world without keys and double the odd ranks' share
__device__ __forceinline__ uint64_t key_owner(uint64_t hi, int world) {
  return (hi >> 1) % uint64_t(world);
}
// The export in pair order, without a sort (round 4).  Every keyed pair is
// exported -- the in-batch first occurrence is the owner's to decide, like
// the earlier batches' (in-batch duplicates are ~1% of the keys) -- and each
// owner's segment of the send buffer holds its keys in pair order: a stable
// multi-split.  Global pair order is (step, rank, pair), so an owner's
// receive buffer (source ranks in rank order, each segment in pair order)
// lists this step's keys in global order, and the first claim in that order
// is the first-wins pair of smashMEM.py:217-228.
//
// k_export_count: per block b and owner o, the keyed pairs and their hit
//   words, packed as keys << 32 | words into bc[o * nblk + b] (owner-major).
//   An exclusive scan of bc then gives every (owner, block) its offsets in the
//   owner-major send buffer: the owner's segment start plus the blocks
//   before it.  Exact while a batch's words stay below 2^32: a pair exports
//   at most 2 * slots words, and smash_pipeline_create refuses max_pairs *
//   2 * slots >= 2^32 (smash_pipeline_max_batch; 16.39 M pairs at 150 bp,
//   3.28e9 words at the bench's 12.5 M).
// k_export_fill: the same per-block grouping, each lane's rank among its
//   block's keys of the same owner (wave ballots, then the waves before it),
//   and the scanned block offset: the header, the words and the pair index
//   of the send slot.
constexpr uint32_t kExWaves = kB / 64;

// per wave: for every owner present, the group's key count and word total
// (s_e / s_w[wave][o], written by the group's first lane); each lane gets its
// rank in the group and the words before it
struct WaveGroup {
  uint32_t rank, wbefore;
};
__device__ __forceinline__ WaveGroup wave_owner_groups(bool act, uint32_t ow, uint32_t k,
                                                       uint32_t *s_e, uint32_t *s_w) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1;
  WaveGroup mine{0, 0};
  uint64_t todo = __ballot(act);
  while (todo) {
    const int leader = __builtin_ctzll(todo);
    const uint32_t o = uint32_t(__shfl(int(ow), leader, 64));
    const bool in = act && ow == o;
    const uint64_t same = __ballot(in);
    uint32_t x = in ? k : 0u;   // inclusive scan of the group's word counts
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= uint32_t(d)) x += y;
    }
    const uint32_t wsum = __shfl(x, 63, 64);
    if (lane == uint32_t(leader)) {
      s_e[o] = uint32_t(__popcll(same));
      s_w[o] = wsum;
    }
    if (in) {
      mine.rank = uint32_t(__popcll(same & below));
      mine.wbefore = x - k;
    }
    todo &= ~same;
  }
  return mine;
}

__global__ __launch_bounds__(kB) void k_export_count(const int32_t *nk, const uint64_t *hash,
                                                     uint64_t n, int world, uint32_t nblk,
                                                     uint64_t *bc) {
  __shared__ uint32_t s_e[kExWaves][64], s_w[kExWaves][64];
  const uint32_t wv = threadIdx.x >> 6;
  for (uint32_t o = threadIdx.x; o < kExWaves * 64; o += blockDim.x) {
    (&s_e[0][0])[o] = 0;
    (&s_w[0][0])[o] = 0;
  }
  __syncthreads();
  const uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const bool act = q < n && nk[q] >= 0;
  const uint32_t ow = act ? uint32_t(key_owner(hash[2 * q], world)) : 0u;
  (void)wave_owner_groups(act, ow, act ? uint32_t(nk[q]) : 0u, s_e[wv], s_w[wv]);
  __syncthreads();
  for (uint32_t o = threadIdx.x; o < uint32_t(world); o += blockDim.x) {
    uint64_t e = 0, w = 0;
    for (uint32_t v = 0; v < kExWaves; ++v) {
      e += s_e[v][o];
      w += s_w[v][o];
    }
    bc[uint64_t(o) * nblk + blockIdx.x] = (e << 32) | w;
  }
}

// per owner: keys, words (host images: the collectives' split sizes)
__global__ void k_export_totals(const uint64_t *bc, const uint64_t *boff, int world,
                                uint32_t nblk, unsigned long long *tot) {
  const uint32_t o = threadIdx.x;
  if (o >= uint32_t(world)) return;
  const uint64_t last = uint64_t(o + 1) * nblk - 1;
  const uint64_t end = boff[last] + bc[last], beg = boff[uint64_t(o) * nblk];
  tot[o] = (end >> 32) - (beg >> 32);
  tot[64 + o] = (end & 0xFFFFFFFFull) - (beg & 0xFFFFFFFFull);
}

__global__ __launch_bounds__(kB) void k_export_fill(const int32_t *nk, const uint64_t *hash,
                                                    HitRows hits,
                                                    uint64_t n, int world, uint32_t nblk,
                                                    uint64_t gbase, const uint64_t *boff,
                                                    uint64_t *hdr, uint64_t *words,
                                                    uint32_t *send_q, bool coop) {
  __shared__ uint32_t s_e[kExWaves][64], s_w[kExWaves][64];
  const uint32_t wv = threadIdx.x >> 6;
  for (uint32_t o = threadIdx.x; o < kExWaves * 64; o += blockDim.x) {
    (&s_e[0][0])[o] = 0;
    (&s_w[0][0])[o] = 0;
  }
  __syncthreads();
  const uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const bool act = q < n && nk[q] >= 0;
  const uint32_t ow = act ? uint32_t(key_owner(hash[2 * q], world)) : 0u;
  const uint32_t k = act ? uint32_t(nk[q]) : 0u;
  const WaveGroup g = wave_owner_groups(act, ow, k, s_e[wv], s_w[wv]);
  __syncthreads();
  uint64_t w = 0;
  if (act) {
    uint64_t e = g.rank;
    w = g.wbefore;
    for (uint32_t v = 0; v < wv; ++v) {   // the block's earlier waves' keys of this owner
      e += s_e[v][ow];
      w += s_w[v][ow];
    }
    const uint64_t bo = boff[uint64_t(ow) * nblk + blockIdx.x];
    const uint64_t seg_w = boff[uint64_t(ow) * nblk] & 0xFFFFFFFFull;   // owner's word segment
    e += bo >> 32;
    w += bo & 0xFFFFFFFFull;
    (void)gbase;   // the receive order is the global order: no pair index travels
    // the key's words travel and its hashes do not: the owner recomputes
    // them from the words (key_hashes), 8 B of header per key instead of 24
    hdr[kHdrWords * e] = uint64_t(k) << 40 | (w - seg_w);   // offset in the owner's words
    send_q[e] = uint32_t(q);
    if (!coop) {   // (SMASH_COOP_COPY=0: one key per lane, the round-3 form)
      const uint64_t *src = hits.row(q, int32_t(k));
      for (uint32_t i = 0; i < k; ++i) words[w + i] = src[i];
    }
  }
  if (!coop) return;
  // the keys' words, the wave together: word t of the wave's concatenated
  // key lists (lane order) is word t - pre(l) of lane l's key, so
  // consecutive lanes store consecutive words of an owner's segment (a
  // lane-per-key loop stores 64 scattered words per instruction)
  const uint32_t lane = threadIdx.x & 63;
  uint32_t incl = k;   // inclusive scan of the word counts over the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= uint32_t(d)) incl += y;
  }
  const uint32_t total = __shfl(incl, 63, 64);
  const uint64_t row = act ? reinterpret_cast<uint64_t>(hits.row(q, int32_t(k))) : 0ull;
  for (uint32_t t0 = 0; t0 < total; t0 += 64) {   // (wave-uniform: every shuffle has all lanes)
    const uint32_t t = t0 + lane;
    // the lane whose key holds word t: the first l with incl(l) > t
    uint32_t l = 0;
#pragma unroll
    for (uint32_t step = 32; step; step >>= 1)
      if (uint32_t(__shfl(int(incl), int(l + step - 1), 64)) <= t) l += step;
    l = l < 63u ? l : 63u;   // (t >= total: a lane past the end)
    // (the shuffle runs on every lane, outside the select: a cross-lane read
    // under a partial exec mask returns 0 from the lanes it excludes)
    const uint32_t prev = uint32_t(__shfl(int(incl), int((l + 63u) & 63u), 64));
    const uint32_t before = l ? prev : 0u;
    const uint64_t wl = __shfl(w, int(l), 64), rl = __shfl(row, int(l), 64);
    if (t < total) words[wl + (t - before)] = reinterpret_cast<const uint64_t *>(rl)[t - before];
  }
}

// the pair key's two hashes from its hit words, exactly as k_post /
// k_post_fast fold them while they build the key (a word is tid << 48 | pos0,
// pos0 < 2^48, so the | there is the ^ here)
__device__ inline void key_hashes(const uint64_t *w, uint32_t nk, uint64_t mask, uint64_t &hh,
                                  uint64_t &hl) {
  hh = 0x9E3779B97F4A7C15ull;
  hl = 0xD1B54A32D192ED03ull;
  for (uint32_t i = 0; i < nk; ++i) {
    const uint64_t x = w[i];
    hh = mix64(hh ^ x) + 0x632BE59BD9B4E019ull;
    hl = mix64(hl + x * 0x9E3779B97F4A7C15ull) ^ (hl >> 29);
  }
  hh = (mix64(hh ^ uint64_t(nk)) & mask) | 1;
  hl = (mix64(hl + uint64_t(nk)) & mask) | 1;
}

// base[0..world]: header prefix per source rank; base[65..65+world]: word
// prefix per source rank.  hi: the key's hash hi (recomputed, like .lo)
__device__ __forceinline__ KeyRef recv_key(const uint64_t *recv, const uint64_t *words,
                                           const uint64_t *base, int world, uint64_t j,
                                           uint64_t hmask, uint64_t *hi = nullptr) {
  int r = 0;
  while (r + 1 < world && j >= base[r + 1]) ++r;
  const uint64_t nw = recv[kHdrWords * j];
  KeyRef k{words + base[65 + r] + (nw & kHdrOffMask), uint32_t(nw >> 40), 0};
  uint64_t h = 0;
  key_hashes(k.w, k.nk, hmask, h, k.lo);
  if (hi) *hi = h;
  return k;
}

// The owner's first-wins decision, the single-GPU claim / decide scheme
// (k_dedup_claim / k_dedup_decide) over the received keys: key j claims an
// empty slot with ref = epoch << 40 | (j + 1), or lowers a same-key claim of
// this launch with atomicMin (the receive order is the global pair order, so
// the smallest j is the first pair), or finds the key published by an
// earlier launch (a duplicate).  k_owner_decide: j is kept iff the slot still
// holds its own claim; the winner writes the record and publishes it.
__global__ void k_owner_claim(const uint64_t *recv, const uint64_t *words, const uint64_t *base,
                              int world, uint64_t n, uint64_t *table, uint64_t mask,
                              const uint64_t *arena, uint64_t epoch, uint64_t *slot_of,
                              unsigned long long *stats, uint64_t hmask) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  int32_t err = 0;
  for (uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; j < n; j += stride) {
    uint64_t hi = 0;
    const KeyRef me = recv_key(recv, words, base, world, j, hmask, &hi);
    const unsigned long long mine = (epoch << kRefShift) | (j + 1);
    uint64_t res = kSlotNone;
    uint64_t i = (hi ^ (hi >> 31)) & mask;
    uint32_t waits = 0;
    for (uint64_t probe = 0; probe <= mask;) {
      unsigned long long *sh = reinterpret_cast<unsigned long long *>(&table[2 * i]);
      unsigned long long *sr = sh + 1;
      unsigned long long cur = __hip_atomic_load(sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == 0) {
        const unsigned long long prev = atomicCAS(sh, 0ull, (unsigned long long)hi);
        if (prev == 0) {
          __hip_atomic_store(sr, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          res = i;
          break;
        }
        cur = prev;
      }
      if (cur == hi) {
        const unsigned long long ref =
            __hip_atomic_load(sr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ref == 0) {   // the claimer is between its CAS and its ref store (k_dedup_claim)
          if (++waits > (1u << 22)) {
            err = SMASH_ERR_UNSUPPORTED;
            break;
          }
          continue;
        }
        if (ref & kRefPub) {
          if ((ref >> kRefShift) != epoch &&
              same_key(arena + ((ref & (kRefPub - 1)) - 1), me)) {
            res = kSlotOld;
            break;
          }
        } else if ((ref >> kRefShift) == epoch) {
          const uint64_t j2 = (ref & (kRefPub - 1)) - 1;
          if (same_key(me, recv_key(recv, words, base, world, j2, hmask))) {
            atomicMin(sr, mine);
            res = i;
            break;
          }
        }
      }
      ++probe;
      i = (i + 1) & mask;
    }
    if (res == kSlotNone && err == 0) err = SMASH_ERR_NOMEM;   // the set is full
    slot_of[j] = res;
  }
  if (err) atomicCAS(&stats[S_ERR], 0ull, (unsigned long long)(unsigned)err);
}

__global__ void k_owner_decide(const uint64_t *recv, const uint64_t *words, const uint64_t *base,
                               int world, uint64_t n, uint64_t *table, uint64_t *arena,
                               uint64_t arena_cap, unsigned long long *arena_top, uint64_t epoch,
                               const uint64_t *__restrict__ slot_of, uint8_t *flags,
                               unsigned long long *stats, bool coop, uint64_t hmask) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  bool full = false;
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t c0 = (uint64_t(blockIdx.x) * blockDim.x + (threadIdx.x & ~63u)) * kDecGroups;
       c0 < n; c0 += stride * kDecGroups) {
    bool wins[kDecGroups];
    uint32_t needs[kDecGroups], incls[kDecGroups], tots[kDecGroups];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t g = 0; g < kDecGroups; ++g) {
      const uint64_t j = c0 + 64 * g + lane;
      bool win = false;
      uint32_t m = 0;
      if (j < n) {
        m = uint32_t(recv[kHdrWords * j] >> 40);
        const uint64_t sl = slot_of[j];
        if (sl < kSlotNone) {
          const unsigned long long ref = __hip_atomic_load(
              reinterpret_cast<unsigned long long *>(&table[2 * sl + 1]), __ATOMIC_RELAXED,
              __HIP_MEMORY_SCOPE_AGENT);
          win = ref == ((epoch << kRefShift) | (j + 1));
        }
      }
      wins[g] = win;
      needs[g] = win ? 2u + m : 0u;
      incls[g] = wave_incl(needs[g], tots[g]);
      sum += tots[g];
    }
    unsigned long long wbase = 0;
    if (lane == 63 && sum) wbase = atomicAdd(arena_top, (unsigned long long)sum);
    wbase = __shfl(wbase, 63, 64);
#pragma unroll
    for (uint32_t g = 0; g < kDecGroups; ++g) {
      const uint64_t j = c0 + 64 * g + lane;
      const bool win = wins[g];
      const uint32_t need = needs[g], incl = incls[g], total = tots[g];
      const uint32_t m = win ? need - 2u : 0u;
      const uint64_t off = uint64_t(wbase) + incl - need;
      wbase += total;
      const bool ok = win && off + need <= arena_cap;
      KeyRef me{words, 0u, 0ull};
      if (win) me = recv_key(recv, words, base, world, j, hmask);
      wave_fill_records(arena, off, incl, total, ok, me.lo, win ? m : 0u, me.w, coop);
      if (win) {
        if (!ok) {
          full = true;   // the slot stays a claim: never matched (no kRefPub)
        } else {
          __hip_atomic_store(reinterpret_cast<unsigned long long *>(&table[2 * slot_of[j] + 1]),
                             (unsigned long long)((epoch << kRefShift) | kRefPub | (off + 1)),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (j < n) flags[j] = win ? 1 : 0;
    }
  }
  if (full) atomicCAS(&stats[S_ERR], 0ull, (unsigned long long)(unsigned)SMASH_ERR_NOMEM);
}
__global__ void k_import(const uint8_t *flags, const uint32_t *send_q, uint64_t n_export,
                         uint8_t *keep) {
  const uint64_t o = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (o < n_export) keep[send_q[o]] = flags[o];
}
__global__ void k_import_stats(const uint8_t *keep, const int32_t *nk, uint64_t n,
                               unsigned long long *stats) {
  const uint64_t q = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const bool keyed = q < n && nk[q] >= 0;
  // the wave's sums, one atomic each on its stats row (not one per pair)
  wave_stats(stats, S_KEYPAIRS, keyed ? 1ull : 0ull, S_DUPEPAIRS,
             keyed && !keep[q] ? 1ull : 0ull, 0);
}
}  // namespace
}  // namespace smash

extern "C" int smash_phase_export(smash_pipeline *p, int world, uint64_t global_base,
                                  int64_t *h_send_counts, int64_t *h_send_words,
                                  const uint64_t **d_send, const uint64_t **d_send_words,
                                  void *stream) {
  if (!p || world < 1 || world > 64 || !h_send_counts || !h_send_words || !d_send ||
      !d_send_words) {
    set_error("smash_phase_export: bad arguments");
    return SMASH_ERR_ARG;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  p->last = s;
  const uint64_t n = p->n_pairs;
  const uint32_t nblk = uint32_t(std::max<uint64_t>(1, (n + kB - 1) / kB));
  SMASH_HIP(hipMemsetAsync(p->d_keep, 0, n ? n : 1, s));
  // per-owner totals to the host (the collectives' split sizes): the one
  // synchronisation of the exchange
  unsigned long long *cnt = p->h_owner;
  std::fill(cnt, cnt + 128, 0ull);
  if (n) {
    k_export_count<<<nblk, kB, 0, s>>>(p->d_nk, p->d_hash, n, world, nblk, p->d_bcnt);
    size_t tb = p->scan_temp_bytes;
    SMASH_HIP(hipcub::DeviceScan::ExclusiveSum(p->d_scan_temp, tb, p->d_bcnt, p->d_boff,
                                               uint64_t(world) * nblk, s));
    k_export_totals<<<1, 64, 0, s>>>(p->d_bcnt, p->d_boff, world, nblk, p->d_owner);
    SMASH_HIP(hipGetLastError());
    SMASH_HIP(hipMemcpyAsync(cnt, p->d_owner, 8 * 128, hipMemcpyDeviceToHost, s));
    SMASH_HIP(hipStreamSynchronize(s));
  }
  uint64_t tot = 0, wtot = 0;
  for (int r = 0; r < world; ++r) {
    tot += cnt[r];
    wtot += cnt[64 + r];
    h_send_counts[r] = int64_t(cnt[r]);
    h_send_words[r] = int64_t(cnt[64 + r]);
  }
  p->n_export = tot;
  if (wtot > p->send_words_cap) {   // (the stream is synchronised above)
    if (p->d_send_words) SMASH_HIP(hipFree(p->d_send_words));
    p->send_words_cap = wtot + wtot / 4 + 1024;
    SMASH_HIP(hipMalloc(&p->d_send_words, 8 * p->send_words_cap));
  }
  if (n)
    k_export_fill<<<nblk, kB, 0, s>>>(p->d_nk, p->d_hash, hit_rows(p), n, world, nblk,
                                      global_base, p->d_boff, p->d_send_hdr, p->d_send_words,
                                      p->d_send_q, (p->coop_copy & 1u) != 0);
  SMASH_HIP(hipGetLastError());
  *d_send = p->d_send_hdr;
  *d_send_words = p->d_send_words;
  return SMASH_OK;
}

extern "C" int smash_dedup_owner(smash_pipeline *p, const uint64_t *d_recv, uint64_t n_recv,
                                 const uint64_t *d_recv_words, const int64_t *h_recv_counts,
                                 const int64_t *h_recv_words, int world, uint8_t *d_flags,
                                 void *stream) {
  if (!p || world < 1 || world > 64 || !h_recv_counts || !h_recv_words ||
      (n_recv && (!d_recv || !d_flags))) {
    set_error("smash_dedup_owner: bad arguments");
    return SMASH_ERR_ARG;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  SMASH_HIP(hipEventSynchronize(p->ev_base));   // (the last upload of the image read it)
  uint64_t *base = p->h_recv_base;
  std::fill(base, base + 2 * 65, uint64_t(0));
  uint64_t hs = 0, ws = 0;
  for (int r = 0; r < world; ++r) {
    base[r] = hs;
    base[65 + r] = ws;
    hs += uint64_t(h_recv_counts[r]);
    ws += uint64_t(h_recv_words[r]);
  }
  if (hs != n_recv || (ws && !d_recv_words)) {
    set_error("smash_dedup_owner: per-source counts do not add up to n_recv");
    return SMASH_ERR_ARG;
  }
  base[world] = hs;
  base[65 + world] = ws;
  p->last = s;
  if (!n_recv) return SMASH_OK;
  if (n_recv > p->oslot_cap) {   // the claims' slot per received key
    SMASH_HIP(hipStreamSynchronize(s));
    if (p->d_oslot) SMASH_HIP(hipFree(p->d_oslot));
    p->oslot_cap = n_recv + n_recv / 4 + 1024;
    SMASH_HIP(hipMalloc(reinterpret_cast<void **>(&p->d_oslot), 8 * p->oslot_cap));
  }
  SMASH_HIP(hipMemcpyAsync(p->d_recv_base, base, 8 * 2 * 65, hipMemcpyHostToDevice, s));
  SMASH_HIP(hipEventRecord(p->ev_base, s));
  const uint64_t epoch = next_epoch(p);
  k_owner_claim<<<grid_for(n_recv, kB, 8192), kB, 0, s>>>(
      d_recv, d_recv_words, p->d_recv_base, world, n_recv, p->d_table, p->table_mask, p->d_arena,
      epoch, p->d_oslot, p->d_stats, p->hash_mask);
  SMASH_HIP(hipGetLastError());
  k_owner_decide<<<grid_for((n_recv + kDecGroups - 1) / kDecGroups, kB, 8192), kB, 0, s>>>(
      d_recv, d_recv_words, p->d_recv_base, world, n_recv, p->d_table, p->d_arena, p->arena_cap,
      p->d_arena_top, epoch, p->d_oslot, d_flags, p->d_stats, (p->coop_copy & 4u) != 0,
      p->hash_mask);
  SMASH_HIP(hipGetLastError());
  return SMASH_OK;
}

extern "C" int smash_phase_import(smash_pipeline *p, const uint8_t *d_flags_back,
                                  void *stream) {
  if (!p) return SMASH_ERR_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  p->last = s;
  if (p->n_export)
    k_import<<<grid_for(p->n_export, kB, 1u << 30), kB, 0, s>>>(d_flags_back, p->d_send_q,
                                                               p->n_export, p->d_keep);
  if (p->n_pairs)
    k_import_stats<<<grid_for(p->n_pairs, kB, 1u << 30), kB, 0, s>>>(p->d_keep, p->d_nk,
                                                                    p->n_pairs, p->d_stats);
  SMASH_HIP(hipGetLastError());
  return SMASH_OK;
}

extern "C" int smash_pipeline_error(smash_pipeline *p, void *stream, int32_t *err) {
  if (!p || !err) return SMASH_ERR_ARG;
  SMASH_HIP(hipSetDevice(p->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  // (the owner counts' pinned image is free here: phase_export has read it)
  SMASH_HIP(hipMemcpyAsync(p->h_owner + 192, p->d_stats + S_ERR, 8, hipMemcpyDeviceToHost, s));
  SMASH_HIP(hipStreamSynchronize(s));
  *err = int32_t(p->h_owner[192]);
  return SMASH_OK;
}

extern "C" int smash_pipeline_stats(smash_pipeline *p, smash_stats *o) {
  if (!p || !o) return SMASH_ERR_ARG;
  SMASH_HIP(hipSetDevice(p->device));
  if (p->last) SMASH_HIP(hipStreamSynchronize(p->last));
  SMASH_HIP(hipDeviceSynchronize());
  if (int rc = probe_check(p->ix)) return rc;   // k_mam_sm's sticky probe check
  unsigned long long rows[kStatWords], st[S_N] = {0};
  SMASH_HIP(hipMemcpy(rows, p->d_stats, sizeof(rows), hipMemcpyDeviceToHost));
  for (uint32_t r = 0; r < kStatStripes; ++r)
    for (int k = 0; k < S_N; ++k)
      if (k != S_ERR) st[k] += rows[r * kStatStride + k];
  st[S_ERR] = rows[S_ERR];
  o->pairs = st[S_PAIRS];
  o->key_pairs = st[S_KEYPAIRS];
  o->dupe_pairs = st[S_DUPEPAIRS];
  o->positions = st[S_POS];
  o->dups = st[S_DUPS];
  o->kept = st[S_KEPT];
  o->matches = st[S_MATCHES];
  o->error = int32_t(st[S_ERR]);
  return SMASH_OK;
}

extern "C" int smash_pipeline_peek(smash_pipeline *p, int32_t *h_nk, uint8_t *h_keep,
                                   uint64_t *h_hits, uint64_t *h_hash) {
  if (!p) return SMASH_ERR_ARG;
  SMASH_HIP(hipSetDevice(p->device));
  SMASH_HIP(hipDeviceSynchronize());
  const uint64_t n = p->n_pairs;
  if (!n) return SMASH_OK;
  if (h_nk) SMASH_HIP(hipMemcpy(h_nk, p->d_nk, 4 * n, hipMemcpyDeviceToHost));
  if (h_keep) SMASH_HIP(hipMemcpy(h_keep, p->d_keep, n, hipMemcpyDeviceToHost));
  if (h_hits) {
    // the ABI's layout, [n][2 * slots] words: the full rows, with the pairs
    // whose hits live in their dense head rows (HitRows) copied in
    const uint64_t W = 2 * uint64_t(p->slots);
    SMASH_HIP(hipMemcpy(h_hits, p->d_hits, 8 * n * W, hipMemcpyDeviceToHost));
    std::vector<int32_t> nk(n);
    std::vector<uint64_t> head(n * smash::kHitHead);
    SMASH_HIP(hipMemcpy(nk.data(), p->d_nk, 4 * n, hipMemcpyDeviceToHost));
    SMASH_HIP(hipMemcpy(head.data(), p->d_hhead, 8 * n * smash::kHitHead, hipMemcpyDeviceToHost));
    for (uint64_t q = 0; q < n; ++q)
      if (nk[q] > 0 && nk[q] <= int32_t(smash::kHitHead))
        std::memcpy(h_hits + q * W, head.data() + q * smash::kHitHead, 8 * size_t(nk[q]));
  }
  if (h_hash) SMASH_HIP(hipMemcpy(h_hash, p->d_hash, 16 * n, hipMemcpyDeviceToHost));
  return SMASH_OK;
}

// Growth of a set that holds keys: every occupied slot {hash hi, ref} of the
// old table moves to the first empty slot of its probe sequence in the new
// one (the claim kernels' (hi ^ hi >> 31) & mask, linear).  Between batches
// every ref is published (an arena offset, copied with the arena), so the
// keys, their records and the first-wins decisions stay as they were; two
// keys with one hi take two slots, as they did.
__global__ void k_rehash(const uint64_t *__restrict__ old, uint64_t old_slots, uint64_t *nt,
                         uint64_t mask) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < old_slots; i += stride) {
    const uint64_t hi = old[2 * i];
    if (!hi) continue;
    uint64_t j = (hi ^ (hi >> 31)) & mask;
    for (uint64_t probe = 0; probe <= mask; ++probe, j = (j + 1) & mask) {
      unsigned long long *sh = reinterpret_cast<unsigned long long *>(&nt[2 * j]);
      if (atomicCAS(sh, 0ull, (unsigned long long)hi) == 0ull) {
        nt[2 * j + 1] = old[2 * i + 1];
        break;
      }
    }
  }
}

extern "C" int smash_pipeline_reserve_keys(smash_pipeline *p, uint64_t keys, void *stream) {
  if (!p) return SMASH_ERR_ARG;
  uint64_t slots = 0, words = 0;
  key_set_geometry(keys, p->max_pairs, &slots, &words);
  slots = std::max<uint64_t>(slots, p->table_mask + 1);
  words = std::max<uint64_t>(words, p->arena_cap);
  if (slots <= p->table_mask + 1 && words <= p->arena_cap) return SMASH_OK;
  SMASH_HIP(hipSetDevice(p->device));
  SMASH_HIP(hipDeviceSynchronize());   // (no kernel may hold the old set)
  unsigned long long top = 0;
  SMASH_HIP(hipMemcpy(&top, p->d_arena_top, 8, hipMemcpyDeviceToHost));
  uint64_t *t = nullptr, *a = nullptr;
  if (hipMalloc(reinterpret_cast<void **>(&t), 16 * slots) != hipSuccess ||
      hipMalloc(reinterpret_cast<void **>(&a), 8 * words) != hipSuccess) {
    (void)hipFree(t);
    set_error("smash_pipeline_reserve_keys: out of device memory for " + std::to_string(keys) +
              " keys");
    return SMASH_ERR_NOMEM;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  SMASH_HIP(hipMemsetAsync(t, 0, 16 * slots, s));
  if (top) {   // the keys move: arena words as they are, slots rehashed
    SMASH_HIP(hipMemcpyAsync(a, p->d_arena, 8 * std::min<uint64_t>(top, p->arena_cap),
                             hipMemcpyDeviceToDevice, s));
    const uint64_t old_slots = p->table_mask + 1;
    k_rehash<<<grid_for(old_slots, 256, 1u << 16), 256, 0, s>>>(p->d_table, old_slots, t, slots - 1);
    SMASH_HIP(hipGetLastError());
  }
  SMASH_HIP(hipStreamSynchronize(s));
  SMASH_HIP(hipFree(p->d_table));
  SMASH_HIP(hipFree(p->d_arena));
  p->d_table = t;
  p->d_arena = a;
  p->table_mask = slots - 1;
  p->arena_cap = words;
  return SMASH_OK;
}

namespace smash {
// the single-GPU set must take the next n_next pairs' keys: grow it (at
// least doubling) when the keys so far plus those could overflow it
int ensure_keys(smash_pipeline *p, uint64_t n_next, hipStream_t s) {
  const uint64_t need = p->keys_bound + n_next, cap = smash_pipeline_key_capacity(p);
  if (need <= cap) return SMASH_OK;
  return smash_pipeline_reserve_keys(p, std::max(need, 2 * cap), s);
}
}  // namespace smash

extern "C" uint64_t smash_pipeline_key_capacity(const smash_pipeline *p) {
  // keys the set takes for sure: half its slots, and 16 words of arena each
  return p ? std::min<uint64_t>((p->table_mask + 1) / 2, p->arena_cap / 16) : 0;
}

extern "C" int smash_pipeline_map_hints(const smash_pipeline *p) { return p && p->mhint ? 1 : 0; }

extern "C" int smash_pipeline_reset_ex(smash_pipeline *p, uint32_t flags, void *stream) {
  if (!p || (flags & ~uint32_t(SMASH_RESET_KEEP_SEARCH))) return SMASH_ERR_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  SMASH_HIP(hipSetDevice(p->device));
  SMASH_HIP(hipMemsetAsync(p->d_table, 0, 16 * (p->table_mask + 1), s));
  SMASH_HIP(hipMemsetAsync(p->d_arena_top, 0, 8, s));
  p->keys_bound = 0;
  SMASH_HIP(hipMemsetAsync(p->d_stats, 0, 8 * kStatWords, s));
  k_reset_prev<<<1, 1, 0, s>>>(p->d_prev);   // no host source: stays asynchronous
  SMASH_HIP(hipGetLastError());
  // a look-ahead search not consumed before the reset is dropped (the next
  // phase_map searches its reads again; its set stays busy until ev_found)
  // unless the caller keeps it: it read only the reads and the index, and
  // its post stage, which writes the stats and the keys, runs in the new run
  if (!(flags & SMASH_RESET_KEEP_SEARCH))
    for (int k = 0; k < 2; ++k) {
      p->searched[k] = false;
      p->pref_reads[k] = nullptr;
      p->pref_n[k] = 0;
    }
  return SMASH_OK;
}

extern "C" int smash_pipeline_reset(smash_pipeline *p, void *stream) {
  return smash_pipeline_reset_ex(p, 0, stream);
}

extern "C" int smash_pipeline_reads_resident(smash_pipeline *p, int on) {
  if (!p) return SMASH_ERR_ARG;
  p->reads_resident = on != 0;
  return SMASH_OK;
}

extern "C" int smash_pipeline_profile(smash_pipeline *p, int enable) {
  if (!p) return SMASH_ERR_ARG;
  p->prof = enable != 0;
  p->n_ev = 0;
  p->prof_reads = 0;
  return SMASH_OK;
}

extern "C" int smash_pipeline_profile_read(smash_pipeline *p, double *search_ms,
                                           uint64_t *launches, uint64_t *reads) {
  if (!p) return SMASH_ERR_ARG;
  SMASH_HIP(hipSetDevice(p->device));
  double ms = 0;
  for (uint64_t i = 0; i < p->n_ev; ++i) {
    SMASH_HIP(hipEventSynchronize(p->ev[2 * i + 1]));
    float t = 0;
    SMASH_HIP(hipEventElapsedTime(&t, p->ev[2 * i], p->ev[2 * i + 1]));
    ms += t;
  }
  if (search_ms) *search_ms = ms;
  if (launches) *launches = p->n_ev;
  if (reads) *reads = p->prof_reads;
  return SMASH_OK;
}

extern "C" int smash_pipeline_profile_intervals(smash_pipeline *p, double *h_ms, uint64_t cap,
                                                uint64_t *n) {
  if (!p || !n || (cap && !h_ms)) return SMASH_ERR_ARG;
  SMASH_HIP(hipSetDevice(p->device));
  *n = p->n_ev;
  for (uint64_t i = 0; i < p->n_ev && i < cap; ++i) {
    SMASH_HIP(hipEventSynchronize(p->ev[2 * i + 1]));
    float a = 0, b = 0;
    SMASH_HIP(hipEventElapsedTime(&a, p->ev[0], p->ev[2 * i]));
    SMASH_HIP(hipEventElapsedTime(&b, p->ev[0], p->ev[2 * i + 1]));
    h_ms[2 * i] = a;
    h_ms[2 * i + 1] = b;
  }
  return SMASH_OK;
}

// The time at least one profiled k_mam_sm launch was running: the union of
// the launches' [start, end] event intervals (launches on the two search
// streams overlap, so their summed durations count the overlap twice).
extern "C" int smash_pipeline_profile_active(smash_pipeline *p, double *active_ms) {
  if (!p || !active_ms) return SMASH_ERR_ARG;
  SMASH_HIP(hipSetDevice(p->device));
  std::vector<std::pair<double, double>> iv;
  for (uint64_t i = 0; i < p->n_ev; ++i) {
    SMASH_HIP(hipEventSynchronize(p->ev[2 * i + 1]));
    float a = 0, b = 0;
    SMASH_HIP(hipEventElapsedTime(&a, p->ev[0], p->ev[2 * i]));
    SMASH_HIP(hipEventElapsedTime(&b, p->ev[0], p->ev[2 * i + 1]));
    iv.emplace_back(a, b);
  }
  std::sort(iv.begin(), iv.end());
  double tot = 0, cs = 0, ce = -1e300;
  for (const auto &x : iv) {
    if (x.first > ce) {
      if (ce > cs) tot += ce - cs;
      cs = x.first;
      ce = x.second;
    } else if (x.second > ce) {
      ce = x.second;
    }
  }
  if (!iv.empty() && ce > cs) tot += ce - cs;
  *active_ms = tot;
  return SMASH_OK;
}

// The positions the last batch emitted (the awk/perl output of
// smash_mapping.sh:29 that varbin.py reads): pos0 and absolute position, in
// emission order.  Synchronises.
extern "C" int smash_pipeline_positions(smash_pipeline *p, int64_t *h_pos0, int64_t *h_abspos,
                                        uint64_t cap, uint64_t *n_out) {
  if (!p || !n_out) return SMASH_ERR_ARG;
  SMASH_HIP(hipSetDevice(p->device));
  if (p->pos_dirty && p->n_pairs) {   // fused path: write the last batch's positions now
    SMASH_HIP(ensure_positions(p));
    k_emit<<<grid_for(p->n_pairs, kB, 1u << 30), kB, 0, p->last>>>(
        p->d_keep, p->d_nk, hit_rows(p), p->d_posoff, p->n_pairs, p->d_chrom_off,
        p->d_pos0, p->d_abs);
    SMASH_HIP(hipGetLastError());
    p->pos_dirty = false;
  }
  if (p->last) SMASH_HIP(hipStreamSynchronize(p->last));
  uint32_t n = 0;
  if (p->n_pairs)
    SMASH_HIP(hipMemcpy(&n, p->d_posoff + p->n_pairs, 4, hipMemcpyDeviceToHost));
  *n_out = n;
  const uint64_t k = n < cap ? n : cap;
  if (k && h_pos0) SMASH_HIP(hipMemcpy(h_pos0, p->d_pos0, 8 * k, hipMemcpyDeviceToHost));
  if (k && h_abspos) SMASH_HIP(hipMemcpy(h_abspos, p->d_abs, 8 * k, hipMemcpyDeviceToHost));
  return SMASH_OK;
}

// varbin.py's loop (varbin.py:52-92) over positions already filtered to
// binned chromosomes (varbin.py:38-49): adjacent de-dup on pos0 against the
// previous line (prev_pos0 < 0: none), bisect_right over the bin starts,
// count.  h_stats[0..2] += TotalReads, DupsRemoved, ReadsKept.  Synchronises.
extern "C" int smash_bin_positions(const int64_t *d_pos0, const int64_t *d_abspos, uint64_t n,
                                   int64_t prev_pos0, const int64_t *d_bin_starts,
                                   uint32_t nbins, uint64_t *d_counts, uint64_t *h_stats,
                                   void *stream) {
  if ((n && (!d_pos0 || !d_abspos)) || !d_bin_starts || nbins == 0 || !d_counts || !h_stats) {
    set_error("smash_bin_positions: bad arguments");
    return SMASH_ERR_ARG;
  }
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint64_t *scratch = nullptr;   // [0] npos (u32) [1] prev [2..] stats
  SMASH_HIP(hipMallocAsync(reinterpret_cast<void **>(&scratch), 8 * (2 + S_N), s));
  SMASH_HIP(hipMemsetAsync(scratch, 0, 8 * (2 + S_N), s));
  int rc = SMASH_OK;
  for (uint64_t b = 0; b < n && rc == SMASH_OK; b += (1ull << 30)) {
    const uint64_t m = n - b < (1ull << 30) ? n - b : (1ull << 30);
    const uint32_t m32 = uint32_t(m);
    // the line before the chunk: the caller's prev_pos0, then the previous chunk's last
    const bool first = b == 0;
    if (hipMemcpyAsync(scratch, &m32, 4, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(scratch + 1, first ? static_cast<const void *>(&prev_pos0) : &d_pos0[b - 1],
                       8, first ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice,
                       s) != hipSuccess) {
      rc = SMASH_ERR_HIP;
      break;
    }
    k_bin<<<2048, kB, 0, s>>>(d_pos0 + b, d_abspos + b, reinterpret_cast<const uint32_t *>(scratch),
                              reinterpret_cast<const int64_t *>(scratch + 1), d_bin_starts, nbins,
                              nullptr, 0, 0,
                              reinterpret_cast<unsigned long long *>(d_counts),
                              reinterpret_cast<unsigned long long *>(scratch + 2));
    if (hipGetLastError() != hipSuccess) rc = SMASH_ERR_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) rc = SMASH_ERR_HIP;   // m32/prev are host locals
  }
  uint64_t st[S_N] = {0};
  if (rc == SMASH_OK && hipMemcpyAsync(st, scratch + 2, sizeof(st), hipMemcpyDeviceToHost, s) != hipSuccess)
    rc = SMASH_ERR_HIP;
  if (hipStreamSynchronize(s) != hipSuccess) rc = SMASH_ERR_HIP;
  (void)hipFree(scratch);
  if (rc != SMASH_OK) {
    set_error("smash_bin_positions: HIP error");
    return rc;
  }
  h_stats[0] += st[S_POS];
  h_stats[1] += st[S_DUPS];
  h_stats[2] += st[S_KEPT];
  return SMASH_OK;
}
