/*
 * oracle/smash_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference (yamrom/smash-paper) read -> bin-count
 * chain.  It is the CHECKER for the MI355X product path and the timed CPU
 * baseline ("port") of bench.py; it is never linked into the product
 * (smash-paper_amd/), which fails loudly without its HIP library.
 *
 * Parity pin: tests/test_oracle_golden.py checks every function here against
 * golden vectors produced by the compiled UPSTREAM binaries (oracle/_ref, built
 * from /root/reference by oracle/Makefile) and the upstream varbin.py run under
 * python3 (tools/make_golden.sh).  smashMEM.py could not be run (pysam is not
 * installed and may not be fetched): orc_smash_pair() is "parity unpinned"
 * except through the reasoning in DESIGN.md and the hand-made edge cases in
 * tests/test_oracle_smash.py.
 */
#ifndef SMASH_ORACLE_H_
#define SMASH_ORACLE_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- text (fasta.cpp:139-236) ------------------------------------------ */
/* Parses a FASTA exactly like Sequence::Sequence with rcref (fasta.cpp:
 * 189-250) and returns a malloc'd text + contig tables.  Returns 0 on success.
 * startpos/sizes have 2 entries per contig (fwd, rc); names n_contig. */
typedef struct {
  uint64_t N;
  uint8_t *T;            /* N bytes + 64 bytes of zero padding */
  uint32_t n_seq;        /* 2 * n_contig */
  uint64_t *startpos;    /* [n_seq] */
  uint64_t *sizes;       /* [n_seq] */
  char **names;          /* [n_seq] (fwd and rc share the name) */
} orc_text;
int orc_text_from_fasta(const char *path, orc_text *out);
void orc_text_free(orc_text *t);

/* ---- index (longSA.cpp:94-237) ----------------------------------------- */
/* Suffix array of T[0..N) (bytes, '$' last & unique).  Prefix doubling with
 * counting sorts (NOT qsufsort): the SA of a text with a unique sentinel is
 * unique, so any correct builder reproduces rc1.i*.index.sa.bin byte for
 * byte. */
int orc_build_sa(const uint8_t *T, uint64_t N, uint64_t *SA);
void orc_build_isa(const uint64_t *SA, uint64_t N, uint64_t *ISA);
/* Kasai LCP (longSA.cpp:224-237): LCP[0]=0, LCP[r]=lcp(SA[r-1],SA[r]). */
void orc_build_lcp(const uint8_t *T, uint64_t N, const uint64_t *SA,
                   const uint64_t *ISA, uint64_t *LCP);

typedef struct {
  uint64_t N, logN;
  const uint8_t *T;
  const void *SA, *ISA;   /* idx_bytes-wide elements (ANINT, size.h:33-38) */
  uint32_t idx_bytes;     /* 4 or 8 */
  /* vec_uchar (longSA.h:18-61): u8 vector, 255 -> lower_bound in the
   * {idx, val} overflow table sorted by idx */
  const uint8_t *L8;
  const uint64_t *ovf;
  uint64_t n_ovf;
  uint32_t n_seq;
  const uint64_t *startpos, *sizes;
  /* element bits of an SA / ISA word: ~0, or 2^33 - 1 for the device's
   * packed words (smash-paper_amd/csrc/common.hpp), whose high bits hold the
   * search's hints (0 is read as ~0) */
  uint64_t pos_mask;
} orc_index;
/* logN = ceil(log(N)/log(2.0)) (longSA.cpp:97) */
uint64_t orc_logN(uint64_t N);

typedef struct { uint64_t ref, query, len; } orc_match;  /* longSA.h:78-92 */

/* Access accounting for the roofline: distinct 64-B line transitions per
 * array (BASELINE.md "B_read"), counted on the algorithm as run. */
typedef struct {
  uint64_t sa_loads, isa_loads, ref_loads, lcp_loads;
  uint64_t sa_lines, isa_lines, ref_lines, lcp_lines;
  uint64_t last_sa, last_isa, last_ref, last_lcp;
  uint64_t ovf_lookups;   /* vec_uchar overflow lower_bounds (not on the
                             device path: it compares min(LCP,255)) */
  uint64_t kt_lines, u_lines;       /* accelerated path only */
  uint64_t last_kt, last_u;
  uint64_t bm_lines, last_bm;       /* v3 bitmap */
} orc_counters;

/* Search accelerators of the device path (smash-paper_amd/csrc/
 * aux_build.hip), restated here so that the accelerated algorithm can be
 * checked on the CPU (it must emit exactly orc_mam's matches) and so that its
 * line transitions can be counted for the roofline:
 *   U[x]  = min(255, max(LCP[ISA[x]], LCP[ISA[x]+1]))    (N + 64 bytes)
 *   KT[w] = {lo, hi} SA interval of ACGT k-mer w, lo > hi if absent. */
typedef struct {
  const uint8_t *U;
  const uint64_t *KT;
  uint32_t K;
  /* v3: presence bitmap of every ACGT B-mer of the text (bit code(w)), and
   * the set of bytes occurring in the text */
  const uint64_t *BM;
  uint32_t B;
  uint8_t in_text[256];
} orc_accel;
uint32_t orc_accel_b(uint64_t N);
/* BM must hold 4^B bits (zeroed by the callee) */
void orc_build_bitmap(const orc_index *ix, uint32_t B, uint64_t *BM, uint8_t *in_text);
/* v3 search: positions evaluated independently (MAM output is a function of
 * the per-position matching statistics); same matches as
 * orc_mam. */
int orc_mam_v3(const orc_index *ix, const orc_accel *acc, const uint8_t *P,
               uint32_t L, uint32_t min_len, orc_match *out, uint32_t cap,
               orc_counters *ctr);
uint64_t orc_map_only_v3(const orc_index *ix, const orc_accel *acc,
                         const uint8_t *reads, uint32_t L, uint64_t stride,
                         uint64_t n, uint32_t min_len, int threads,
                         orc_counters *ctr);
uint32_t orc_accel_k(uint64_t N);
void orc_build_accel(const orc_index *ix, uint32_t K, uint8_t *U, uint64_t *KT);
/* the device's k-mer table layout (smash-paper_amd/csrc/common.hpp,
 * aux_build.hip k_kfilter): KTF[2w + i] = KT[2w + i] (low 40 bits) | presence
 * bits of the (K+2)-mers holding w (high 24 bits); KTF: 2 * 4^K words */
void orc_build_ktf(const orc_index *ix, uint32_t K, const uint64_t *KT, uint64_t *KTF);
int orc_mam_fast(const orc_index *ix, const orc_accel *acc, const uint8_t *P,
                 uint32_t L, uint32_t min_len, orc_match *out, uint32_t cap,
                 orc_counters *ctr);
uint64_t orc_map_only_fast(const orc_index *ix, const orc_accel *acc,
                           const uint8_t *reads, uint32_t L, uint64_t stride,
                           uint64_t n, uint32_t min_len, int threads,
                           orc_counters *ctr);


/* longSA::MAM (longSA.cpp:503-536).  P: lowercased read.  Returns the number
 * of matches (written up to cap). */
int orc_mam(const orc_index *ix, const uint8_t *P, uint32_t L,
            uint32_t min_len, orc_match *out, uint32_t cap, orc_counters *ctr);
/* longSA::MEM -> findMEM (longSA.cpp:395-435,587-590), bug-compatible
 * (starts at prefix 1). */
int orc_mem(const orc_index *ix, const uint8_t *P, uint32_t L,
            uint32_t min_len, orc_match *out, uint32_t cap, orc_counters *ctr);
/* mem.hip's probe sequence for the same matches (k-mer table from the root,
 * 8-byte singleton compares): the device MEM path's algorithmic lines */
int orc_mem_dev(const orc_index *ix, const orc_accel *acc, const uint8_t *P, uint32_t L,
                uint32_t min_len, orc_match *out, uint32_t cap, orc_counters *ctr);
/* MEM over n reads on `threads` threads (acc NULL: orc_mem, else orc_mem_dev);
 * per-read counts into n_out (or NULL); returns the total */
uint64_t orc_mem_batch(const orc_index *ix, const orc_accel *acc, const uint8_t *reads,
                       uint32_t L, uint64_t stride, uint64_t n, uint32_t min_len, int threads,
                       uint32_t *n_out, orc_counters *ctr);
/* longSA::MUM (longSA.cpp:549-585). */
int orc_mum(const orc_index *ix, const uint8_t *P, uint32_t L,
            uint32_t min_len, orc_match *out, uint32_t cap, orc_counters *ctr);

/* ---- hit resolution (query.cpp:68-97, 231-306) -------------------------- */
#define ORC_CIGAR_MAX 1024   /* <= 254 matches x "255=255M" */
#define ORC_MAX_MATCH 256     /* MAM/MUM matches per read: <= L - min_len + 1 <= 254 */
#define ORC_ERR_CAP 9         /* a fixed oracle capacity would be exceeded: never truncate */
typedef struct {
  uint32_t tid;          /* forward contig index = seq_index/2 */
  uint32_t rc;
  int64_t pos;           /* 0-based (SAM POS - 1) */
  int64_t qpos;          /* to_print key */
  uint32_t n_matches, n_unique, n_matched;   /* XM, XU, XE */
  uint32_t hi, nh;
  uint32_t qstart, qend; /* pysam semantics: leading S, rlen - trailing S */
  uint32_t first_off, first_len;   /* first '=' block in CIGAR walk */
  int32_t L0, R0;        /* mappability_tag.cpp:98-101 (filled by orc_tag) */
  char cigar[ORC_CIGAR_MAX];
} orc_hit;
/* Resolve + merge + order (prepare_matches with sam_out).  Returns the number
 * of printed hits (groups with n_matches > 0), in HI order; `mate_best`
 * receives (tid,pos) of the to_print-front alignment (best_alignment) or
 * tid = UINT32_MAX when the read has no match. */
int orc_resolve(const orc_index *ix, const uint8_t *P, uint32_t L,
                const orc_match *m, uint32_t n, orc_hit *out, uint32_t cap,
                uint32_t *best_tid, int64_t *best_pos);

/* ---- mappability (longSA.cpp:612-690) ----------------------------------- */
/* Writes map.bin content: 2 junk bytes (caller-chosen, byte-compared
 * separately), then [left,right] per forward base of every contig. out must
 * hold 2 + 2*sum(forward sizes).  min_lengths is recomputed per rank. */
int orc_mappability(const orc_index *ix, uint8_t *out);
/* The same bytes for forward bases [g0, g1) of the concatenated forward
 * contigs only (out: 2*(g1-g0) bytes), m[r] computed per base from the exact
 * LCP instead of an N-sized array; returns the number of those bases whose
 * k-mer is unique (1 <= right <= k) -- the C5 self-scan's restatement. */
uint64_t orc_mappability_range(const orc_index *ix, uint64_t g0, uint64_t g1,
                               uint32_t k, uint8_t *out);

/* ---- mappability_tag (mappability_tag.cpp:93-124) ----------------------- */
/* offsets: u32 sam_header offsets per tid; map: map.bin content;
 * small_chr: name contains "_gl000" or "chrM".  Fills L0/R0; returns 0, or
 * 1 / 2 for the "left/right mappability too big" throws. */
int orc_tag(orc_hit *h, const uint32_t *offsets, const uint8_t *map,
            uint64_t map_size, int small_chr);

/* ---- smashMEM.py per name (smashMEM.py:154-228), args 0 0 10000 4 -------- */
/* Input: hits of read1 / read2 in HI order (mapped only).  Output: kept hits
 * (r1 then r2, each in HI order) as (tid,pos) into out_tid/out_pos; returns
 * count, or -1 when the pair produces no key (both lists empty). */
int orc_smash_pair(const orc_hit *h1, uint32_t n1, const orc_hit *h2,
                   uint32_t n2, int min_excess, int64_t hit_window,
                   uint32_t *out_tid, int64_t *out_pos);

/* ---- varbin.py (varbin.py:6-118) ---------------------------------------- */
typedef struct {
  uint64_t total, dups, kept;
  int64_t prev_pos;      /* -1 = none; carried across calls */
} orc_varbin_state;
/* positions: (counted, pos0, abspos) already chromosome-filtered
 * (counted=0 entries are skipped).  bin_starts sorted ascending. */
void orc_varbin(const int64_t *pos0, const int64_t *abspos, uint64_t n,
                const int64_t *bin_starts, uint32_t nbins, uint64_t *counts,
                orc_varbin_state *st);

/* ---- whole chain (bench cpu_baseline + end-to-end tests) ---------------- */
typedef struct {
  const orc_index *ix;
  uint32_t min_len;
  const uint32_t *tag_offsets;   /* [n_contig] sam_header offsets */
  const uint8_t *small_chr;      /* [n_contig] */
  const uint8_t *major;          /* [n_contig] counted by perl+varbin filter */
  const int64_t *chrom_off;      /* [n_contig] chrom_sizes offset (col 3) */
  const uint8_t *map; uint64_t map_size;
  const int64_t *bin_starts; uint32_t nbins;
} orc_pipeline;
/* reads: n_pairs * 2 mates, mate k at reads + k*stride, length L, already
 * lowercased with N->z.  Runs map -> resolve -> tag -> smash -> dedup ->
 * varbin on `threads` threads for the per-pair part.  Returns 0 or the
 * first tag error code.  keys are kept in a process-global table owned by
 * `dedup` (opaque, NULL = fresh). */
typedef struct orc_dedup orc_dedup;
orc_dedup *orc_dedup_new(void);
void orc_dedup_free(orc_dedup *d);
int orc_run_pairs(const orc_pipeline *p, const uint8_t *reads, uint32_t L,
                  uint64_t stride, uint64_t n_pairs, int threads,
                  orc_dedup *dedup, uint64_t *counts, orc_varbin_state *st,
                  uint64_t *n_dupe_pairs, uint64_t *n_pos_out);
/* MAM only, over n reads on `threads` threads: returns total matches;
 * ctr (optional) sums line transitions. */
uint64_t orc_map_only(const orc_index *ix, const uint8_t *reads, uint32_t L,
                      uint64_t stride, uint64_t n, uint32_t min_len,
                      int threads, orc_counters *ctr);

#ifdef __cplusplus
}
#endif
#endif
