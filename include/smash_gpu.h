/*
 * include/smash_gpu.h -- C ABI of the MI355X-native SMASH read -> bin-count
 * path (libsmashgpu.so, built from the HIP sources in smash-paper_amd/csrc/
 * for gfx950).
 *
 * The reference has no FFI: its seams are in-process C++ calls and files.
 * Each entry point below names the reference interface it replaces.
 *
 * Conventions: plain pointers and sizes; `d_` = device pointer (HBM of the
 * handle's device), `h_` = host pointer; int status codes (SMASH_OK = 0),
 * never exceptions across the ABI; caller-owned output buffers; one handle
 * per device; an index is immutable after creation; streams are
 * hipStream_t passed as void* (0 = default stream); no global state.
 */
#ifndef SMASH_GPU_H_
#define SMASH_GPU_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes -------------------------------------------------------- */
#define SMASH_OK 0
#define SMASH_ERR_ARG (-1)       /* bad argument / shape */
#define SMASH_ERR_HIP (-2)       /* HIP runtime error (message: smash_last_error) */
#define SMASH_ERR_IO (-3)        /* file missing / unreadable / inconsistent */
#define SMASH_ERR_NOMEM (-4)     /* device allocation failed; as a pipeline data
                                    error: the de-dup key set is full */
#define SMASH_ERR_UNSUPPORTED (-5)
/* pipeline data errors (positive), reported by smash_pipeline_stats:        */
#define SMASH_ERR_TAG_LEFT 1     /* "left mappability too big"  mappability_tag.cpp:107-111 */
#define SMASH_ERR_TAG_RIGHT 2    /* "right mappability too big" mappability_tag.cpp:112-113 */

const char *smash_last_error(void);   /* thread-local text of the last error */

/* ---- reference text (Sequence::Sequence, fasta.cpp:133-285) -------------- */
/* Parses a FASTA exactly like the reference with -rcref (lowercase, '`'
 * separators, reverse complements, final '$') into malloc'd host arrays:
 * text[N], startpos/sizes[n_seq], names[n_seq] (2 entries per contig).
 * Free with smash_text_free. */
int smash_text_from_fasta(const char *path, uint8_t **text, uint64_t *N,
                          uint32_t *n_seq, uint64_t **startpos,
                          uint64_t **sizes, char ***names);
/* The same with the layout chosen: rcref = 1 as above; rcref = 0 the
 * forward-only text of `mummer` without -rcref (fasta.cpp:160-169:
 * c1 ` c2 ` ... cn $, one entry per contig). */
int smash_text_from_fasta_layout(const char *path, int rcref, uint8_t **text, uint64_t *N,
                                 uint32_t *n_seq, uint64_t **startpos, uint64_t **sizes,
                                 char ***names);
void smash_text_free(uint8_t *text, uint32_t n_seq, uint64_t *startpos,
                     uint64_t *sizes, char **names);

/* ---- search modes (query.h:126 mum_t) ------------------------------------ */
#define SMASH_MODE_MAM 1         /* -mumreference / default (longSA.cpp:503) */
#define SMASH_MODE_MAM_PLAIN 2   /* same matches, the reference's probe
                                    sequence without the accelerators (A/B) */
#define SMASH_MODE_MUM 3         /* -mum: MAM, then cleanMUMcand per read
                                    (longSA::MUM, longSA.cpp:549-585) */
#define SMASH_MODE_MEM 4         /* -maxmatch: longSA::MEM / findMEM
                                    (longSA.cpp:395-490, 587-590); only via
                                    smash_match_batch (lengths may exceed 255) */

/* ========================================================================== */
/* Index: replaces longSA::longSA (longSA.cpp:94-210) + Sequence (fasta.cpp)  */
/* ========================================================================== */
typedef struct smash_index smash_index;

/* Build the whole index ON THE DEVICE from the doubled text (layout of
 * fasta.cpp:189-247: c1 ` rc(c1) ` c2 ... rc(cn) $): suffix array (GPU prefix
 * doubling, byte-identical to qsufsort's since the SA of a '$'-terminated
 * text is unique), ISA, LCP (u8 saturated + exact overflow table, as
 * vec_uchar longSA.h:18-61) and map.bin (longSA::show, longSA.cpp:612-690).
 * startpos/sizes/names: 2 entries per contig (forward, reverse complement);
 * names may be NULL (only smash_index_save writes them). */
int smash_index_create(const uint8_t *h_text, uint64_t N, uint32_t n_seq,
                       const uint64_t *h_startpos, const uint64_t *h_sizes,
                       const char *const *names, int device,
                       smash_index **out);

/* Load the reference's on-disk cache <fasta>.bin/rc1.ref.{bin,seq.bin} and
 * rc1.i{4,8}.index.{bin,sa.bin,isa.bin,lcp.vec.bin,lcp.m.bin} (longSA.cpp:
 * 100-136, fasta.cpp:150-181) and, if present, <fasta>.bin/map.bin; the
 * map is computed on the device otherwise.  Replaces the mmap path of
 * util.cpp:100-125. */
int smash_index_load(const char *fasta_path, int device, smash_index **out);

/* Either text layout (Sequence/longSA with ref.rcref = rcref): rcref = 0
 * takes the forward-only text (one entry per contig, any n_seq) and the
 * rc0.* cache files (fasta.cpp:98, longSA.cpp:103).  Such an index has no
 * map.bin (-mappability requires -rcref, mummer.cpp:145): it serves
 * smash_map_batch / smash_match_batch / smash_sam_records* (mummer without
 * -rcref) and is refused by smash_pipeline_create and
 * smash_mappability_scan, whose SMASH chain always passes -rcref. */
int smash_index_create_layout(const uint8_t *h_text, uint64_t N, uint32_t n_seq,
                              const uint64_t *h_startpos, const uint64_t *h_sizes,
                              const char *const *names, int rcref, int device,
                              smash_index **out);
int smash_index_load_layout(const char *fasta_path, int rcref, int device, smash_index **out);

/* Write the reference's on-disk cache (rc1.i4 when N <= INT32_MAX-100000 as
 * `mummer` would, else rc1.i8, mummer.cpp:156-183) + map.bin
 * (index_setup.sh:19-22).  fasta_size is stored in the headers
 * (longSA.cpp:182, fasta.cpp:265). */
int smash_index_save(const smash_index *ix, const char *fasta_path,
                     uint64_t fasta_size);

void smash_index_free(smash_index *ix);

typedef struct {
  uint64_t N;              /* doubled text length incl. '$' */
  uint64_t logN;           /* ceil(log2 N) (longSA.cpp:97) */
  uint32_t idx_bytes;      /* 4 or 8: SA/ISA element width in HBM */
  uint32_t n_seq;
  uint64_t n_lcp_overflow; /* entries with LCP >= 255 */
  uint64_t map_bytes;      /* 2 + 2 * sum(forward contig sizes) */
  const uint8_t *d_text;   /* N + 64 bytes (zero padded) */
  const void *d_sa;        /* N x idx_bytes (pos_bits: positions in the low bits) */
  const void *d_isa;       /* N x idx_bytes (pos_bits: ranks in the low bits) */
  const uint8_t *d_lcp8;   /* N, min(LCP,255) */
  const uint64_t *d_lcp_ovf; /* n_lcp_overflow x {idx, val} sorted by idx */
  const uint8_t *d_map;    /* map.bin image */
  uint64_t device_bytes;   /* total HBM held by the index */
  double build_seconds;    /* wall time of create/load */
  /* search accelerators (results-preserving):           */
  uint32_t kmer_k;         /* k of the k-mer -> SA-interval table */
  const uint8_t *d_uniq;   /* U[x] = min(255, max(LCP[ISA[x]], LCP[ISA[x]+1])) */
  const uint64_t *d_kmer;  /* 4^k x 16 B: words {lo, hi} in their low 40 bits
                              (lo > hi = absent), and in their high 24 bits
                              48 presence bits of the (k+2)-mers holding the
                              k-mer: bit r1*4+r2 "w r1 r2", 16+l*4+r "l w r",
                              32+l1*4+l2 "l1 l2 w" (bit f at 40 + f % 24 of
                              word f / 24) */
  uint32_t bitmap_b;       /* B = k + 2: the window filter's B-mer length */
  const uint64_t *d_bitmap;/* NULL (round 3: the presence bits are in d_kmer) */
  uint64_t in_text[4];     /* 256-bit set of bytes occurring in the text */
  uint32_t rcref;          /* 1: c ` rc(c) layout; 0: forward only, no map.bin */
  uint32_t pos_bits;       /* 0: plain SA / ISA elements; 33: 8-byte elements
                              whose bits 33..63 hold the search's hints (DESIGN
                              section 3, packed index words): the element is
                              its low 33 bits.  smash_index_save writes plain
                              elements either way (SMASH_PACK_IDX=0 at create /
                              load: never packed) */
} smash_index_info;
int smash_index_query(const smash_index *ix, smash_index_info *out);
/* Packed index words: pack != 0 puts the search's hints
 * into the high bits of the 8-byte SA / ISA elements (what create / load do
 * by default when N < 2^33), 0 strips them.  Results never change; the
 * search reads fewer random lines with them.  A no-op for 4-byte elements.
 * Synchronous; no search may run on the index meanwhile. */
int smash_index_pack(smash_index *ix, int pack, void *stream);

/* ========================================================================== */
/* Search: replaces longSA::MAM(Aligner&) (longSA.cpp:503-536) for a batch   */
/* (mode MAM / MAM_PLAIN; MUM as longSA::MUM, longSA.cpp:549-585).            */
/* Each read's matches go to slots [i*cap_per_read, ...) as packed u64:       */
/*   bits 0-47 ref (text position), 48-55 query offset, 56-63 length          */
/* (match_t, longSA.h:78-92; reads <= 255 bp), in emission order (ascending   */
/* query offset, as process_match receives them, query.cpp:436-438).          */
/* d_n_out[i] = number of matches (written up to cap_per_read).               */
/* Reads: d_seqs + i*stride, length d_lens[i] (or `len` when d_lens==NULL),   */
/* already lowercased as NewQuery::extend does (query.cpp:125-144).           */
/* ========================================================================== */
int smash_map_batch(const smash_index *ix, int mode, uint32_t min_len,
                    const uint8_t *d_seqs, uint64_t stride,
                    const uint16_t *d_lens, uint32_t len, uint64_t n_reads,
                    uint64_t *d_out, uint32_t cap_per_read, uint32_t *d_n_out,
                    void *stream);

/* The three search modes with unpacked records (match_t, longSA.h:78-92):  */
/* mode = SMASH_MODE_MAM, _MUM or _MEM (memsam's default / -mum / -maxmatch,  */
/* mummer.cpp:77-96).  Read i's matches go to d_out[i*cap_per_read ...] in    */
/* the order longSA::MAM / MUM / MEM pass them to process_match; d_n_out[i] = */
/* how many there are (records beyond cap_per_read are counted, not written). */
/* ========================================================================== */
typedef struct {
  uint64_t ref;            /* text position (longSA.h:80) */
  uint32_t query;          /* query offset */
  uint32_t len;            /* match length */
} smash_match;
int smash_match_batch(const smash_index *ix, int mode, uint32_t min_len,
                      const uint8_t *d_seqs, uint64_t stride,
                      const uint16_t *d_lens, uint32_t len, uint64_t n_reads,
                      smash_match *d_out, uint32_t cap_per_read,
                      uint32_t *d_n_out, void *stream);

/* ========================================================================== */
/* Mappability self-scan (BASELINE config C5): replaces longSA::show ->       */
/* map.bin (longSA.cpp:612-690, `mummer -rcref -mappability`, index_setup.sh: */
/* 22) for the forward bases [begin, end) of the concatenated forward contigs */
/* (map.bin byte 2 + 2*g is base g), from the resident ISA + LCP.             */
/*  d_map_out: 2*(end-begin) bytes [left, right] per base, or NULL;           */
/*  derived counts of unique k-mers (the k-mer at a base is unique iff        */
/*  1 <= right <= k): d_contig_counts[n_seq/2] += per contig (or NULL), and,  */
/*  when d_bin_starts is given, d_bin_counts[nbins] += per bin of              */
/*  abspos = h_chrom_off[contig] + base (contigs with offset < 0 unbinned;    */
/*  bisect_right as varbin.py:89-92).  Asynchronous on `stream`.              */
/* ========================================================================== */
int smash_mappability_scan(const smash_index *ix, uint64_t begin, uint64_t end,
                           uint32_t k, uint8_t *d_map_out,
                           const int64_t *h_chrom_off,
                           const int64_t *d_bin_starts, uint32_t nbins,
                           uint64_t *d_bin_counts, uint64_t *d_contig_counts,
                           void *stream);

/* C5's own preparation from the index arrays: rebuilds, from the suffix     */
/* array and the LCP bytes (m[r] = max(LCP[r], LCP[r+1]) in rank order,       */
/* longSA.cpp:628-641, scattered to text position SA[r]), the per-position    */
/* unique lengths U -- and their directory -- that smash_mappability_scan of  */
/* the same [begin, end) reads, in place in the index (the values are the     */
/* index build's).  Three streaming partition passes (csrc/uniq_build.hip);   */
/* ~4 B per window position of scratch HBM, kept until                        */
/* smash_mappability_release.  Asynchronous on `stream`; no search or scan    */
/* may run on the index concurrently.                                         */
int smash_mappability_prepare(const smash_index *ix, uint64_t begin, uint64_t end,
                              void *stream);
/* smash_mappability_prepare keeps its scratch HBM (4 B per window position +
 * 2 GB) in the index for the next call; this frees it (synchronous). */
int smash_mappability_release(const smash_index *ix);
/* The text window [*lo, *hi) that smash_mappability_prepare(begin, end)     */
/* rebuilds (the forward and reverse-complement positions of those bases).    */
int smash_mappability_window(const smash_index *ix, uint64_t begin, uint64_t end,
                             uint64_t *lo, uint64_t *hi);

/* ========================================================================== */
/* Pipeline: prepare_matches (query.cpp:231-306) + mappability_tag           */
/* (mappability_tag.cpp:93-124) + smashMEM.py filters & global pair de-dup   */
/* (smashMEM.py:154-228) + varbin.py (varbin.py:52-92), fused per batch.      */
/* ========================================================================== */
typedef struct smash_pipeline smash_pipeline;

typedef struct {
  uint32_t min_len;          /* MAM minimum length (query.h:129: 20) */
  uint32_t read_len;         /* fixed mate length of the batches (<= 255) */
  uint64_t max_pairs;        /* batch capacity */
  uint32_t n_contig;         /* forward contigs = n_seq / 2 */
  const uint32_t *h_tag_offsets; /* [n_contig] sam_header.txt offsets (u32, chromosomes.h:169-196) */
  const uint8_t *h_small_chr;    /* [n_contig] name has "_gl000" or "chrM" (mappability_tag.cpp:82) */
  const int64_t *h_chrom_off;    /* [n_contig] chrom_sizes.txt col 3, or -1 = not binned
                                    (perl ^chr(\d+|[XY])$ smash_mapping.sh:29 + varbin.py:38-49) */
  uint32_t nbins;
  const int64_t *h_bin_starts;   /* [nbins] bins.txt col 3 (start abspos), ascending */
  int32_t min_excess;        /* smashMEM arg 5 (smash_mapping.sh:25: 4) */
  int64_t hit_window;        /* smashMEM arg 4 (10000) */
  uint64_t dedup_capacity;   /* distinct pair keys the persistent set holds
                                (exact keys: ~16 hit words per key of arena) */
  uint32_t read_stride;      /* bytes from one mate to the next in d_reads: 0 or
                                read_len (dense), or smash_read_stride(read_len):
                                the device's native rows (16-byte aligned d_reads,
                                the bytes past read_len of every row zero) -- the
                                search copies each mate straight from its row
                                instead of building a record of it first */
} smash_pipeline_cfg;

/* The native row of a mate of read_len bases (bytes; a multiple of 16). */
uint32_t smash_read_stride(uint32_t read_len);

/* The largest cfg.max_pairs smash_pipeline_create accepts for mates of
 * read_len bases: a batch's hit rows hold 2 * (read_len - min_len + 1) u64
 * per pair, and the batch's position offsets and export word prefixes are
 * 32-bit, so max_pairs * 2 * slots < 2^32 (16 393 004 pairs at 150 bp with
 * min_len 20).  0 when read_len / min_len are out of range. */
uint64_t smash_pipeline_max_batch(uint32_t read_len, uint32_t min_len);

/* SMASH_ERR_ARG for a bad configuration, max_pairs above
 * smash_pipeline_max_batch included (checked before the index is touched). */
int smash_pipeline_create(const smash_index *ix, const smash_pipeline_cfg *cfg,
                          smash_pipeline **out);
void smash_pipeline_free(smash_pipeline *p);
/* Grow the persistent pair-key set (smashMEM.py:217-228's `seen`) to hold
 * `keys` keys: a no-op when it does already; else a larger set, into which
 * the keys it holds move (their records copied, their slots rehashed), so it
 * may be called between batches; SMASH_ERR_NOMEM when HBM cannot hold it
 * (the old set is kept then).  Synchronous: it waits for the device.  The
 * multi-GPU driver sizes each owner's set from the run's pair count and the
 * owner skew of its first batch (dist.py); smash_count_fastq grows the
 * single-GPU set as its batches arrive (a gzip input's pair count is not
 * known before it is inflated). */
int smash_pipeline_reserve_keys(smash_pipeline *p, uint64_t keys, void *stream);
/* The keys the set takes for sure (a full set is SMASH_ERR_NOMEM in the
 * pipeline's statistics, never a silent cut). */
uint64_t smash_pipeline_key_capacity(const smash_pipeline *p);
/* 1 when the pipeline's searches hand the post stage each forward match's
 * right map.bin byte with the match (from the packed SA word of its row,
 * DESIGN.md section 3), so that byte is not loaded: the index is packed, its
 * map.bin was computed from it (not read from a file), and the tag offsets
 * are its contig offsets.  SMASH_MAP_HINT=0 at creation turns it off. */
int smash_pipeline_map_hints(const smash_pipeline *p);
/* The data error recorded so far (0: none; the error of smash_stats), as of
 * the work queued on `stream`: waits for that stream only (not for a search
 * running on the pipeline's own streams). */
int smash_pipeline_error(smash_pipeline *p, void *stream, int32_t *err);

/* One batch of n_pairs pairs: d_reads holds 2*n_pairs mates of cfg->read_len
 * bytes (rows of cfg->read_stride), mate 2q = read 1, 2q+1 = read 2 of pair q (Pair::run alternation,
 * query.cpp:486-505), pairs in name order (samtools sort -n).  Runs map ->
 * resolve -> tag -> filter -> de-dup (first wins, against every earlier
 * batch) -> adjacent de-dup (carried across batches) -> bin, adding into
 * d_counts[nbins] (u64).  Asynchronous on `stream`. */
int smash_count_batch(smash_pipeline *p, const uint8_t *d_reads,
                      uint64_t n_pairs, uint64_t *d_counts, void *stream);
/* n_pairs resident pairs in batches of batch_pairs (<= cfg.max_pairs), the
 * same chain and result as smash_count_batch per batch in order; the search
 * of each batch runs on one of two pipeline streams, so batch b + 1's search
 * starts under the tail of batch b's.  Asynchronous on `stream` (every batch's
 * reads must be ready by the work already on `stream`). */
int smash_count_batches(smash_pipeline *p, const uint8_t *d_reads, uint64_t n_pairs,
                        uint64_t batch_pairs, uint64_t *d_counts, void *stream);
/* smash_count_batches with the reads' readiness stated by the caller rather
 * than by the work on `stream`: `ready` is an event (hipEvent_t) after which
 * every batch's reads are complete, or NULL: they are complete already (no
 * pending writes on any stream).  The searches then wait for nothing queued on
 * `stream` -- a run's first searches start under the post stage of the run
 * queued before it (the de-dup set reset, the counts and every post-stage
 * kernel stay ordered on `stream`). */
int smash_count_batches_ready(smash_pipeline *p, const uint8_t *d_reads, uint64_t n_pairs,
                              uint64_t batch_pairs, uint64_t *d_counts, void *stream,
                              void *ready);

#define SMASH_EXPORT_HDR_WORDS 1   /* u64 words per key in smash_phase_export's d_send */

/* Multi-GPU phases (one rank per GPU; the caller runs the collectives):
 *  1. smash_phase_map      -- map/resolve/tag/filter/hash + in-batch first-wins
 *  2. smash_phase_export   -- the keyed pairs grouped by owner rank
 *                             ((hash >> 1) % world), each owner's segment in
 *                             pair order: per key a SMASH_EXPORT_HDR_WORDS-word
 *                             header {nk << 40 | word offset in its owner
 *                             segment} in *d_send (the owner recomputes the
 *                             key's hashes from its words) and the key's nk
 *                             canonical hit words (tid << 48 | pos0) in
 *                             *d_send_words (both pipeline-owned, valid until
 *                             the next export); h_send_counts[world] /
 *                             h_send_words[world] filled (synchronises)
 *     caller: all_to_all of the counts, then of d_send (1 word per key) and
 *             of d_send_words -> d_recv, d_recv_words (source-rank order)
 *  3. smash_dedup_owner    -- owner side: first-wins in receive order (source
 *                             ranks in rank order = the global pair order)
 *                             over the EXACT keys, against the persistent set;
 *                             inserts winners; one byte per received header
 *                             into d_flags (1 = keep).  h_recv_counts /
 *                             h_recv_words: per source rank (synchronises)
 *     caller: all_to_all(d_flags) back, in d_send order
 *  4. smash_phase_import   -- apply the returned flags
 *  5. smash_phase_positions-- emit kept positions; d_tail[2] = {count, last
 *                             pos0 or -1} for the adjacent-dup boundary
 *     caller: all_gather(d_tail) -> previous rank's last pos (d_prev)
 *  6. smash_phase_bin      -- adjacent de-dup against *d_prev, bin, add. */
int smash_phase_map(smash_pipeline *p, const uint8_t *d_reads, uint64_t n_pairs,
                    void *stream);
/* smash_phase_map, then the search of the NEXT batch (d_next, n_next pairs,
 * its reads ready by the work already on `stream`) issued at once on the
 * pipeline's other search stream: it runs while the caller exchanges this
 * batch's keys; the next smash_phase_map[_ahead] with the same reads uses it.
 * d_next must stay allocated and UNMODIFIED until that call: the search reads
 * it asynchronously and its result is matched by (pointer, n_next) only.
 * smash_pipeline_reset drops a look-ahead that was not consumed. */
int smash_phase_map_ahead(smash_pipeline *p, const uint8_t *d_reads, uint64_t n_pairs,
                          const uint8_t *d_next, uint64_t n_next, void *stream);
/* After smash_phase_export of batch b: the search of batch b + 2 (d_reads,
 * n_pairs) issued into the search set batch b used, whose matches b's post
 * stage has read by then; with batch b + 1's search (smash_phase_map_ahead)
 * already running, the device has two searches queued while the caller
 * exchanges batch b's keys.  Batch b + 2's smash_phase_map[_ahead] with the
 * same (pointer, n_pairs) uses it; same lifetime rule as d_next above. */
int smash_phase_search_ahead(smash_pipeline *p, const uint8_t *d_reads, uint64_t n_pairs,
                             void *stream);
int smash_phase_export(smash_pipeline *p, int world, uint64_t global_base,
                       int64_t *h_send_counts, int64_t *h_send_words,
                       const uint64_t **d_send, const uint64_t **d_send_words,
                       void *stream);
int smash_dedup_owner(smash_pipeline *p, const uint64_t *d_recv, uint64_t n_recv,
                      const uint64_t *d_recv_words, const int64_t *h_recv_counts,
                      const int64_t *h_recv_words, int world, uint8_t *d_flags,
                      void *stream);
int smash_phase_import(smash_pipeline *p, const uint8_t *d_flags_back,
                       void *stream);
int smash_phase_positions(smash_pipeline *p, int64_t *d_tail, void *stream);
int smash_phase_bin(smash_pipeline *p, const int64_t *d_prev, uint64_t *d_counts,
                    void *stream);

typedef struct {
  uint64_t pairs;          /* pairs processed */
  uint64_t key_pairs;      /* pairs that produced a key (smashMEM.py:162) */
  uint64_t dupe_pairs;     /* "N dupes" (smashMEM.py:227-230) */
  uint64_t positions;      /* lines reaching varbin (TotalReads) */
  uint64_t dups;           /* DupsRemoved (varbin.py:56-58) */
  uint64_t kept;           /* ReadsKept */
  uint64_t matches;        /* MAM matches */
  int32_t error;           /* first data error (SMASH_ERR_TAG_*), 0 = none */
} smash_stats;
/* Synchronises the pipeline's last stream. */
int smash_pipeline_stats(smash_pipeline *p, smash_stats *out);

/* Kernel timing for the roofline: when enabled, HIP events are recorded on
 * the launch stream around the search kernel (k_mam) of every phase_map /
 * count_batch; _read synchronises and returns the summed milliseconds, the
 * number of launches and of reads searched since the last enable. */
int smash_pipeline_profile(smash_pipeline *p, int enable);
int smash_pipeline_profile_read(smash_pipeline *p, double *search_ms,
                                uint64_t *launches, uint64_t *reads);
/* The time at least one profiled search launch was running (the union of
 * the launches' event intervals; launches on the two search streams of
 * smash_count_batches overlap).  Synchronises. */
int smash_pipeline_profile_active(smash_pipeline *p, double *active_ms);
/* Every profiled launch's [start, end] in milliseconds from the first one's
 * start (h_ms[2i], h_ms[2i + 1]), for up to cap launches; *n = launches.
 * Synchronises. */
int smash_pipeline_profile_intervals(smash_pipeline *p, double *h_ms, uint64_t cap,
                                     uint64_t *n);

/* Start a new run: clears the pair-key set, the carried adjacent-dup state
 * and the stats (a fresh smashMEM.py + varbin.py invocation). */
int smash_pipeline_reset(smash_pipeline *p, void *stream);
/* smash_pipeline_reset with flags.  SMASH_RESET_KEEP_SEARCH: look-ahead
 * searches already issued (smash_phase_map_ahead / smash_phase_search_ahead)
 * stay valid for the new run -- a search depends on the reads and the index
 * only -- so a caller running back-to-back runs over resident reads can
 * issue the next run's first searches under the last batch's exchange. */
#define SMASH_RESET_KEEP_SEARCH 1u
int smash_pipeline_reset_ex(smash_pipeline *p, uint32_t flags, void *stream);
/* on != 0: every d_reads / d_next later given to the phase calls is resident
 * in HBM and complete before the call (bench.py's sharded step), so their
 * searches wait on nothing queued on the caller's stream -- only on the
 * search set's previous post stage.  Default off: a search waits for the
 * work already on `stream` (the reads' H2D copy of a file-fed batch). */
int smash_pipeline_reads_resident(smash_pipeline *p, int on);

/* The positions the last batch emitted, in order: pos0 (0-based, smashMEM.py
 * column 5) and absolute position (pos0 + chrom_sizes.txt col 3) -- the
 * `chr pos` lines smash_mapping.sh:29 writes for varbin.py, with the chrom
 * recoverable from abspos - pos0.  *n_out = count; up to cap copied to host.
 * Synchronises. */
int smash_pipeline_positions(smash_pipeline *p, int64_t *h_pos0,
                             int64_t *h_abspos, uint64_t cap, uint64_t *n_out);

/* varbin.py's counting loop (varbin.py:52-92) on the device for a positions
 * list already restricted to binned chromosomes (varbin.py:38-49): adjacent
 * de-dup on pos0 against the previous line (prev_pos0 < 0 = none),
 * bisect_right over d_bin_starts[nbins], add into d_counts[nbins];
 * h_stats[0..2] += TotalReads, DupsRemoved, ReadsKept.  Synchronises. */
int smash_bin_positions(const int64_t *d_pos0, const int64_t *d_abspos,
                        uint64_t n, int64_t prev_pos0,
                        const int64_t *d_bin_starts, uint32_t nbins,
                        uint64_t *d_counts, uint64_t *h_stats, void *stream);

/* Debug/test view of the last batch's per-pair filter output: for pair q,
 * h_nk[q] = kept hits (-1 = no key), h_keep[q] = survives de-dup, hits as
 * (tid << 48 | pos0) in h_hits[q*2*slots ...]. slots = read_len - min_len + 1. */
int smash_pipeline_peek(smash_pipeline *p, int32_t *h_nk, uint8_t *h_keep,
                        uint64_t *h_hits, uint64_t *h_hash);

/* ========================================================================== */
/* mapout SAM writer: replaces Aligner::prepare_matches + print_matches       */
/* (query.cpp:231-415, `mummer -rcref -samin -samout [-nomap]`) and, with     */
/* tag = 1, appends mappability_tag's L<i>/R<i> columns (mappability_tag.cpp: */
/* 93-124) to the same lines.                                                 */
/* smash_sam_records: one record per match slot of smash_map_batch's output   */
/* (read i of length d_lens[i], stride >= 255, or `len` when d_lens is NULL)  */
/* (Alignment::resolve, query.cpp:68-97; XE of the match's diagonal,          */
/* :270-274; map.bin L/R of its '=' block when d_tag_offsets, the u32         */
/* sam_header offsets per forward contig, is given).  Asynchronous.           */
/* smash_sam_format: host formatting of 2 mates per pair (read 1, read 2 as   */
/* Pair::run alternates them, query.cpp:486-505) from the records copied to   */
/* the host (pure host code: contigs[] = forward contig names).  names carry the ":0"/":1" mate suffix QueryReader adds          */
/* (query.cpp:641-642); seqs are the original bases, quals the QUAL column    */
/* (NULL: '!' per base), optionals the extra columns, each prefixed by a tab  */
/* (query.cpp:153-156).  *out_text is malloc'ed (smash_sam_free) and holds    */
/* the SAM lines without the header; *tag_error gets the first                */
/* SMASH_ERR_TAG_* that mappability_tag would throw (0 = none).               */
/* cap_per_read: the search's slots per read; h_rec holds read i's records  */
/* at i * cap_per_read.  SMASH_SAM_PACKED | cap: h_rec is packed read after   */
/* read (smash_sam_records_packed with the same cap); either way a count     */
/* h_n[i] > cap (a cut match list) is SMASH_ERR_ARG.  0: packed, unchecked    */
/* (the caller guarantees every h_n[i] <= the records' cap).                  */
#define SMASH_SAM_PACKED 0x80000000u
/* ========================================================================== */
typedef struct {
  int64_t pos;             /* 0-based on the forward contig (< 0: erased)   */
  uint32_t tid;            /* forward contig index                          */
  uint32_t xe;             /* XE (n_matched_bases) of the diagonal          */
  uint16_t prefix, len, suffix, qpos;
  uint8_t rc, pad;
  uint16_t spare;
  int32_t left, right;     /* mappability_tag L/R of this '=' block         */
  uint32_t reserved;       /* 40-byte record                                */
} smash_sam_rec;
int smash_sam_records(const smash_index *ix, const uint8_t *d_reads, uint64_t stride,
                      const uint16_t *d_lens, uint32_t len, uint64_t n_reads,
                      const uint64_t *d_match, uint32_t cap_per_read,
                      const uint32_t *d_n_match, const uint32_t *d_tag_offsets,
                      smash_sam_rec *d_out, void *stream);
/* smash_sam_records_packed: the same records without the per-read slots of   */
/* cap_per_read: read i's min(d_n_match[i], cap) records go to                */
/* d_out[d_rec_off[i] ...] (d_rec_off = exclusive prefix sum of the counts),  */
/* so the table is as large as the matches, not n_reads * cap.  Format them   */
/* with smash_sam_format(..., cap_per_read = 0, ...).                         */
int smash_sam_records_packed(const smash_index *ix, const uint8_t *d_reads, uint64_t stride,
                             const uint16_t *d_lens, uint32_t len, uint64_t n_reads,
                             const uint64_t *d_match, uint32_t cap_per_read,
                             const uint32_t *d_n_match, const uint64_t *d_rec_off,
                             const uint32_t *d_tag_offsets, smash_sam_rec *d_out, void *stream);
int smash_sam_format(const char *const *contigs, uint32_t n_contig,
                     const smash_sam_rec *h_rec,
                     const uint32_t *h_n, uint32_t cap_per_read, uint64_t n_reads,
                     const char *const *names, const char *const *seqs,
                     const char *const *quals, const char *const *optionals,
                     int nomap, int tag, const uint8_t *h_small_chr,
                     char **out_text, uint64_t *out_len, int32_t *tag_error);
void smash_sam_free(char *text);

/* ========================================================================== */
/* Read ingest: replaces `zcat r1s | fastqs_to_sam r1 r2 1 | ... samtools     */
/* sort -n` (smash_mapping.sh:19-23, fastqs_to_sam.cpp:48-96) for the device  */
/* batches.  smash_fastq_read parses up to max_pairs pairs (gzip or plain;    */
/* pairs whose mates both have no bases dropped, a pair with one empty mate  */
/* is SMASH_ERR_ARG) into h_reads[2*n*len] (mate 2q = read 1;                 */
/* N -> Z and lowercase applied) and, if h_names, the read-1 names into       */
/* name_stride-byte NUL-padded slots.  *len = 0 takes the length of the first */
/* pair; every mate must have it.  *n_pairs < max_pairs means the end.        */
/* smash_strnum_order: perm[] = stable `samtools sort -n` order (strnum_cmp)  */
/* of n NUL-padded names.  Host code only.                                    */
/* ========================================================================== */
typedef struct smash_fastq smash_fastq;
int smash_fastq_open(const char *const *r1_paths, uint32_t n1,
                     const char *const *r2_paths, uint32_t n2, smash_fastq **out);
int smash_fastq_read(smash_fastq *f, uint64_t max_pairs, uint32_t *len,
                     uint8_t *h_reads, char *h_names, uint32_t name_stride,
                     uint64_t *n_pairs);
void smash_fastq_close(smash_fastq *f);
int smash_strnum_order(const char *names, uint32_t stride, uint64_t n, uint64_t *perm);

/* ========================================================================== */
/* File-fed counting: smash_mapping.sh:19-25's front (zcat | fastqs_to_sam |  */
/* samtools sort -n) feeding the pipeline, as the reference's reader threads  */
/* feed its workers (query.cpp:614-740).  The two mate lists (gzip or plain)  */
/* are parsed on two threads into pinned host batches of cfg.max_pairs pairs  */
/* (`threads` workers convert / check them: replaceN + lowercase, pairs as    */
/* smash_fastq_read, every mate of cfg.read_len bases), copied H2D on an own  */
/* stream into two device buffers, and counted with smash_count_batch on      */
/* `stream`: parse, copy and compute of consecutive batches overlap.          */
/*  sort_names = 0: the input is in samtools sort -n order already (checked   */
/*                  on the read-1 names; SMASH_ERR_ARG if not: before any     */
/*                  count with strict 4-line FASTQ, else counts partial);     */
/*                  1: all pairs are read, ordered by strnum_cmp (stable),    */
/*                  then streamed.                                            */
/*  Strict 4-line FASTQ (plain or gzip) is read by the parallel reader        */
/*  (smash_fastq_read_parallel); anything else by the streaming reader.       */
/* Adds into d_counts like smash_count_batch (the caller resets the pipeline  */
/* when a new run starts).  Synchronises `stream` before returning.           */
/* ========================================================================== */
typedef struct {
  uint64_t pairs;     /* pairs counted */
  uint64_t batches;
  double wall_s;      /* call start to the last batch's counts */
  double ingest_s;    /* host time parsing / converting / ordering */
  double wait_s;      /* time the device side waited for a parsed batch */
  uint32_t read_len;
  uint32_t parallel;  /* 1: the parallel reader ran (strict 4-line FASTQ), 0: streaming */
  double index_s;     /* parallel reader: map / inflate, index, checks before batch 0 */
} smash_feed_stats;
/* The parallel reader of smash_count_fastq, on its own (host only): every
 * pair of the two lists (strict 4-line FASTQ, plain or gzip; plain files are
 * mapped and indexed by byte range, gzip files inflated one thread per file)
 * as smash_fastq_read returns them, in file order, on `threads` threads.
 * *len: in, the required read length (0: the first pair's); out, the length.
 * h_reads NULL: *n_pairs = the pairs only.  h_names: read-1 names, NUL
 * padded, name_stride bytes each.  SMASH_ERR_UNSUPPORTED: the input is not
 * strict 4-line FASTQ (FASTA records, blank lines, ...): use smash_fastq_read. */
int smash_fastq_read_parallel(const char *const *r1, uint32_t n1, const char *const *r2,
                              uint32_t n2, uint32_t threads, uint32_t *len, uint64_t cap_pairs,
                              uint8_t *h_reads, char *h_names, uint32_t name_stride,
                              uint64_t *n_pairs);
/* The same reader as an object (host only): both lists mapped / inflated and
 * indexed once, the pairs checked and put in samtools sort -n order
 * (sort_names 1: stable sort by read-1 name; 0: the order is checked,
 * SMASH_ERR_ARG if violated); *n_pairs planned pairs, *len their length
 * (in: 0 or the required length).  _pack writes planned pairs [k0, k1) like
 * smash_fastq_read (2 (k1 - k0) len bytes; names optional), on the index's
 * threads -- the multi-GPU driver deals batches to ranks from one index
 * (smash-paper_amd/dist.py count_fastq). */
typedef struct smash_fastq_index smash_fastq_index;
int smash_fastq_index_open(const char *const *r1, uint32_t n1, const char *const *r2,
                           uint32_t n2, uint32_t threads, uint32_t *len, int sort_names,
                           smash_fastq_index **out, uint64_t *n_pairs);
int smash_fastq_index_pack(smash_fastq_index *ix, uint64_t k0, uint64_t k1, uint8_t *h_reads,
                           char *h_names, uint32_t name_stride);
void smash_fastq_index_close(smash_fastq_index *ix);
/* Rank-local ingest for the multi-GPU driver (smash-paper_amd/dist.py): no
 * rank reads the whole input (smash_mapping.sh:19 streams zcat into
 * fastqs_to_sam; query.cpp:614-740 holds one ring of reads at a time).
 *  _scan: the two lists are cut into segments (plain files: 64 MB byte ranges,
 *    gzip files: whole), dealt to `world` ranks; rank `rank` scans its own on
 *    `threads` threads -- records per segment, empty records, read-1 order,
 *    and for gzip restart points every 32 MB of output (zran: compressed
 *    offset, bits, 32 KB window) -- into *blob (free: _free_blob).
 *  _open: every rank passes all ranks' blobs (all-gathered by the caller, in
 *    rank order) and gets the same plan: *n_pairs planned pairs (pairs whose
 *    two mates are empty dropped) of *len bases (in: 0 or the required one).
 *    sort_names 0: out-of-order read-1 names are SMASH_ERR_ARG; 1: the input
 *    must be in order already (SMASH_ERR_UNSUPPORTED otherwise: sorting needs
 *    the whole input, smash_fastq_index).  Not strict 4-line FASTQ, or a last
 *    line without a newline: SMASH_ERR_UNSUPPORTED.
 *  _pack: planned pairs [k0, k1) into h_reads (2 (k1 - k0) len bytes, as
 *    smash_fastq_index_pack) on the plan's threads, reading only those pairs'
 *    bytes (plus at most a segment / restart span before each thread's first).
 *  _stats: bytes scanned and packed by this rank (the share it read). */
typedef struct smash_fastq_shards smash_fastq_shards;
typedef struct {
  uint64_t input_bytes;      /* all files of both lists (on disk) */
  uint64_t scan_segments;    /* segments this rank scanned */
  uint64_t scan_bytes;       /* FASTQ bytes this rank scanned (gzip: inflated) */
  uint64_t scan_bytes_in;    /* file bytes this rank read in the scan */
  double scan_s;
  uint64_t pack_pairs;       /* pairs packed */
  uint64_t pack_bytes;       /* FASTQ bytes parsed by the packs (gzip: inflated) */
  uint64_t pack_bytes_in;    /* compressed bytes the packs read (gzip) */
  double pack_s;
} smash_shard_stats;
int smash_fastq_shard_scan(const char *const *r1, uint32_t n1, const char *const *r2, uint32_t n2,
                           uint32_t world, uint32_t rank, uint32_t threads, void **blob,
                           uint64_t *blob_bytes);
void smash_fastq_shard_free_blob(void *blob);
int smash_fastq_shard_open(const char *const *r1, uint32_t n1, const char *const *r2, uint32_t n2,
                           uint32_t world, uint32_t rank, const void *const *blobs,
                           const uint64_t *blob_bytes, uint32_t threads, uint32_t *len,
                           int sort_names, smash_fastq_shards **out, uint64_t *n_pairs);
int smash_fastq_shard_pack(smash_fastq_shards *h, uint64_t k0, uint64_t k1, uint8_t *h_reads);
int smash_fastq_shard_stats(smash_fastq_shards *h, smash_shard_stats *stats);
void smash_fastq_shard_close(smash_fastq_shards *h);
int smash_count_fastq(smash_pipeline *p, const char *const *r1_paths, uint32_t n1,
                      const char *const *r2_paths, uint32_t n2, int sort_names,
                      uint32_t threads, uint64_t *d_counts, smash_feed_stats *stats,
                      void *stream);

#ifdef __cplusplus
}
#endif
#endif
