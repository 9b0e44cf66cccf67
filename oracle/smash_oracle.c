/*
 * oracle/smash_oracle.c -- TEST INFRASTRUCTURE ONLY (see smash_oracle.h).
 *
 * CPU restatement of the reference algorithms, written from their behaviour
 * (not copied): every function cites the reference file:line it follows.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * this library.
 */
#define _GNU_SOURCE
#include "smash_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ======================================================================== */
/* text: Sequence::Sequence (fasta.cpp:133-285) + reverse_complement (:26)   */
/* ======================================================================== */

static uint8_t rc_char(uint8_t ch) {
  /* reverse_complement switch (fasta.cpp:35-60) */
  switch (ch) {
    case 'a': return 't'; case 'c': return 'g'; case 'g': return 'c';
    case 't': return 'a'; case 'r': return 'y'; case 'y': return 'r';
    case 'm': return 'k'; case 'k': return 'm'; case 'b': return 'v';
    case 'd': return 'h'; case 'h': return 'd'; case 'v': return 'b';
    case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C';
    case 'T': return 'A'; case 'R': return 'Y'; case 'Y': return 'R';
    case 'M': return 'K'; case 'K': return 'M'; case 'B': return 'V';
    case 'D': return 'H'; case 'H': return 'D'; case 'V': return 'B';
    default: return ch;
  }
}

typedef struct { uint8_t *p; uint64_t n, cap; } bytes_t;
static void bpush(bytes_t *b, uint8_t c) {
  if (b->n == b->cap) {
    b->cap = b->cap ? b->cap * 2 : (1u << 20);
    b->p = (uint8_t *)realloc(b->p, b->cap + 64);
  }
  b->p[b->n++] = c;
}

int orc_text_from_fasta(const char *path, orc_text *out) {
  FILE *f = fopen(path, "rb");
  if (!f) return -1;
  fseek(f, 0, SEEK_END);
  long fsz = ftell(f);
  fseek(f, 0, SEEK_SET);
  char *buf = (char *)malloc((size_t)fsz + 1);
  if (fread(buf, 1, (size_t)fsz, f) != (size_t)fsz) { fclose(f); free(buf); return -1; }
  fclose(f);
  bytes_t seq = {0, 0, 0};
  uint64_t cap_s = 64, n_start = 0, n_sizes = 0, n_descr = 0;
  uint64_t *startpos = (uint64_t *)malloc(cap_s * 8);
  uint64_t *sizes = (uint64_t *)malloc(cap_s * 8);
  char **descr = (char **)malloc(cap_s * sizeof(char *));
  startpos[n_start++] = 0;                 /* fasta.cpp:189 */
  char meta[4096]; size_t meta_n = 0; meta[0] = 0;
  uint64_t length = 0;
  long pos = 0;
  int eof = 0;
  while (!eof) {
    /* std::getline emulation: eof only when the read hit end-of-file */
    long a = pos, b;
    if (pos >= fsz) { b = pos; eof = 1; }
    else {
      char *nl = memchr(buf + pos, '\n', (size_t)(fsz - pos));
      if (nl) { b = nl - buf; pos = b + 1; }
      else { b = fsz; pos = fsz; eof = 1; }
    }
    const char *line = buf + a;
    uint64_t lsz = (uint64_t)(b - a);
    if (!eof && lsz == 0) continue;                       /* :197 */
    uint64_t start = 0, end = lsz;
    char c0 = lsz ? line[0] : 0;
    if (eof || c0 == '>') {                               /* :202 */
      if (length > 0) {
        uint64_t this_start = startpos[n_start - 1];
        if (n_descr + 2 > cap_s || n_start + 2 > cap_s || n_sizes + 2 > cap_s) {
          cap_s *= 2;
          startpos = (uint64_t *)realloc(startpos, cap_s * 8);
          sizes = (uint64_t *)realloc(sizes, cap_s * 8);
          descr = (char **)realloc(descr, cap_s * sizeof(char *));
        }
        descr[n_descr++] = strdup(meta);
        /* rcref is always on for SMASH (smash_mapping.sh:19) */
        bpush(&seq, '`');
        startpos[n_start++] = seq.n;
        sizes[n_sizes++] = length;
        descr[n_descr++] = strdup(meta);
        sizes[n_sizes++] = length;
        for (uint64_t k = 0; k < length; ++k)
          bpush(&seq, rc_char(seq.p[this_start + length - 1 - k]));
        if (!eof) {
          bpush(&seq, '`');
          startpos[n_start++] = seq.n;
        }
        if (eof) break;
      }
      start = 1; meta_n = 0; meta[0] = 0; length = 0;
    }
    /* trim (fasta.cpp:109-124), including its `i != 1` lower stop */
    for (uint64_t i = start; i < lsz; ++i)
      if (line[i] != ' ') { start = i; break; }
    for (uint64_t i = lsz; i != 1 && i != 0; --i)
      if (line[i - 1] != ' ') { end = i; break; }
    if (c0 == '>') {
      for (uint64_t i = start; i != end; ++i) {
        if (line[i] == ' ') break;
        if (meta_n + 1 < sizeof(meta)) { meta[meta_n++] = line[i]; meta[meta_n] = 0; }
      }
    } else {
      length += end - start;
      for (uint64_t i = start; i != end; ++i) {
        unsigned char ch = (unsigned char)line[i];
        bpush(&seq, (uint8_t)((ch >= 'A' && ch <= 'Z') ? ch + 32 : ch));
      }
    }
  }
  bpush(&seq, '$');                                       /* :247 */
  free(buf);
  memset(seq.p + seq.n, 0, 64);
  /* startpos can hold one entry more than sizes (trailing push); the
   * reference keeps both vectors; resolve() only uses the first n_sizes. */
  out->N = seq.n;
  out->T = seq.p;
  out->n_seq = (uint32_t)n_sizes;
  out->startpos = startpos;
  out->sizes = sizes;
  out->names = descr;
  return 0;
}

void orc_text_free(orc_text *t) {
  if (!t) return;
  for (uint32_t i = 0; i < t->n_seq; ++i) free(t->names[i]);
  free(t->names); free(t->T); free(t->startpos); free(t->sizes);
  memset(t, 0, sizeof(*t));
}

/* ======================================================================== */
/* index: SA by prefix doubling, ISA, Kasai LCP (longSA.cpp:140-175,224-237) */
/* ======================================================================== */

int orc_build_sa(const uint8_t *T, uint64_t N, uint64_t *SA) {
  if (N == 0) return 0;
  uint64_t *rank = (uint64_t *)malloc(N * 8);
  uint64_t *nrank = (uint64_t *)malloc(N * 8);
  uint64_t *tmp = (uint64_t *)malloc(N * 8);
  uint64_t *ptr = (uint64_t *)malloc((N > 257 ? N : 257) * 8);
  if (!rank || !nrank || !tmp || !ptr) return -1;
  /* round 0: bucket by byte; rank = head index of the bucket */
  uint64_t cnt[257];
  memset(cnt, 0, sizeof(cnt));
  for (uint64_t i = 0; i < N; ++i) cnt[T[i] + 1]++;
  for (int c = 1; c < 257; ++c) cnt[c] += cnt[c - 1];
  for (uint64_t i = 0; i < N; ++i) rank[i] = cnt[T[i]];
  for (uint64_t i = 0; i < N; ++i) SA[cnt[T[i]]++] = i;
  uint64_t groups = 0;
  for (uint64_t k = 0; k < N; ++k)
    if (k == 0 || rank[SA[k]] != rank[SA[k - 1]]) ++groups;
  for (uint64_t h = 1; groups < N; h *= 2) {
    /* tmp: suffixes ordered by second key rank[i+h] (absent = smallest) */
    uint64_t t = 0;
    for (uint64_t i = (N > h ? N - h : 0); i < N; ++i) tmp[t++] = i;
    for (uint64_t k = 0; k < N; ++k)
      if (SA[k] >= h) tmp[t++] = SA[k] - h;
    /* stable distribution by first key (bucket heads) */
    for (uint64_t k = 0; k < N; ++k) ptr[k] = k;
    for (uint64_t k = 0; k < N; ++k) {
      uint64_t i = tmp[k];
      SA[ptr[rank[i]]++] = i;
    }
    groups = 0;
    uint64_t head = 0;
    for (uint64_t k = 0; k < N; ++k) {
      uint64_t i = SA[k];
      if (k == 0) { head = 0; ++groups; }
      else {
        uint64_t j = SA[k - 1];
        uint64_t a2 = i + h < N ? rank[i + h] + 1 : 0;
        uint64_t b2 = j + h < N ? rank[j + h] + 1 : 0;
        if (rank[i] != rank[j] || a2 != b2) { head = k; ++groups; }
      }
      nrank[i] = head;
    }
    uint64_t *sw = rank; rank = nrank; nrank = sw;
  }
  free(rank); free(nrank); free(tmp); free(ptr);
  return 0;
}

void orc_build_isa(const uint64_t *SA, uint64_t N, uint64_t *ISA) {
  for (uint64_t k = 0; k < N; ++k) ISA[SA[k]] = k;
}

void orc_build_lcp(const uint8_t *T, uint64_t N, const uint64_t *SA,
                   const uint64_t *ISA, uint64_t *LCP) {
  uint64_t h = 0;
  for (uint64_t i = 0; i < N; ++i) {
    uint64_t m = ISA[i];
    if (m == 0) {
      LCP[0] = 0;
    } else {
      uint64_t j = SA[m - 1];
      while (i + h < N && j + h < N && T[i + h] == T[j + h]) ++h;
      LCP[m] = h;
    }
    h = h ? h - 1 : 0;
  }
}

uint64_t orc_logN(uint64_t N) {
  return (uint64_t)ceil(log((double)N) / log(2.0));
}

/* ======================================================================== */
/* search kernels (longSA.cpp:297-590)                                       */
/* ======================================================================== */

typedef struct {
  const orc_index *ix;
  orc_counters *c;
  uint32_t isz;      /* element bytes of SA/ISA */
  int dev;           /* mem.hip's probe sequence (orc_mem_dev) */
} ctx_t;

static inline uint64_t idx_at(const orc_index *ix, const void *a, uint32_t isz, uint64_t k) {
  const uint64_t m = ix->pos_mask ? ix->pos_mask : ~(uint64_t)0;
  return (isz == 4 ? ((const uint32_t *)a)[k] : ((const uint64_t *)a)[k]) & m;
}

/* vec_uchar::operator[] (longSA.h:34-39) */
static uint64_t lcp_exact(const orc_index *ix, uint64_t k, orc_counters *c) {
  const uint8_t v = ix->L8[k];
  if (v != 255) return v;
  if (c) c->ovf_lookups++;
  uint64_t lo = 0, hi = ix->n_ovf;
  while (lo < hi) {
    uint64_t mid = (lo + hi) / 2;
    if (ix->ovf[2 * mid] < k) lo = mid + 1; else hi = mid;
  }
  return ix->ovf[2 * lo + 1];
}

static inline void tick(uint64_t *loads, uint64_t *lines, uint64_t *last,
                        uint64_t byte_addr) {
  ++*loads;
  uint64_t line = byte_addr >> 6;
  if (line != *last) { ++*lines; *last = line; }
}
static inline uint64_t SAat(const ctx_t *x, uint64_t k) {
  if (x->c) tick(&x->c->sa_loads, &x->c->sa_lines, &x->c->last_sa, k * x->isz);
  return idx_at(x->ix, x->ix->SA, x->isz, k);
}
static inline uint64_t ISAat(const ctx_t *x, uint64_t k) {
  if (x->c) tick(&x->c->isa_loads, &x->c->isa_lines, &x->c->last_isa, k * x->isz);
  return idx_at(x->ix, x->ix->ISA, x->isz, k);
}
static inline int64_t Tat(const ctx_t *x, uint64_t k) {
  if (x->c) tick(&x->c->ref_loads, &x->c->ref_lines, &x->c->last_ref, k);
  return (int64_t)(int8_t)x->ix->T[k];
}
static inline uint64_t LCPat(const ctx_t *x, uint64_t k) {
  if (x->c) tick(&x->c->lcp_loads, &x->c->lcp_lines, &x->c->last_lcp, k);
  return lcp_exact(x->ix, k, x->c);
}

typedef struct { uint64_t depth, start, end; } ival_t;   /* longSA.h:64-75 */

/* top_down_faster (longSA.cpp:322-380): narrow [start,end] at depth i by c */
static int td_faster(const ctx_t *x, int64_t c, uint64_t i, uint64_t *start,
                     uint64_t *end) {
  uint64_t l, r, m, r2 = *end, l2 = *start;
  int64_t v;
  int found = 0;
  const int64_t cf = c - Tat(x, SAat(x, *start) + i);
  const int64_t cl = c - Tat(x, SAat(x, *end) + i);
  if (cf < 0) {
    l = *start + 1; l2 = *start;
  } else if (cl > 0) {
    l = *end + 1; l2 = *end;
  } else {
    l = *start; r = *end;
    if (cf == 0) {
      found = 1; r2 = r;
    } else {
      while (r > l + 1) {
        m = (l + r) / 2;
        v = c - Tat(x, SAat(x, m) + i);
        if (v <= 0) {
          if (!found && v == 0) { found = 1; l2 = m; r2 = r; }
          r = m;
        } else {
          l = m;
        }
      }
      l = r;
    }
    if (!found) l2 = l - 1;
    if (cl == 0) {
      l2 = *end;
    } else {
      while (r2 > l2 + 1) {
        m = (l2 + r2) / 2;
        v = c - Tat(x, SAat(x, m) + i);
        if (v < 0) r2 = m; else l2 = m;
      }
    }
  }
  *start = l;
  *end = l2;
  return l <= l2;
}

/* traverse (longSA.cpp:297-316) */
static void traverse(const ctx_t *x, const uint8_t *P, uint64_t L,
                     uint64_t prefix, ival_t *cur, uint64_t min_len) {
  if (cur->depth >= min_len) return;
  while (prefix + cur->depth < L) {
    uint64_t s = cur->start, e = cur->end;
    if (!td_faster(x, (int64_t)(int8_t)P[prefix + cur->depth], cur->depth, &s, &e))
      return;
    cur->depth += 1;
    cur->start = s;
    cur->end = e;
    if (cur->depth == min_len) return;
  }
}

/* expand_link (longSA.h:158-174) */
static int expand_link(const ctx_t *x, ival_t *link) {
  const uint64_t thresh = 2 * link->depth * x->ix->logN;
  uint64_t exp = 0, s = link->start, e = link->end;
  while (LCPat(x, s) >= link->depth) {
    if (++exp >= thresh) return 0;
    --s;
  }
  while (e < x->ix->N - 1 && LCPat(x, e + 1) >= link->depth) {
    if (++exp >= thresh) return 0;
    ++e;
  }
  link->start = s;
  link->end = e;
  return 1;
}

/* suffixlink (longSA.cpp:383-392) */
static int suffixlink(const ctx_t *x, ival_t *m) {
  if (m->depth <= 1) { m->depth = 0; return 0; }
  --m->depth;
  m->start = ISAat(x, SAat(x, m->start) + 1);
  m->end = ISAat(x, SAat(x, m->end) + 1);
  return expand_link(x, m);
}

typedef struct { orc_match *out; uint32_t cap, n; } sink_t;
static void emit(sink_t *s, uint64_t ref, uint64_t q, uint64_t len) {
  if (s->n < s->cap) { s->out[s->n].ref = ref; s->out[s->n].query = q; s->out[s->n].len = len; }
  ++s->n;
}

static ctx_t mkctx(const orc_index *ix, orc_counters *c) {
  ctx_t x;
  x.ix = ix; x.c = c;
  x.isz = ix->idx_bytes == 4 ? 4 : 8;
  x.dev = 0;
  return x;
}

int orc_mam(const orc_index *ix, const uint8_t *P, uint32_t L,
            uint32_t min_len, orc_match *out, uint32_t cap, orc_counters *ctr) {
  ctx_t x = mkctx(ix, ctr);
  sink_t s = {out, cap, 0};
  const uint64_t N = ix->N;
  ival_t cur = {0, 0, N - 1};
  uint64_t prefix = 0;
  while (prefix < L) {                                   /* longSA.cpp:507 */
    traverse(&x, P, L, prefix, &cur, L);
    if (cur.depth <= 1) {
      cur.depth = 0; cur.start = 0; cur.end = N - 1;
      ++prefix;
      continue;
    }
    if (cur.end - cur.start + 1 == 1 && cur.depth >= min_len) {
      uint64_t p2 = SAat(&x, cur.start);
      /* is_leftmaximal (longSA.cpp:540-546) */
      int lm = (prefix == 0 || p2 == 0) ? 1
               : ((int64_t)(int8_t)P[prefix - 1] != Tat(&x, p2 - 1));
      if (lm) emit(&s, SAat(&x, cur.start), prefix, cur.depth);
    }
    do {                                                 /* :523-534 */
      cur.depth = cur.depth - 1;
      cur.start = ISAat(&x, SAat(&x, cur.start) + 1);
      cur.end = ISAat(&x, SAat(&x, cur.end) + 1);
      ++prefix;
      if (cur.depth == 0 || !expand_link(&x, &cur)) {
        cur.depth = 0; cur.start = 0; cur.end = N - 1;
        break;
      }
    } while (cur.depth > 0 && cur.end - cur.start + 1 == 1);
  }
  return (int)s.n;
}

/* find_Lmaximal (longSA.cpp:438-457) */
static void find_lmax(const ctx_t *x, sink_t *s, const uint8_t *P,
                      uint32_t min_len, uint64_t prefix, uint64_t i,
                      uint64_t len) {
  if (prefix == 0 || i == 0) {
    if (len >= min_len) emit(s, i, prefix, len);
    return;
  } else if ((int64_t)(int8_t)P[prefix - 1] != Tat(x, i - 1)) {
    if (len >= min_len) emit(s, i, prefix, len);
    return;
  }
}

/* find_Lmaximal of the suffix at SA rank `rank`.  mem.hip over packed
 * words (pos_mask, 8-byte elements): a word whose tag (bits 33-35) is 0..3
 * names T[i - 1] as a c g t, so the device compares with it instead of
 * loading the text byte (csrc/mem.hip left_max); the outcome is the same */
static void find_lmax_rank(const ctx_t *x, sink_t *s, const uint8_t *P, uint32_t min_len,
                           uint64_t prefix, uint64_t rank, uint64_t len) {
  const uint64_t i = SAat(x, rank);
  if (x->dev && x->ix->pos_mask && x->isz == 8 && prefix != 0 && i != 0) {
    const unsigned tag = (unsigned)((((const uint64_t *)x->ix->SA)[rank] >> 33) & 7);
    if (tag < 4) {
      if (P[prefix - 1] != (uint8_t)"acgt"[tag] && len >= min_len) emit(s, i, prefix, len);
      return;
    }
  }
  find_lmax(x, s, P, min_len, prefix, i, len);
}

/* collectMEMs (longSA.cpp:461-490) */
static void collect_mems(const ctx_t *x, sink_t *s, const uint8_t *P,
                         uint32_t min_len, uint64_t prefix, ival_t mli,
                         ival_t xmi) {
  const uint64_t N = x->ix->N;
  for (uint64_t i = xmi.start; i <= xmi.end; ++i)
    find_lmax_rank(x, s, P, min_len, prefix, i, xmi.depth);
  if (mli.start == xmi.start && mli.end == xmi.end) return;
  while (xmi.depth >= mli.depth) {
    if (xmi.end + 1 < N) {
      uint64_t a = LCPat(x, xmi.start), b = LCPat(x, xmi.end + 1);
      xmi.depth = a > b ? a : b;
    } else {
      xmi.depth = LCPat(x, xmi.start);
    }
    if (xmi.depth >= mli.depth) {
      while (LCPat(x, xmi.start) >= xmi.depth) {
        --xmi.start;
        find_lmax_rank(x, s, P, min_len, prefix, xmi.start, xmi.depth);
      }
      while (xmi.end + 1 < N && LCPat(x, xmi.end + 1) >= xmi.depth) {
        ++xmi.end;
        find_lmax_rank(x, s, P, min_len, prefix, xmi.end, xmi.depth);
      }
    }
  }
}

static int acgt(uint8_t c);

/* traverse as smash-paper_amd/csrc/mem.hip's traverse_x runs it (same
 * outcome, fewer probes): (C) a descent from the root with K ACGT bases
 * available starts at depth K from the k-mer table (one 16-byte entry);
 * (A) a singleton extends by comparing the read with the text 8 bytes per
 * load (load8: the aligned 8-byte word(s) holding them).  Counted like the
 * device loads them: one k-mer-table line, text lines per aligned word. */
static void traverse_dev(const ctx_t *x, const orc_accel *acc, const uint8_t *P, uint64_t L,
                         uint64_t prefix, ival_t *cur, uint64_t limit) {
  const uint64_t N = x->ix->N;
  const uint32_t K = acc->K;
  if (cur->depth >= limit) return;
  if (cur->depth == 0 && cur->start == 0 && cur->end == N - 1 && K > 0 && K <= limit &&
      prefix + K <= L) {
    uint64_t w = 0;
    int ok = 1;
    for (uint32_t k = 0; k < K; ++k) {
      const int v = acgt(P[prefix + k]);
      ok = ok && v >= 0;
      w = (w << 2) | (uint64_t)(v & 3);
    }
    if (ok) {
      if (x->c) tick(&x->c->sa_loads, &x->c->kt_lines, &x->c->last_kt, 16 * w);
      const uint64_t lo = acc->KT[2 * w] & ((1ull << 40) - 1);
      const uint64_t hi = acc->KT[2 * w + 1] & ((1ull << 40) - 1);
      if (lo <= hi) {
        cur->depth = K; cur->start = lo; cur->end = hi;
        if (cur->depth == limit) return;
      }
    }
  }
  while (prefix + cur->depth < L) {
    if (cur->start == cur->end) {                                  /* (A) */
      const uint64_t pos = SAat(x, cur->start);
      while (prefix + cur->depth < L && cur->depth < limit) {
        const uint64_t rr = L - prefix - cur->depth, rl = limit - cur->depth;
        const uint64_t rem = rr < rl ? rr : rl;
        const uint32_t lim = rem < 8 ? (uint32_t)rem : 8u;
        const uint64_t a = pos + cur->depth;
        if (x->c) {
          tick(&x->c->ref_loads, &x->c->ref_lines, &x->c->last_ref, a & ~7ull);
          if (a & 7) tick(&x->c->ref_loads, &x->c->ref_lines, &x->c->last_ref, (a & ~7ull) + 8);
        }
        uint32_t k = 0;
        while (k < lim && x->ix->T[a + k] == P[prefix + cur->depth + k]) ++k;
        cur->depth += k;
        if (k < lim) break;
      }
      return;
    }
    uint64_t s = cur->start, e = cur->end;
    if (!td_faster(x, (int64_t)(int8_t)P[prefix + cur->depth], cur->depth, &s, &e)) return;
    cur->depth += 1;
    cur->start = s;
    cur->end = e;
    if (cur->depth == limit) return;
  }
}

static int mem_core(const orc_index *ix, const orc_accel *acc, const uint8_t *P, uint32_t L,
                    uint32_t min_len, orc_match *out, uint32_t cap, orc_counters *ctr);

int orc_mem(const orc_index *ix, const uint8_t *P, uint32_t L,
            uint32_t min_len, orc_match *out, uint32_t cap, orc_counters *ctr) {
  return mem_core(ix, NULL, P, L, min_len, out, cap, ctr);
}

int orc_mem_dev(const orc_index *ix, const orc_accel *acc, const uint8_t *P, uint32_t L,
                uint32_t min_len, orc_match *out, uint32_t cap, orc_counters *ctr) {
  return mem_core(ix, acc, P, L, min_len, out, cap, ctr);
}

/* findMEM (longSA.cpp:395-431); acc: mem.hip's traverse (traverse_dev) */
static int mem_core(const orc_index *ix, const orc_accel *acc, const uint8_t *P, uint32_t L,
                    uint32_t min_len, orc_match *out, uint32_t cap, orc_counters *ctr) {
  if (min_len < 1) return 0;                           /* longSA.cpp:588 */
  ctx_t x = mkctx(ix, ctr);
  x.dev = acc != NULL;
  sink_t s = {out, cap, 0};
  const uint64_t N = ix->N;
  uint64_t prefix = 1;                                 /* longSA.cpp:398 */
  ival_t mli = {0, 0, N - 1}, xmi = {0, 0, N - 1};
#define TRAV(cur, lim) (acc ? traverse_dev(&x, acc, P, L, prefix, cur, lim) \
                            : traverse(&x, P, L, prefix, cur, lim))
  while (prefix <= L) {
    TRAV(&mli, min_len);
    if (mli.depth > xmi.depth) xmi = mli;
    if (mli.depth <= 1) {
      mli.depth = 0; mli.start = 0; mli.end = N - 1;
      xmi = mli;
      ++prefix;
      continue;
    }
    if (mli.depth >= min_len) {
      TRAV(&xmi, L);
      collect_mems(&x, &s, P, min_len, prefix, mli, xmi);
      ++prefix;
      if (!suffixlink(&x, &mli)) {
        mli.depth = 0; mli.start = 0; mli.end = N - 1;
        xmi = mli;
        continue;
      }
      suffixlink(&x, &xmi);
    } else {
      ++prefix;
      if (!suffixlink(&x, &mli)) {
        mli.depth = 0; mli.start = 0; mli.end = N - 1;
        xmi = mli;
        continue;
      }
      xmi = mli;
    }
  }
#undef TRAV
  return (int)s.n;
}

/* MEM (-maxmatch) over n reads on `threads` host threads: the reference's
 * probe sequence (acc == NULL, orc_mem) or mem.hip's (orc_mem_dev); per-read
 * match counts into n_out (or NULL); returns the matches found */
typedef struct {
  const orc_index *ix;
  const orc_accel *acc;
  const uint8_t *reads;
  uint32_t L, min_len;
  uint64_t stride, begin, end, total;
  uint32_t *n_out;
  orc_counters ctr;
  int count;
} memjob_t;

static void *mem_worker(void *arg) {
  memjob_t *j = (memjob_t *)arg;
  orc_match m[64];
  memset(&j->ctr, 0, sizeof(j->ctr));
  j->ctr.last_sa = j->ctr.last_isa = j->ctr.last_ref = j->ctr.last_lcp = ~0ull;
  j->ctr.last_kt = j->ctr.last_u = j->ctr.last_bm = ~0ull;
  for (uint64_t q = j->begin; q < j->end; ++q) {
    const int n = mem_core(j->ix, j->acc, j->reads + q * j->stride, j->L, j->min_len, m, 64,
                           j->count ? &j->ctr : NULL);
    if (j->n_out) j->n_out[q] = (uint32_t)n;
    j->total += (uint64_t)n;
  }
  return NULL;
}

uint64_t orc_mem_batch(const orc_index *ix, const orc_accel *acc, const uint8_t *reads,
                       uint32_t L, uint64_t stride, uint64_t n, uint32_t min_len, int threads,
                       uint32_t *n_out, orc_counters *ctr) {
  if (threads < 1) threads = 1;
  if (threads > 1024) threads = 1024;
  pthread_t th[1024];
  memjob_t *jobs = (memjob_t *)calloc((size_t)threads, sizeof(memjob_t));
  for (int t = 0; t < threads; ++t) {
    jobs[t].ix = ix; jobs[t].acc = acc; jobs[t].reads = reads; jobs[t].L = L;
    jobs[t].min_len = min_len; jobs[t].stride = stride; jobs[t].n_out = n_out;
    jobs[t].begin = n * (uint64_t)t / (uint64_t)threads;
    jobs[t].end = n * (uint64_t)(t + 1) / (uint64_t)threads;
    jobs[t].count = ctr != NULL;
    pthread_create(&th[t], NULL, mem_worker, &jobs[t]);
  }
  uint64_t total = 0;
  if (ctr) memset(ctr, 0, sizeof(*ctr));
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    total += jobs[t].total;
    if (ctr) {
      ctr->sa_loads += jobs[t].ctr.sa_loads; ctr->sa_lines += jobs[t].ctr.sa_lines;
      ctr->isa_loads += jobs[t].ctr.isa_loads; ctr->isa_lines += jobs[t].ctr.isa_lines;
      ctr->ref_loads += jobs[t].ctr.ref_loads; ctr->ref_lines += jobs[t].ctr.ref_lines;
      ctr->lcp_loads += jobs[t].ctr.lcp_loads; ctr->lcp_lines += jobs[t].ctr.lcp_lines;
      ctr->ovf_lookups += jobs[t].ctr.ovf_lookups; ctr->kt_lines += jobs[t].ctr.kt_lines;
    }
  }
  free(jobs);
  return total;
}

static int by_ref_cmp(const void *a, const void *b) {   /* longSA.cpp:492-499 */
  const orc_match *x = (const orc_match *)a, *y = (const orc_match *)b;
  if (x->ref == y->ref) return (x->len > y->len) ? -1 : (x->len < y->len);
  return x->ref < y->ref ? -1 : 1;
}

int orc_mum(const orc_index *ix, const uint8_t *P, uint32_t L,
            uint32_t min_len, orc_match *out, uint32_t cap, orc_counters *ctr) {
  orc_match tmp[1024];
  int n = orc_mam(ix, P, L, min_len, tmp, 1024, ctr);
  if (n > 1024) n = 1024;
  qsort(tmp, (size_t)n, sizeof(orc_match), by_ref_cmp);
  sink_t s = {out, cap, 0};
  uint64_t dbright = 0, currentright;
  int ignorecurrent, ignoreprevious = 0;
  for (int i = 0; i < n; ++i) {                         /* :561-579 */
    ignorecurrent = 0;
    currentright = tmp[i].ref + tmp[i].len - 1;
    if (dbright > currentright) {
      ignorecurrent = 1;
    } else if (dbright == currentright) {
      ignorecurrent = 1;
      if (!ignoreprevious && tmp[i - 1].ref == tmp[i].ref) ignoreprevious = 1;
    } else {
      dbright = currentright;
    }
    if (i > 0 && !ignoreprevious) emit(&s, tmp[i - 1].ref, tmp[i - 1].query, tmp[i - 1].len);
    ignoreprevious = ignorecurrent;
  }
  if (!ignoreprevious && n > 0) emit(&s, tmp[n - 1].ref, tmp[n - 1].query, tmp[n - 1].len);
  return (int)s.n;
}

/* ======================================================================== */
/* prepare_matches (query.cpp:68-97, 203-306)                               */
/* ======================================================================== */

typedef struct {
  int64_t rcpos, pos, qpos;
  uint64_t seq_index, prefix, length, suffix;
  uint32_t rc, n_matches, n_unique, n_matched;
  int end_of_group;
  char cigar[ORC_CIGAR_MAX];
  uint8_t nb; uint16_t boff[16], blen[16];
} aln_t;

/* comparators take the alignment base explicitly (thread-safe; the worker
 * threads of orc_run_pairs resolve concurrently) */
static int to_merge_cmp(const aln_t *base, uint32_t ia, uint32_t ib) {
  const aln_t *a = base + ia;
  const aln_t *b = base + ib;
  if (a->rc != b->rc) return a->rc < b->rc ? -1 : 1;
  if (a->seq_index != b->seq_index) return a->seq_index < b->seq_index ? -1 : 1;
  if (a->pos != b->pos) return a->pos < b->pos ? -1 : 1;
  if (a->prefix != b->prefix) return a->prefix < b->prefix ? -1 : 1;
  return 0;
}
static int to_print_cmp(const aln_t *base, uint32_t ia, uint32_t ib) {
  const aln_t *a = base + ia;
  const aln_t *b = base + ib;
  if (a->qpos != b->qpos) return a->qpos < b->qpos ? -1 : 1;
  if (a->rc != b->rc) return a->rc < b->rc ? -1 : 1;
  /* ties only between members of one diagonal group: equal seq/pos */
  return (a->n_matches > b->n_matches) ? -1 : (a->n_matches < b->n_matches);
}

static void isort(uint32_t *idx, uint32_t n, const aln_t *base,
                  int (*cmp)(const aln_t *, uint32_t, uint32_t)) {
  for (uint32_t i = 1; i < n; ++i) {
    uint32_t t = idx[i];
    uint32_t j = i;
    while (j > 0 && cmp(base, t, idx[j - 1]) < 0) { idx[j] = idx[j - 1]; --j; }
    idx[j] = t;
  }
}

int orc_resolve(const orc_index *ix, const uint8_t *P, uint32_t L,
                const orc_match *m, uint32_t n, orc_hit *out, uint32_t cap,
                uint32_t *best_tid, int64_t *best_pos) {
  aln_t al[ORC_MAX_MATCH];
  uint32_t idx[ORC_MAX_MATCH];
  uint32_t na = 0;
  *best_tid = UINT32_MAX;
  *best_pos = 0;
  if (n > ORC_MAX_MATCH) return -ORC_ERR_CAP;   /* never truncate */
  for (uint32_t k = 0; k < n; ++k) {
    aln_t *a = &al[na];
    memset(a, 0, sizeof(*a));
    /* resolve (query.cpp:68-97) */
    uint32_t lo = 0, hi = ix->n_seq;          /* upper_bound(startpos, ref) */
    while (lo < hi) {
      uint32_t mid = (lo + hi) / 2;
      if (ix->startpos[mid] <= m[k].ref) lo = mid + 1; else hi = mid;
    }
    uint64_t si = lo - 1;
    a->seq_index = si;
    a->rcpos = (int64_t)(m[k].ref - m[k].query);
    a->pos = (int64_t)((uint64_t)a->rcpos - ix->startpos[si]);
    const uint32_t extra = (uint32_t)(L - m[k].len - m[k].query);
    if (si % 2 == 1) {
      a->seq_index = si - 1;
      a->pos = (int64_t)(ix->sizes[si - 1] - (uint64_t)a->pos);
      a->pos -= (int64_t)L;
      a->prefix = extra;
      a->suffix = m[k].query;
      a->rc = 1;
    } else {
      a->prefix = m[k].query;
      a->suffix = extra;
      a->rc = 0;
    }
    a->qpos = (int64_t)m[k].query;
    a->length = m[k].len;
    if (a->pos >= 0) ++na;                     /* erase pos < 0 (:239-246) */
  }
  if (na == 0) return 0;
  for (uint32_t i = 0; i < na; ++i) idx[i] = i;
  isort(idx, na, al, to_merge_cmp);
  /* merge equal diagonals into one CIGAR (query.cpp:252-289) */
  uint32_t gstart = 0;
  char cig[ORC_CIGAR_MAX];
  int cend = 0;
  uint64_t last_end = 0;
  uint8_t nb = 0; uint16_t boff[16], blen[16];
  uint64_t off_walk = 0;
  int cig_over = 0;   /* a CIGAR longer than ORC_CIGAR_MAX - 1 (never truncated) */
  for (uint32_t i = 0; i < na; ++i) {
    aln_t *a = &al[idx[i]];
    aln_t *nx = (i + 1 == na) ? NULL : &al[idx[i + 1]];
    if (a->prefix) {
      cend += snprintf(cig + cend, sizeof(cig) - (size_t)cend, "%lu%c",
                       (unsigned long)(a->prefix - last_end), last_end ? 'M' : 'S');
      off_walk += a->prefix - last_end;
    }
    if (nb < 16) { boff[nb] = (uint16_t)off_walk; blen[nb] = (uint16_t)a->length; }
    ++nb;
    cend += snprintf(cig + cend, sizeof(cig) - (size_t)cend, "%lu=",
                     (unsigned long)a->length);
    off_walk += a->length;
    if (!nx || nx->pos != a->pos || nx->seq_index != a->seq_index || nx->rc != a->rc) {
      if (a->suffix)
        cend += snprintf(cig + cend, sizeof(cig) - (size_t)cend, "%luS",
                         (unsigned long)a->suffix);
      if (cend >= (int)sizeof(cig) - 1) { cig_over = 1; cend = (int)sizeof(cig) - 1; }
      uint32_t nm = 0;
      for (uint32_t j = 0; j < L; ++j) {
        int64_t rp = a->rcpos + (int64_t)j;
        if (rp >= 0 && rp < (int64_t)ix->N && ix->T[rp] == P[j]) ++nm;
      }
      a->n_matched = nm;
      a->n_matches = i - gstart + 1;
      uint64_t su = 0;
      int64_t qmin = a->qpos;
      for (uint32_t g = gstart; g <= i; ++g) {
        su += al[idx[g]].length;
        if (al[idx[g]].qpos < qmin) qmin = al[idx[g]].qpos;
      }
      a->n_unique = (uint32_t)su;
      a->qpos = qmin;
      a->end_of_group = 1;
      memcpy(a->cigar, cig, (size_t)cend + 1);
      a->nb = nb > 16 ? 16 : nb;
      memcpy(a->boff, boff, sizeof(boff));
      memcpy(a->blen, blen, sizeof(blen));
      gstart = i + 1; cend = 0; last_end = 0; nb = 0; off_walk = 0;
    } else {
      last_end = a->prefix + a->length;
    }
  }
  /* to_print order (query.cpp:290-303) */
  for (uint32_t i = 0; i < na; ++i) idx[i] = i;
  isort(idx, na, al, to_print_cmp);
  *best_tid = (uint32_t)(al[idx[0]].seq_index / 2);
  *best_pos = al[idx[0]].pos;
  uint32_t nh = 0;
  for (uint32_t i = 0; i < na; ++i) if (al[i].n_matches) ++nh;
  uint32_t hi = 0;
  if (cig_over) return -ORC_ERR_CAP;
  for (uint32_t i = 0; i < na; ++i) {
    aln_t *a = &al[idx[i]];
    if (!a->n_matches) continue;
    if (hi >= cap) return -ORC_ERR_CAP;          /* never truncate */
    if (hi < cap) {
      orc_hit *h = &out[hi];
      memset(h, 0, sizeof(*h));
      h->tid = (uint32_t)(a->seq_index / 2);
      h->rc = a->rc;
      h->pos = a->pos;
      h->qpos = a->qpos;
      h->n_matches = a->n_matches;
      h->n_unique = a->n_unique;
      h->n_matched = a->n_matched;
      h->hi = hi;
      h->nh = nh;
      /* pysam qstart/qend from the CIGAR's soft clips */
      h->qstart = a->boff[0];
      h->qend = L - (uint32_t)a->suffix;      /* trailing S */
      h->first_off = a->boff[0];
      h->first_len = a->blen[0];
      h->L0 = h->R0 = -1;
      memcpy(h->cigar, a->cigar, sizeof(h->cigar));
    }
    ++hi;
  }
  return (int)hi;
}

/* ======================================================================== */
/* mappability (longSA.cpp:612-690)                                          */
/* ======================================================================== */

int orc_mappability(const orc_index *ix, uint8_t *out) {
  const uint64_t N = ix->N;
  uint64_t *ml = (uint64_t *)malloc(N * 8);
  if (!ml) return -1;
  for (uint64_t i = 0; i < N; ++i) {
    ml[i] = lcp_exact(ix, i, NULL) + 1;
    if (i && ml[i - 1] < ml[i]) ml[i - 1] = ml[i];
  }
  out[0] = 0; out[1] = 0;          /* 2 junk bytes (longSA.cpp:617) */
  uint64_t w = 2;
  for (uint32_t chrom = 0; chrom < ix->n_seq; chrom += 2) {
    const uint64_t sp = ix->startpos[chrom], sz = ix->sizes[chrom];
    for (uint64_t i = 0; i < sz; ++i) {
      const uint64_t sapos = idx_at(ix, ix->ISA, ix->idx_bytes, i + sp);
      const uint64_t rcsapos = idx_at(ix, ix->ISA, ix->idx_bytes, sp + 2 * sz - i);
      if (ml[sapos] + i >= sz) ml[sapos] = 0;
      if (ml[rcsapos] >= i) ml[rcsapos] = 0;
      out[w++] = (uint8_t)(ml[rcsapos] < 255 ? ml[rcsapos] : 255);
      out[w++] = (uint8_t)(ml[sapos] < 255 ? ml[sapos] : 255);
    }
  }
  free(ml);
  return 0;
}

static uint64_t min_len_at(const orc_index *ix, uint64_t r) {   /* :628-641 */
  const uint64_t a = lcp_exact(ix, r, NULL);
  const uint64_t b = r + 1 < ix->N ? lcp_exact(ix, r + 1, NULL) : 0;
  return (a > b ? a : b) + 1;
}

uint64_t orc_mappability_range(const orc_index *ix, uint64_t g0, uint64_t g1,
                               uint32_t k, uint8_t *out) {
  uint64_t g = 0, w = 0, uniq = 0;
  for (uint32_t chrom = 0; chrom < ix->n_seq && g < g1; chrom += 2) {
    const uint64_t sp = ix->startpos[chrom], sz = ix->sizes[chrom];
    const uint64_t a = g0 > g ? g0 - g : 0, b = g1 < g + sz ? g1 - g : sz;
    for (uint64_t i = a; i < b; ++i) {
      const uint64_t sapos = idx_at(ix, ix->ISA, ix->idx_bytes, i + sp);
      const uint64_t rcsapos = idx_at(ix, ix->ISA, ix->idx_bytes, sp + 2 * sz - i);
      uint64_t right = min_len_at(ix, sapos), left = min_len_at(ix, rcsapos);
      if (right + i >= sz) right = 0;                  /* :666 */
      if (left >= i) left = 0;                         /* :667 */
      if (right > 255) right = 255;
      out[w++] = (uint8_t)(left < 255 ? left : 255);
      out[w++] = (uint8_t)right;
      uniq += right >= 1 && right <= k;
    }
    g += sz;
  }
  return uniq;
}

/* ======================================================================== */
/* mappability_tag (mappability_tag.cpp:81-124)                              */
/* ======================================================================== */

static inline unsigned mapbyte(const uint8_t *map, uint64_t size, uint64_t at) {
  return at < size ? map[at] : 0;  /* past EOF inside the mmap page reads 0 */
}

int orc_tag(orc_hit *h, const uint32_t *offsets, const uint8_t *map,
            uint64_t map_size, int small_chr) {
  const uint32_t abspos = offsets[h->tid] + (uint32_t)(h->pos + 1);
  /* walk the CIGAR text exactly like the istringstream loop (:95-122) */
  const char *c = h->cigar;
  int offset = 0, uindex = 0, err = 0;
  while (*c) {
    uint32_t count = 0;
    while (*c >= '0' && *c <= '9') { count = count * 10 + (uint32_t)(*c - '0'); ++c; }
    char code = *c++;
    if (code == '=') {
      const uint32_t li = abspos + (uint32_t)offset + count - 1;
      const unsigned left_m = mapbyte(map, map_size, 2 + li * 2ull);
      const unsigned left = left_m ? left_m - 1 : 255;
      const uint32_t ri = abspos + (uint32_t)offset - 1;
      const unsigned right_m = mapbyte(map, map_size, 2 + ri * 2ull + 1);
      const unsigned right = right_m ? right_m : 255;
      if (uindex == 0) { h->L0 = (int32_t)left; h->R0 = (int32_t)right; }
      if (!err && left > count && !small_chr) err = 1;
      if (!err && right > count && !small_chr) err = 2;
      ++uindex;
    }
    offset += (int)count;
  }
  return err;
}

/* ======================================================================== */
/* smashMEM.py (smashMEM.py:84-92,154-228) with args 0 0 10000 4             */
/* ======================================================================== */

int orc_smash_pair(const orc_hit *h1, uint32_t n1, const orc_hit *h2,
                   uint32_t n2, int min_excess, int64_t hit_window,
                   uint32_t *out_tid, int64_t *out_pos) {
  uint32_t k1[ORC_MAX_MATCH], k2[ORC_MAX_MATCH], m1 = 0, m2 = 0;
  if (n1 > ORC_MAX_MATCH || n2 > ORC_MAX_MATCH) return -2;   /* never truncate */
  for (uint32_t i = 0; i < n1; ++i) {
    int qlen = (int)h1[i].qend - (int)h1[i].qstart;
    int mx = h1[i].L0 > h1[i].R0 ? h1[i].L0 : h1[i].R0;
    if (qlen - mx >= min_excess) k1[m1++] = i;
  }
  for (uint32_t i = 0; i < n2; ++i) {
    int qlen = (int)h2[i].qend - (int)h2[i].qstart;
    int mx = h2[i].L0 > h2[i].R0 ? h2[i].L0 : h2[i].R0;
    if (qlen - mx >= min_excess) k2[m2++] = i;
  }
  if (m1 == 0 && m2 == 0) return -1;                   /* smashMEM.py:162 */
  int n = 0;
  for (uint32_t a = 0; a < m1; ++a) {                  /* HI order already */
    out_tid[n] = h1[k1[a]].tid;
    out_pos[n] = h1[k1[a]].pos;
    ++n;
  }
  for (uint32_t b = 0; b < m2; ++b) {                  /* :193-208 */
    const orc_hit *x = &h2[k2[b]];
    int close = 0;
    for (uint32_t a = 0; a < m1; ++a) {
      int64_t d = h1[k1[a]].pos - x->pos;
      if (d < 0) d = -d;
      if (h1[k1[a]].tid == x->tid && d < hit_window) { close = 1; break; }
    }
    if (!close) {
      out_tid[n] = x->tid;
      out_pos[n] = x->pos;
      ++n;
    }
  }
  return n;
}

/* ======================================================================== */
/* varbin.py main loop (varbin.py:52-92)                                    */
/* ======================================================================== */

void orc_varbin(const int64_t *pos0, const int64_t *abspos, uint64_t n,
                const int64_t *bin_starts, uint32_t nbins, uint64_t *counts,
                orc_varbin_state *st) {
  for (uint64_t k = 0; k < n; ++k) {
    st->total++;
    if (st->prev_pos >= 0 && pos0[k] == st->prev_pos) { st->dups++; continue; }
    /* bisect.bisect_right(binStarts, abspos) */
    uint32_t lo = 0, hi = nbins;
    while (lo < hi) {
      uint32_t mid = (lo + hi) / 2;
      if (abspos[k] < bin_starts[mid]) hi = mid; else lo = mid + 1;
    }
    uint32_t b = lo == 0 ? nbins - 1 : lo - 1;          /* binCounts[-1] */
    counts[b]++;
    st->kept++;
    st->prev_pos = pos0[k];
  }
}

/* ======================================================================== */
/* global pair de-dup set (smashMEM.py:149,217-228)                         */
/* ======================================================================== */

struct orc_dedup {
  uint64_t cap, n;
  uint64_t *hash;
  uint8_t **key;
  uint32_t *klen;
};

orc_dedup *orc_dedup_new(void) {
  orc_dedup *d = (orc_dedup *)calloc(1, sizeof(orc_dedup));
  d->cap = 1 << 16;
  d->hash = (uint64_t *)calloc(d->cap, 8);
  d->key = (uint8_t **)calloc(d->cap, sizeof(uint8_t *));
  d->klen = (uint32_t *)calloc(d->cap, 4);
  return d;
}
void orc_dedup_free(orc_dedup *d) {
  if (!d) return;
  for (uint64_t i = 0; i < d->cap; ++i) free(d->key[i]);
  free(d->hash); free(d->key); free(d->klen); free(d);
}
static uint64_t fnv(const uint8_t *p, uint32_t n) {
  uint64_t h = 1469598103934665603ull;
  for (uint32_t i = 0; i < n; ++i) { h ^= p[i]; h *= 1099511628211ull; }
  return h | 1;
}
static int dedup_insert(orc_dedup *d, const uint8_t *k, uint32_t n);
static void dedup_grow(orc_dedup *d) {
  orc_dedup o = *d;
  d->cap *= 2; d->n = 0;
  d->hash = (uint64_t *)calloc(d->cap, 8);
  d->key = (uint8_t **)calloc(d->cap, sizeof(uint8_t *));
  d->klen = (uint32_t *)calloc(d->cap, 4);
  for (uint64_t i = 0; i < o.cap; ++i)
    if (o.hash[i]) { dedup_insert(d, o.key[i], o.klen[i]); free(o.key[i]); }
  free(o.hash); free(o.key); free(o.klen);
}
/* returns 1 if newly inserted, 0 if already present */
static int dedup_insert(orc_dedup *d, const uint8_t *k, uint32_t n) {
  if (2 * (d->n + 1) > d->cap) dedup_grow(d);
  uint64_t h = fnv(k, n), i = h & (d->cap - 1);
  while (d->hash[i]) {
    if (d->hash[i] == h && d->klen[i] == n && !memcmp(d->key[i], k, n)) return 0;
    i = (i + 1) & (d->cap - 1);
  }
  d->hash[i] = h;
  d->key[i] = (uint8_t *)malloc(n ? n : 1);
  memcpy(d->key[i], k, n);
  d->klen[i] = n;
  d->n++;
  return 1;
}

/* ======================================================================== */
/* whole chain                                                               */
/* ======================================================================== */

#define PAIR_CAP (2 * ORC_MAX_MATCH)   /* kept hits of a pair: <= hits(r1) + hits(r2) */
#define PAIR_CHUNK 16384               /* pairs per worker round (bounds the out arrays) */
typedef struct {
  int32_t nkept;          /* -1: no key */
  int32_t err;
  uint32_t tid[PAIR_CAP];
  int64_t pos[PAIR_CAP];
} pair_out_t;

typedef struct {
  const orc_pipeline *p;
  const uint8_t *reads;
  uint32_t L;
  uint64_t stride, begin, end;
  pair_out_t *out;
} job_t;

/* every capacity below holds the largest possible input (reads <= 255 bp:
 * <= 254 matches, hits <= matches); exceeding one is an error, never a cut */
static void process_mate(const orc_pipeline *p, const uint8_t *P, uint32_t L,
                         orc_hit *hits, uint32_t *nh, int *err) {
  orc_match m[ORC_MAX_MATCH];
  *nh = 0;
  int n = orc_mam(p->ix, P, L, p->min_len, m, ORC_MAX_MATCH, NULL);
  if (n > ORC_MAX_MATCH) { if (!*err) *err = ORC_ERR_CAP; return; }
  uint32_t bt; int64_t bp;
  int k = orc_resolve(p->ix, P, L, m, (uint32_t)n, hits, ORC_MAX_MATCH, &bt, &bp);
  if (k < 0) { if (!*err) *err = ORC_ERR_CAP; return; }
  for (int i = 0; i < k; ++i) {
    int e = orc_tag(&hits[i], p->tag_offsets, p->map, p->map_size,
                    p->small_chr[hits[i].tid]);
    if (e && !*err) *err = e;
  }
  *nh = (uint32_t)k;
}

static void *pair_worker(void *arg) {
  job_t *j = (job_t *)arg;
  const orc_pipeline *p = j->p;
  orc_hit *h1 = (orc_hit *)malloc(2 * ORC_MAX_MATCH * sizeof(orc_hit));
  orc_hit *h2 = h1 + ORC_MAX_MATCH;
  for (uint64_t q = j->begin; q < j->end; ++q) {
    uint32_t n1 = 0, n2 = 0;
    int err = 0;
    process_mate(p, j->reads + (2 * q) * j->stride, j->L, h1, &n1, &err);
    process_mate(p, j->reads + (2 * q + 1) * j->stride, j->L, h2, &n2, &err);
    pair_out_t *o = &j->out[q - j->begin];
    o->err = err;
    o->nkept = orc_smash_pair(h1, n1, h2, n2, 4, 10000, o->tid, o->pos);
    if (o->nkept < -1) { o->err = ORC_ERR_CAP; o->nkept = -1; }
  }
  free(h1);
  return NULL;
}

int orc_run_pairs(const orc_pipeline *p, const uint8_t *reads, uint32_t L,
                  uint64_t stride, uint64_t n_pairs, int threads,
                  orc_dedup *dedup, uint64_t *counts, orc_varbin_state *st,
                  uint64_t *n_dupe_pairs, uint64_t *n_pos_out) {
  if (threads < 1) threads = 1;
  const uint64_t chunk = n_pairs < PAIR_CHUNK * (uint64_t)threads ? (n_pairs ? n_pairs : 1)
                                                                    : PAIR_CHUNK * (uint64_t)threads;
  pair_out_t *out = (pair_out_t *)malloc(chunk * sizeof(pair_out_t));
  pthread_t th[1024];
  job_t jobs[1024];
  if (threads > 1024) threads = 1024;
  int err = 0;
  uint8_t key[PAIR_CAP * 12 + 4];
  int64_t pos0[PAIR_CAP], absp[PAIR_CAP];
  for (uint64_t c0 = 0; c0 < n_pairs; c0 += chunk) {
    const uint64_t cn = n_pairs - c0 < chunk ? n_pairs - c0 : chunk;
    for (int t = 0; t < threads; ++t) {
      jobs[t].p = p; jobs[t].reads = reads; jobs[t].L = L; jobs[t].stride = stride;
      jobs[t].begin = c0 + cn * (uint64_t)t / (uint64_t)threads;
      jobs[t].end = c0 + cn * (uint64_t)(t + 1) / (uint64_t)threads;
      jobs[t].out = out + (jobs[t].begin - c0);
      pthread_create(&th[t], NULL, pair_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    for (uint64_t q = 0; q < cn; ++q) {
      pair_out_t *o = &out[q];
      if (o->err && !err) err = o->err;
      if (o->nkept < 0) continue;
      uint32_t kl = 0;
      for (int32_t i = 0; i < o->nkept; ++i) {
        memcpy(key + kl, &o->tid[i], 4); kl += 4;
        memcpy(key + kl, &o->pos[i], 8); kl += 8;
      }
      if (!dedup_insert(dedup, key, kl)) { if (n_dupe_pairs) (*n_dupe_pairs)++; continue; }
      uint64_t np = 0;
      for (int32_t i = 0; i < o->nkept; ++i) {
        if (!p->major[o->tid[i]]) continue;
        pos0[np] = o->pos[i];
        absp[np] = o->pos[i] + p->chrom_off[o->tid[i]];
        ++np;
      }
      if (n_pos_out) *n_pos_out += np;
      orc_varbin(pos0, absp, np, p->bin_starts, p->nbins, counts, st);
    }
  }
  free(out);
  return err;
}

typedef struct {
  const orc_index *ix;
  const uint8_t *reads;
  uint32_t L, min_len;
  uint64_t stride, begin, end, total;
  orc_counters ctr;
  int count;
} mjob_t;

static void *map_worker(void *arg) {
  mjob_t *j = (mjob_t *)arg;
  orc_match m[256];
  memset(&j->ctr, 0, sizeof(j->ctr));
  j->ctr.last_sa = j->ctr.last_isa = j->ctr.last_ref = j->ctr.last_lcp = ~0ull;
  j->ctr.last_kt = j->ctr.last_u = j->ctr.last_bm = ~0ull;
  for (uint64_t q = j->begin; q < j->end; ++q)
    j->total += (uint64_t)orc_mam(j->ix, j->reads + q * j->stride, j->L,
                                  j->min_len, m, 256, j->count ? &j->ctr : NULL);
  return NULL;
}

uint64_t orc_map_only(const orc_index *ix, const uint8_t *reads, uint32_t L,
                      uint64_t stride, uint64_t n, uint32_t min_len,
                      int threads, orc_counters *ctr) {
  if (threads < 1) threads = 1;
  if (threads > 1024) threads = 1024;
  pthread_t th[1024];
  mjob_t *jobs = (mjob_t *)calloc((size_t)threads, sizeof(mjob_t));
  for (int t = 0; t < threads; ++t) {
    jobs[t].ix = ix; jobs[t].reads = reads; jobs[t].L = L; jobs[t].min_len = min_len;
    jobs[t].stride = stride;
    jobs[t].begin = n * (uint64_t)t / (uint64_t)threads;
    jobs[t].end = n * (uint64_t)(t + 1) / (uint64_t)threads;
    jobs[t].count = ctr != NULL;
    pthread_create(&th[t], NULL, map_worker, &jobs[t]);
  }
  uint64_t total = 0;
  if (ctr) memset(ctr, 0, sizeof(*ctr));
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    total += jobs[t].total;
    if (ctr) {
      ctr->sa_loads += jobs[t].ctr.sa_loads; ctr->sa_lines += jobs[t].ctr.sa_lines;
      ctr->isa_loads += jobs[t].ctr.isa_loads; ctr->isa_lines += jobs[t].ctr.isa_lines;
      ctr->ref_loads += jobs[t].ctr.ref_loads; ctr->ref_lines += jobs[t].ctr.ref_lines;
      ctr->lcp_loads += jobs[t].ctr.lcp_loads; ctr->lcp_lines += jobs[t].ctr.lcp_lines;
      ctr->ovf_lookups += jobs[t].ctr.ovf_lookups;
    }
  }
  free(jobs);
  return total;
}

/* ======================================================================== */
/* accelerated search (device SMASH_MODE_MAM), restated for checking        */
/* ======================================================================== */

uint32_t orc_accel_k(uint64_t N) {
  uint32_t K = 4;                       /* aux_build.hip: floor(log4 N), <= 16 */
  while (K < 16 && (1ull << (2 * (K + 1))) <= N) ++K;
  return K;
}

static int acgt(uint8_t c) {
  return c == 'a' ? 0 : c == 'c' ? 1 : c == 'g' ? 2 : c == 't' ? 3 : -1;
}

void orc_build_accel(const orc_index *ix, uint32_t K, uint8_t *U, uint64_t *KT) {
  const uint64_t N = ix->N;
  const uint32_t isz = ix->idx_bytes == 4 ? 4 : 8;
  for (uint64_t x = 0; x < N; ++x) {
    const uint64_t r = idx_at(ix, ix->ISA, isz, x);
    const uint8_t a = ix->L8[r], b = r + 1 < N ? ix->L8[r + 1] : 0;
    U[x] = a > b ? a : b;
  }
  memset(U + N, 0, 64);
  const uint64_t nk = 1ull << (2 * K);
  for (uint64_t w = 0; w < nk; ++w) { KT[2 * w] = 1; KT[2 * w + 1] = 0; }
  uint64_t prev = ~0ull;
  for (uint64_t r = 0; r < N; ++r) {
    const uint64_t x = idx_at(ix, ix->SA, isz, r);
    uint64_t code = 0;
    int ok = x + K <= N;
    for (uint32_t k = 0; ok && k < K; ++k) {
      int v = acgt(ix->T[x + k]);
      if (v < 0) ok = 0;
      code = (code << 2) | (uint64_t)(v & 3);
    }
    if (!ok) { prev = ~0ull; continue; }
    if (code != prev) KT[2 * code] = r;
    KT[2 * code + 1] = r;
    prev = code;
  }
}

/* k-mer table with the (K+2)-mer presence bits (aux_build.hip k_kfilter
 * restated): every ACGT (K+2)-mer b0 .. b(K+1) of the text sets bit
 * b(K)*4+b(K+1) of the entry of b0..b(K-1), bit 16+b0*4+b(K+1) of b1..b(K)'s
 * and bit 32+b0*4+b1 of b2..b(K+1)'s; filter bit f is bit 40 + f % 24 of word
 * f / 24. */
static void ktf_set(uint64_t *E, uint64_t w, uint32_t f) {
  E[2 * w + (f >= 24)] |= 1ull << (40 + (f >= 24 ? f - 24 : f));
}

void orc_build_ktf(const orc_index *ix, uint32_t K, const uint64_t *KT, uint64_t *KTF) {
  const uint64_t nk = 1ull << (2 * K), mask = nk - 1;
  memcpy(KTF, KT, 16 * nk);
  const uint64_t N = ix->N;
  uint64_t c = 0;
  uint32_t run = 0;   /* consecutive ACGT bytes ending at x */
  for (uint64_t x = 0; x < N; ++x) {
    const int v = acgt(ix->T[x]);
    if (v < 0) { run = 0; c = 0; continue; }
    c = (c << 2) | (uint64_t)v;          /* (only the low 2K + 4 bits are used) */
    if (++run < K + 2) continue;
    const uint64_t b = c & ((1ull << (2 * K + 4)) - 1);   /* the (K+2)-mer ending at x */
    const uint32_t b0 = (uint32_t)(b >> (2 * K + 2)) & 3, b1 = (uint32_t)(b >> (2 * K)) & 3;
    const uint32_t r1 = (uint32_t)(b >> 2) & 3, r2 = (uint32_t)b & 3;
    ktf_set(KTF, b >> 4, r1 * 4 + r2);
    ktf_set(KTF, (b >> 2) & mask, 16 + b0 * 4 + r2);
    ktf_set(KTF, b & mask, 32 + b0 * 4 + b1);
  }
}

int orc_mam_fast(const orc_index *ix, const orc_accel *acc, const uint8_t *P,
                 uint32_t L, uint32_t min_len, orc_match *out, uint32_t cap,
                 orc_counters *ctr) {
  ctx_t x = mkctx(ix, ctr);
  sink_t s = {out, cap, 0};
  const uint64_t N = ix->N;
  const uint32_t K = acc->K;
  ival_t cur = {0, 0, N - 1};
  uint64_t prefix = 0, pos = 0;
  int have_pos = 0;
  while (prefix < L) {
    if (cur.depth == 0 && prefix + K <= L) {                 /* (C) */
      uint64_t w = 0;
      int ok = 1;
      for (uint32_t k = 0; k < K; ++k) {
        int v = acgt(P[prefix + k]);
        if (v < 0) ok = 0;
        w = (w << 2) | (uint64_t)(v & 3);
      }
      if (ok) {
        if (ctr) tick(&ctr->sa_loads, &ctr->kt_lines, &ctr->last_kt, 16 * w);
        const uint64_t lo = acc->KT[2 * w], hi = acc->KT[2 * w + 1];
        if (lo <= hi) { cur.depth = K; cur.start = lo; cur.end = hi; have_pos = 0; }
      }
    }
    if (cur.depth < L) {
      while (prefix + cur.depth < L) {
        if (cur.start == cur.end) {                          /* (A) */
          if (!have_pos) { pos = SAat(&x, cur.start); have_pos = 1; }
          while (prefix + cur.depth < L) {
            if (ctr) tick(&ctr->ref_loads, &ctr->ref_lines, &ctr->last_ref, pos + cur.depth);
            const uint64_t rem = L - prefix - cur.depth;
            const uint32_t lim = rem < 8 ? (uint32_t)rem : 8u;
            uint32_t k = 0;
            while (k < lim && P[prefix + cur.depth + k] == ix->T[pos + cur.depth + k]) ++k;
            cur.depth += k;
            if (k < lim) break;
          }
          break;
        }
        uint64_t st = cur.start, en = cur.end;
        if (!td_faster(&x, (int64_t)(int8_t)P[prefix + cur.depth], cur.depth, &st, &en)) break;
        cur.depth += 1; cur.start = st; cur.end = en; have_pos = 0;
        if (cur.depth == L) break;
      }
    }
    if (cur.depth <= 1) {
      cur.depth = 0; cur.start = 0; cur.end = N - 1; have_pos = 0;
      ++prefix;
      continue;
    }
    if (cur.start == cur.end) {
      if (!have_pos) { pos = SAat(&x, cur.start); have_pos = 1; }
      if (cur.depth >= min_len) {
        int lm = (prefix == 0 || pos == 0) ? 1
                 : ((int64_t)(int8_t)P[prefix - 1] != Tat(&x, pos - 1));
        if (lm) emit(&s, pos, prefix, cur.depth);
      }
      const uint64_t d = cur.depth;                          /* (B) */
      uint64_t j = 1;
      int hit = 0;
      while (j < d) {
        if (ctr) tick(&ctr->lcp_loads, &ctr->u_lines, &ctr->last_u, pos + j);
        const uint64_t rem = d - j;
        const uint32_t lim = rem < 8 ? (uint32_t)rem : 8u;
        uint32_t k = 0;
        while (k < lim && (uint64_t)acc->U[pos + j + k] < d - j - k) ++k;
        if (k < lim) { j += k; hit = 1; break; }
        j += lim;
      }
      prefix += j;
      if (!hit) { cur.depth = 0; cur.start = 0; cur.end = N - 1; have_pos = 0; continue; }
      cur.depth = d - j;
      cur.start = cur.end = ISAat(&x, pos + j);
      have_pos = 0;
      if (!expand_link(&x, &cur)) { cur.depth = 0; cur.start = 0; cur.end = N - 1; }
      continue;
    }
    cur.depth -= 1;
    cur.start = ISAat(&x, SAat(&x, cur.start) + 1);
    cur.end = ISAat(&x, SAat(&x, cur.end) + 1);
    ++prefix;
    have_pos = 0;
    if (cur.depth == 0 || !expand_link(&x, &cur)) { cur.depth = 0; cur.start = 0; cur.end = N - 1; }
  }
  return (int)s.n;
}

typedef struct {
  const orc_index *ix;
  const orc_accel *acc;
  const uint8_t *reads;
  uint32_t L, min_len;
  uint64_t stride, begin, end, total;
  orc_counters ctr;
  int count;
} fjob_t;

static void *fast_worker(void *arg) {
  fjob_t *j = (fjob_t *)arg;
  orc_match m[256];
  memset(&j->ctr, 0, sizeof(j->ctr));
  j->ctr.last_sa = j->ctr.last_isa = j->ctr.last_ref = j->ctr.last_lcp = ~0ull;
  j->ctr.last_kt = j->ctr.last_u = j->ctr.last_bm = ~0ull;
  for (uint64_t q = j->begin; q < j->end; ++q)
    j->total += (uint64_t)orc_mam_fast(j->ix, j->acc, j->reads + q * j->stride, j->L,
                                       j->min_len, m, 256, j->count ? &j->ctr : NULL);
  return NULL;
}

uint64_t orc_map_only_fast(const orc_index *ix, const orc_accel *acc,
                           const uint8_t *reads, uint32_t L, uint64_t stride,
                           uint64_t n, uint32_t min_len, int threads,
                           orc_counters *ctr) {
  if (threads < 1) threads = 1;
  if (threads > 1024) threads = 1024;
  pthread_t th[1024];
  fjob_t *jobs = (fjob_t *)calloc((size_t)threads, sizeof(fjob_t));
  for (int t = 0; t < threads; ++t) {
    jobs[t].ix = ix; jobs[t].acc = acc; jobs[t].reads = reads; jobs[t].L = L;
    jobs[t].min_len = min_len; jobs[t].stride = stride;
    jobs[t].begin = n * (uint64_t)t / (uint64_t)threads;
    jobs[t].end = n * (uint64_t)(t + 1) / (uint64_t)threads;
    jobs[t].count = ctr != NULL;
    pthread_create(&th[t], NULL, fast_worker, &jobs[t]);
  }
  uint64_t total = 0;
  if (ctr) memset(ctr, 0, sizeof(*ctr));
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    total += jobs[t].total;
    if (ctr) {
      ctr->sa_lines += jobs[t].ctr.sa_lines; ctr->isa_lines += jobs[t].ctr.isa_lines;
      ctr->ref_lines += jobs[t].ctr.ref_lines; ctr->lcp_lines += jobs[t].ctr.lcp_lines;
      ctr->kt_lines += jobs[t].ctr.kt_lines; ctr->u_lines += jobs[t].ctr.u_lines;
      ctr->sa_loads += jobs[t].ctr.sa_loads; ctr->isa_loads += jobs[t].ctr.isa_loads;
      ctr->ref_loads += jobs[t].ctr.ref_loads; ctr->lcp_loads += jobs[t].ctr.lcp_loads;
    }
  }
  free(jobs);
  return total;
}

/* ======================================================================== */
/* v3: per-position evaluation                                              */
/* ======================================================================== */

uint32_t orc_accel_b(uint64_t N) {
  uint32_t B = 8;
  while (B < 18 && (1ull << (2 * (B - 1))) <= N) ++B;
  return B;
}

void orc_build_bitmap(const orc_index *ix, uint32_t B, uint64_t *BM, uint8_t *in_text) {
  const uint64_t N = ix->N;
  memset(BM, 0, ((1ull << (2 * B)) / 64 + 1) * 8);
  memset(in_text, 0, 256);
  uint64_t code = 0, mask = (1ull << (2 * B)) - 1;
  uint32_t run = 0;    /* consecutive ACGT chars ending at x */
  for (uint64_t x = 0; x < N; ++x) {
    in_text[ix->T[x]] = 1;
    int v = acgt(ix->T[x]);
    if (v < 0) { run = 0; code = 0; continue; }
    code = ((code << 2) | (uint64_t)v) & mask;
    if (++run >= B) BM[code >> 6] |= 1ull << (code & 63);
  }
}

#define V3_SCAN 32

/* window filter: can P[p .. p+min_len) occur in the text at all?  0 = no
 * (then ms(p) < min_len and p cannot emit). */
static int v3_window(const orc_accel *acc, const uint8_t *P, uint64_t p,
                     uint32_t min_len, orc_counters *ctr, uint64_t *next_p) {
  *next_p = p + 1;
  for (uint64_t k = p + min_len; k-- > p;)
    if (!acc->in_text[P[k]]) { *next_p = k + 1; return 0; }
  const uint32_t B = acc->B;
  if (B > min_len) return 1;
  const uint64_t bmask = (1ull << (2 * B)) - 1;
  for (int end = 0; end < 2; ++end) {
    const uint64_t q = end ? p + min_len - B : p;
    uint64_t code = 0;
    for (uint32_t k = 0; k < B; ++k) {
      int v = acgt(P[q + k]);
      if (v < 0) return 1;          /* non-ACGT text byte: no bitmap verdict */
      code = ((code << 2) | (uint64_t)v) & bmask;
    }
    if (ctr) tick(&ctr->sa_loads, &ctr->bm_lines, &ctr->last_bm, code >> 3);
    if (!((acc->BM[code >> 6] >> (code & 63)) & 1)) return 0;
  }
  return 1;
}

/* final state of a traverse over a small interval: each candidate suffix is
 * compared with P directly (independent loads); the suffixes sharing the
 * longest match form the new interval (contiguous in SA order). */
static void v3_scan(const ctx_t *x, const uint8_t *P, uint64_t L, uint64_t p,
                    ival_t *cur, uint64_t *pos) {
  int64_t best = -1;
  uint64_t bl = cur->start, bh = cur->start, bpos = 0;
  const uint64_t d = cur->depth, rem = L - p - d;
  for (uint64_t m = cur->start; m <= cur->end; ++m) {
    const uint64_t sp = SAat(x, m);
    uint64_t l = 0;
    while (l < rem) {
      if (x->c) tick(&x->c->ref_loads, &x->c->ref_lines, &x->c->last_ref, sp + d + l);
      uint32_t k = 0;
      const uint32_t lim = rem - l < 8 ? (uint32_t)(rem - l) : 8u;
      while (k < lim && P[p + d + l + k] == x->ix->T[sp + d + l + k]) ++k;
      l += k;
      if (k < lim) break;
    }
    if ((int64_t)l > best) { best = (int64_t)l; bl = bh = m; bpos = sp; }
    else if ((int64_t)l == best) bh = m;
  }
  cur->depth = d + (uint64_t)best;
  cur->start = bl;
  cur->end = bh;
  *pos = bpos;
}

int orc_mam_v3(const orc_index *ix, const orc_accel *acc, const uint8_t *P,
               uint32_t L, uint32_t min_len, orc_match *out, uint32_t cap,
               orc_counters *ctr) {
  ctx_t x = mkctx(ix, ctr);
  sink_t s = {out, cap, 0};
  const uint64_t N = ix->N;
  const uint32_t K = acc->K;
  ival_t cur = {0, 0, N - 1};
  uint64_t prefix = 0, pos = 0;
  int have_pos = 0;
  while (prefix < L) {
    /* (F) a shallow state can be dropped at any prefix whose min_len window
     * does not occur: ms(prefix) < min_len, nothing is emitted there */
    if (cur.depth < min_len) {
      if (prefix + min_len > L) break;
      uint64_t nxt;
      if (!v3_window(acc, P, prefix, min_len, ctr, &nxt)) {
        cur.depth = 0; cur.start = 0; cur.end = N - 1; have_pos = 0;
        prefix = nxt;
        continue;
      }
    }
    if (cur.depth == 0 && prefix + K <= L) {                 /* (C) */
      uint64_t w = 0;
      int ok = 1;
      for (uint32_t k = 0; k < K; ++k) {
        int v = acgt(P[prefix + k]);
        if (v < 0) ok = 0;
        w = (w << 2) | (uint64_t)(v & 3);
      }
      if (ok) {
        if (ctr) tick(&ctr->sa_loads, &ctr->kt_lines, &ctr->last_kt, 16 * w);
        const uint64_t lo = acc->KT[2 * w], hi = acc->KT[2 * w + 1];
        if (lo <= hi) { cur.depth = K; cur.start = lo; cur.end = hi; have_pos = 0; }
      }
    }
    if (cur.depth < L) {
      while (prefix + cur.depth < L) {
        if (cur.start == cur.end) {                          /* (A) */
          if (!have_pos) { pos = SAat(&x, cur.start); have_pos = 1; }
          while (prefix + cur.depth < L) {
            if (ctr) tick(&ctr->ref_loads, &ctr->ref_lines, &ctr->last_ref, pos + cur.depth);
            const uint64_t rem = L - prefix - cur.depth;
            const uint32_t lim = rem < 8 ? (uint32_t)rem : 8u;
            uint32_t k = 0;
            while (k < lim && P[prefix + cur.depth + k] == ix->T[pos + cur.depth + k]) ++k;
            cur.depth += k;
            if (k < lim) break;
          }
          break;
        }
        if (cur.end - cur.start + 1 <= V3_SCAN) {            /* (S) */
          v3_scan(&x, P, L, prefix, &cur, &pos);
          have_pos = cur.start == cur.end;
          break;
        }
        uint64_t st = cur.start, en = cur.end;
        if (!td_faster(&x, (int64_t)(int8_t)P[prefix + cur.depth], cur.depth, &st, &en)) break;
        cur.depth += 1; cur.start = st; cur.end = en; have_pos = 0;
        if (cur.depth == L) break;
      }
    }
    if (cur.depth <= 1) {
      cur.depth = 0; cur.start = 0; cur.end = N - 1; have_pos = 0;
      ++prefix;
      continue;
    }
    if (cur.start == cur.end) {
      if (!have_pos) { pos = SAat(&x, cur.start); have_pos = 1; }
      if (cur.depth >= min_len) {
        int lm = (prefix == 0 || pos == 0) ? 1
                 : ((int64_t)(int8_t)P[prefix - 1] != Tat(&x, pos - 1));
        if (lm) emit(&s, pos, prefix, cur.depth);
      }
      const uint64_t d = cur.depth;                          /* (B) */
      uint64_t j = 1;
      int hit = 0;
      while (j < d) {
        if (ctr) tick(&ctr->lcp_loads, &ctr->u_lines, &ctr->last_u, pos + j);
        const uint64_t rem = d - j;
        const uint32_t lim = rem < 8 ? (uint32_t)rem : 8u;
        uint32_t k = 0;
        while (k < lim && (uint64_t)acc->U[pos + j + k] < d - j - k) ++k;
        if (k < lim) { j += k; hit = 1; break; }
        j += lim;
      }
      prefix += j;
      if (!hit) { cur.depth = 0; cur.start = 0; cur.end = N - 1; have_pos = 0; continue; }
      cur.depth = d - j;
      cur.start = cur.end = ISAat(&x, pos + j);
      have_pos = 0;
      if (!expand_link(&x, &cur)) { cur.depth = 0; cur.start = 0; cur.end = N - 1; }
      continue;
    }
    cur.depth -= 1;
    cur.start = ISAat(&x, SAat(&x, cur.start) + 1);
    cur.end = ISAat(&x, SAat(&x, cur.end) + 1);
    ++prefix;
    have_pos = 0;
    if (cur.depth == 0 || !expand_link(&x, &cur)) { cur.depth = 0; cur.start = 0; cur.end = N - 1; }
  }
  return (int)s.n;
}

typedef struct {
  const orc_index *ix;
  const orc_accel *acc;
  const uint8_t *reads;
  uint32_t L, min_len;
  uint64_t stride, begin, end, total;
  orc_counters ctr;
  int count;
} v3job_t;

static void *v3_worker(void *arg) {
  v3job_t *j = (v3job_t *)arg;
  orc_match m[256];
  memset(&j->ctr, 0, sizeof(j->ctr));
  j->ctr.last_sa = j->ctr.last_isa = j->ctr.last_ref = j->ctr.last_lcp = ~0ull;
  j->ctr.last_kt = j->ctr.last_u = j->ctr.last_bm = ~0ull;
  for (uint64_t q = j->begin; q < j->end; ++q)
    j->total += (uint64_t)orc_mam_v3(j->ix, j->acc, j->reads + q * j->stride, j->L,
                                     j->min_len, m, 256, j->count ? &j->ctr : NULL);
  return NULL;
}

uint64_t orc_map_only_v3(const orc_index *ix, const orc_accel *acc,
                         const uint8_t *reads, uint32_t L, uint64_t stride,
                         uint64_t n, uint32_t min_len, int threads,
                         orc_counters *ctr) {
  if (threads < 1) threads = 1;
  if (threads > 1024) threads = 1024;
  pthread_t th[1024];
  v3job_t *jobs = (v3job_t *)calloc((size_t)threads, sizeof(v3job_t));
  for (int t = 0; t < threads; ++t) {
    jobs[t].ix = ix; jobs[t].acc = acc; jobs[t].reads = reads; jobs[t].L = L;
    jobs[t].min_len = min_len; jobs[t].stride = stride;
    jobs[t].begin = n * (uint64_t)t / (uint64_t)threads;
    jobs[t].end = n * (uint64_t)(t + 1) / (uint64_t)threads;
    jobs[t].count = ctr != NULL;
    pthread_create(&th[t], NULL, v3_worker, &jobs[t]);
  }
  uint64_t total = 0;
  if (ctr) memset(ctr, 0, sizeof(*ctr));
  for (int t = 0; t < threads; ++t) {
    pthread_join(th[t], NULL);
    total += jobs[t].total;
    if (ctr) {
      ctr->sa_lines += jobs[t].ctr.sa_lines; ctr->isa_lines += jobs[t].ctr.isa_lines;
      ctr->ref_lines += jobs[t].ctr.ref_lines; ctr->lcp_lines += jobs[t].ctr.lcp_lines;
      ctr->kt_lines += jobs[t].ctr.kt_lines; ctr->u_lines += jobs[t].ctr.u_lines;
      ctr->bm_lines += jobs[t].ctr.bm_lines;
    }
  }
  free(jobs);
  return total;
}
