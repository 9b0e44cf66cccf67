// smash-paper_amd/csrc/ingest.cpp -- native read ingest for the device batches.
//
// Replaces the `zcat r1s | fastqs_to_sam ... | samtools sort -n` front of
// smash_mapping.sh:19-23 for the counting path:
//  * smash_fastq_*: the FASTQ/FASTA lists of both mates (gzip or plain, zlib
//    reads both), parsed as fastqs_to_sam.cpp:48-96 does (blank lines
//    skipped, '@'/'>' records, name = first token after the marker, '+' line
//    and qualities for '@' records, a pair whose two mates have no bases
//    dropped, a pair with ONE empty mate rejected), with
//    replaceN (N -> Z, fastqs_to_sam.cpp:74 with argc == 4) and the
//    NewQuery::extend lowercasing (query.cpp:125-144) applied on the way into
//    the caller's (pinned) mate matrix: mate 2q = read 1, 2q + 1 = read 2.
//  * smash_strnum_order: the pair order of `samtools sort -n` (strnum_cmp:
//    digit runs compare as numbers), stable, so read 1 stays before read 2.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "fastq_par.hpp"
#include "ingest.hpp"

namespace smash {
void set_error(const std::string &msg);
}
using smash::set_error;
using smash::ingest::Chunk;
using smash::ingest::Reader;
using smash::ingest::strnum_cmp;

struct smash_fastq {
  Reader r1, r2;
  Chunk c1, c2;   // parse buffers, reused
  uint32_t L = 0;
  bool done = false;
};

extern "C" int smash_fastq_open(const char *const *r1, uint32_t n1, const char *const *r2,
                                uint32_t n2, smash_fastq **out) {
  if (!r1 || !r2 || !out || n1 == 0 || n2 == 0) {
    set_error("smash_fastq_open: need read-1 and read-2 paths");
    return SMASH_ERR_ARG;
  }
  auto *f = new smash_fastq;
  for (uint32_t i = 0; i < n1; ++i) f->r1.paths.emplace_back(r1[i]);
  for (uint32_t i = 0; i < n2; ++i) f->r2.paths.emplace_back(r2[i]);
  *out = f;
  return SMASH_OK;
}


extern "C" int smash_fastq_read(smash_fastq *f, uint64_t max_pairs, uint32_t *len,
                                uint8_t *h_reads, char *h_names, uint32_t name_stride,
                                uint64_t *n_pairs) {
  if (!f || !len || !h_reads || !n_pairs || (h_names && name_stride < 2)) {
    set_error("smash_fastq_read: bad arguments");
    return SMASH_ERR_ARG;
  }
  *n_pairs = 0;
  uint64_t q = 0;
  Chunk &c1 = f->c1, &c2 = f->c2;
  const uint8_t *lut = smash::ingest::lut();
  // the two mate lists are parsed (and inflated) on two threads, then zipped
  while (q < max_pairs && !f->done) {
    const uint64_t want = max_pairs - q;
    std::thread t([&] { c2.parse(f->r2, want, false); });
    c1.parse(f->r1, want, true);
    t.join();
    if (c1.err || c2.err) {
      set_error(c1.err ? f->r1.msg : f->r2.msg);
      return c1.err ? c1.err : c2.err;
    }
    const uint64_t n = std::min(c1.size(), c2.size());
    if (c1.end || c2.end) f->done = true;   // zip(): the shorter list ends the pairs
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t la = c1.boff[i + 1] - c1.boff[i], lb = c2.boff[i + 1] - c2.boff[i];
      if (la == 0 && lb == 0) continue;   // fastqs_to_sam.cpp:80 prints neither
      if (la == 0 || lb == 0) {
        // fastqs_to_sam.cpp:80 would print the other mate alone, which
        // misaligns memsam's read-1 / read-2 alternation (query.cpp:486-505)
        // for every later pair: such input is rejected, not silently changed
        set_error("smash_fastq_read: one mate of a pair has no bases (" +
                  std::string(c1.names.data() + c1.noff[i], c1.noff[i + 1] - c1.noff[i]) + ")");
        return SMASH_ERR_ARG;
      }
      const std::string na(c1.names.data() + c1.noff[i], c1.noff[i + 1] - c1.noff[i]);
      if (*len == 0) {
        if (la > 255) {
          set_error("smash_fastq_read: reads longer than 255 bases");
          return SMASH_ERR_UNSUPPORTED;
        }
        f->L = *len = uint32_t(la);
      }
      if (la != *len || lb != *len) {
        set_error("smash_fastq_read: all mates must have the same length (" + na + ")");
        return SMASH_ERR_ARG;
      }
      const char *a = c1.bases.data() + c1.boff[i], *b = c2.bases.data() + c2.boff[i];
      uint8_t *d = h_reads + q * 2 * *len;
      for (uint32_t j = 0; j < *len; ++j) d[j] = lut[uint8_t(a[j])];
      for (uint32_t j = 0; j < *len; ++j) d[*len + j] = lut[uint8_t(b[j])];
      if (h_names) {
        if (na.size() >= name_stride) {
          set_error("smash_fastq_read: read name longer than name_stride - 1: " + na);
          return SMASH_ERR_ARG;
        }
        char *o = h_names + q * name_stride;
        memcpy(o, na.data(), na.size());
        memset(o + na.size(), 0, name_stride - na.size());
      }
      ++q;
    }
  }
  *n_pairs = q;
  return SMASH_OK;
}

extern "C" void smash_fastq_close(smash_fastq *f) { delete f; }

extern "C" int smash_strnum_order(const char *names, uint32_t stride, uint64_t n,
                                  uint64_t *perm) {
  if ((!names && n) || (!perm && n) || stride == 0) {
    set_error("smash_strnum_order: bad arguments");
    return SMASH_ERR_ARG;
  }
  std::vector<uint32_t> len(n);
  for (uint64_t i = 0; i < n; ++i) len[i] = uint32_t(strnlen(names + i * stride, stride));
  std::iota(perm, perm + n, uint64_t(0));
  std::stable_sort(perm, perm + n, [&](uint64_t x, uint64_t y) {
    return strnum_cmp(names + x * stride, len[x], names + y * stride, len[y]) < 0;
  });
  return SMASH_OK;
}

// The parallel reader (fastq_par.hpp) as an object: the two lists mapped /
// inflated and indexed once, the pairs checked and ordered (plan_pairs);
// any range of the planned pairs is packed on demand (the multi-GPU driver
// deals batches to ranks from one index).  Host only.
struct smash_fastq_index {
  smash::ingest::PairIndex px;
  smash::ingest::Plan pl;
  uint32_t T = 1;
};

extern "C" int smash_fastq_index_open(const char *const *r1, uint32_t n1, const char *const *r2,
                                      uint32_t n2, uint32_t threads, uint32_t *len,
                                      int sort_names, smash_fastq_index **out,
                                      uint64_t *n_pairs) {
  if (!r1 || !r2 || n1 == 0 || n2 == 0 || !len || !out || !n_pairs) {
    set_error("smash_fastq_index_open: bad arguments");
    return SMASH_ERR_ARG;
  }
  auto *f = new smash_fastq_index;
  f->T = threads ? threads : 1;
  std::vector<std::string> p1(r1, r1 + n1), p2(r2, r2 + n2);
  std::string msg;
  int rc = f->px.build(p1, p2, f->T, msg);
  if (rc == SMASH_ERR_UNSUPPORTED) msg = "not strict 4-line FASTQ";
  // sort_names 0: the input must be in samtools sort -n order (checked)
  if (rc == SMASH_OK)
    rc = smash::ingest::plan_pairs(f->px, f->T, *len, sort_names == 0, sort_names != 0, f->pl, msg);
  if (rc != SMASH_OK) {
    set_error("smash_fastq_index_open: " + msg);
    delete f;
    return rc;
  }
  *len = f->pl.L;
  *n_pairs = f->pl.n_out;
  *out = f;
  return SMASH_OK;
}

extern "C" int smash_fastq_index_pack(smash_fastq_index *f, uint64_t k0, uint64_t k1,
                                      uint8_t *h_reads, char *h_names, uint32_t name_stride) {
  if (!f || k1 < k0 || k1 > f->pl.n_out || (k1 > k0 && !h_reads) ||
      (h_names && name_stride < 2)) {
    set_error("smash_fastq_index_pack: bad arguments");
    return SMASH_ERR_ARG;
  }
  if (!smash::ingest::pack_pairs(f->px, f->pl, k0, k1, h_reads, h_names, name_stride, f->T)) {
    set_error("smash_fastq_index_pack: read name longer than name_stride - 1");
    return SMASH_ERR_ARG;
  }
  return SMASH_OK;
}

extern "C" void smash_fastq_index_close(smash_fastq_index *f) { delete f; }

// all pairs at once, in file order (the order check off)
extern "C" int smash_fastq_read_parallel(const char *const *r1, uint32_t n1,
                                         const char *const *r2, uint32_t n2, uint32_t threads,
                                         uint32_t *len, uint64_t cap_pairs, uint8_t *h_reads,
                                         char *h_names, uint32_t name_stride,
                                         uint64_t *n_pairs) {
  if (!r1 || !r2 || n1 == 0 || n2 == 0 || !len || !n_pairs || (h_names && name_stride < 2)) {
    set_error("smash_fastq_read_parallel: bad arguments");
    return SMASH_ERR_ARG;
  }
  smash_fastq_index f;
  f.T = threads ? threads : 1;
  std::vector<std::string> p1(r1, r1 + n1), p2(r2, r2 + n2);
  std::string msg;
  int rc = f.px.build(p1, p2, f.T, msg);
  if (rc == SMASH_ERR_UNSUPPORTED) msg = "not strict 4-line FASTQ";
  if (rc == SMASH_OK) rc = smash::ingest::plan_pairs(f.px, f.T, *len, false, false, f.pl, msg);
  if (rc != SMASH_OK) {
    set_error("smash_fastq_read_parallel: " + msg);
    return rc;
  }
  *len = f.pl.L;
  *n_pairs = f.pl.n_out;
  if (!h_reads) return SMASH_OK;
  if (f.pl.n_out > cap_pairs) {
    set_error("smash_fastq_read_parallel: more pairs than cap_pairs");
    return SMASH_ERR_ARG;
  }
  if (!smash::ingest::pack_pairs(f.px, f.pl, 0, f.pl.n_out, h_reads, h_names, name_stride, f.T)) {
    set_error("smash_fastq_read_parallel: read name longer than name_stride - 1");
    return SMASH_ERR_ARG;
  }
  return SMASH_OK;
}
