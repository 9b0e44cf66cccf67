// smash-paper_amd/csrc/samout.hip -- the memsam `mapout` SAM writer
// (`mummer -rcref -samin -samout`, query.cpp:331-415) and, optionally, the
// mappability_tag L/R tags (mappability_tag.cpp:93-124) on the same lines.
//
// Split: everything that touches the index runs on the device, the text
// formatting on the host (the reference's OutputSorter is host I/O too).
//  k_sam_recs   one thread per match slot of smash_map_batch's output:
//               Alignment::resolve (query.cpp:68-97), the XE count of its
//               diagonal (query.cpp:270-274: text vs query over the whole
//               read) and the mappability L/R of its '=' block, i.e. the
//               map.bin bytes mappability_tag reads for that block
//               (abspos + offset + count - 1 and abspos + offset - 1, u32).
//  smash_sam_format  per pair: erase pos < 0, to_merge sort + diagonal merge
//               with the CIGAR (query.cpp:253-299), to_print order, HI/NH and
//               prev/next links (:300-305), set_nomap (:308-320), set_mate
//               (:424-438), print_matches (:331-415) and the tag columns.
#include <algorithm>
#include <cstdarg>
#include <cstring>
#include <string>

#include "common.hpp"

namespace smash {
namespace {

constexpr int kSB = 256;

__global__ __launch_bounds__(kSB) void k_sam_recs(
    const uint64_t *__restrict__ match, const uint32_t *__restrict__ n_match, uint32_t cap,
    uint64_t n_reads, const uint8_t *__restrict__ reads, uint64_t stride,
    const uint16_t *__restrict__ lens, uint32_t L0,
    const uint8_t *__restrict__ text, uint64_t N, const uint64_t *__restrict__ startpos,
    const uint64_t *__restrict__ sizes, uint32_t n_seq, int rcref,
    const uint32_t *__restrict__ tag_off, const uint8_t *__restrict__ map, uint64_t map_bytes,
    const uint64_t *__restrict__ off, smash_sam_rec *__restrict__ out) {
  const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t r = t / cap;
  const uint32_t k = uint32_t(t % cap);
  if (r >= n_reads) return;
  const uint32_t nm = n_match[r];
  if (k >= nm) return;
  const uint32_t L = lens ? lens[r] : L0;
  const uint64_t w = match[r * cap + k];
  const uint64_t ref = w & 0xFFFFFFFFFFFFull;
  const uint32_t q = uint32_t((w >> 48) & 0xFF), len = uint32_t(w >> 56);
  uint32_t lo = 0, hi = n_seq;   // upper_bound(startpos, ref) - 1
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (startpos[mid] <= ref) lo = mid + 1; else hi = mid;
  }
  uint32_t si = lo ? lo - 1 : 0;
  const int64_t rcpos = int64_t(ref) - int64_t(q);
  int64_t pos = rcpos - int64_t(startpos[si]);
  const uint32_t extra = L - len - q;
  smash_sam_rec o;
  if (rcref && (si & 1)) {   // rcref: odd sequences are reverse complements (query.cpp:80)
    si -= 1;
    pos = int64_t(sizes[si]) - pos - int64_t(L);
    o.prefix = uint16_t(extra);
    o.suffix = uint16_t(q);
    o.rc = 1;
  } else {
    o.prefix = uint16_t(q);
    o.suffix = uint16_t(extra);
    o.rc = 0;
  }
  o.pos = pos;
  o.tid = rcref ? si >> 1 : si;
  o.qpos = uint16_t(q);
  o.len = uint16_t(len);
  // XE of the diagonal: ref_pos = rcpos + j in [0, N) and text == query
  const uint8_t *P = reads + r * stride;
  uint32_t xe = 0;
  for (uint32_t j = 0; j < L; ++j) {
    const int64_t rp = rcpos + int64_t(j);
    xe += (rp >= 0 && rp < int64_t(N) && text[rp] == P[j]) ? 1u : 0u;
  }
  o.xe = xe;
  // mappability_tag of this block: unsigned arithmetic as util.h:138-143
  int32_t left = 0, right = 0;
  if (tag_off && pos >= 0) {
    const uint32_t abspos = tag_off[o.tid] + uint32_t(pos) + 1u;
    const uint32_t li = abspos + o.prefix + len - 1u, ri = abspos + o.prefix - 1u;
    const uint64_t la = 2 + uint64_t(li) * 2, ra = 2 + uint64_t(ri) * 2 + 1;
    const uint32_t lm = la < map_bytes ? map[la] : 0u, rm = ra < map_bytes ? map[ra] : 0u;
    left = lm ? int32_t(lm) - 1 : 255;
    right = rm ? int32_t(rm) : 255;
  }
  o.left = left;
  o.right = right;
  o.pad = 0;
  o.spare = 0;
  o.reserved = 0;
  out[(off ? off[r] : r * cap) + k] = o;   // packed: read r's records from off[r]
}

// ---- host side: one Aligner's prepare_matches + print_matches ------------

struct Al {
  smash_sam_rec r;
  uint32_t n_matches = 0;
  uint64_t n_unique = 0;
  int64_t qpos = 0;
  std::string cigar = "*";
  std::vector<const smash_sam_rec *> blocks;   // the group's '=' blocks, CIGAR order
  int hi = -1;
  int prev = -1, next = -1;
};

struct Mate {
  std::vector<Al> al;
  std::vector<int> printed;   // indices in to_print order with n_matches > 0
  int best = -1;              // best_alignment (to_print front)
  unsigned flag = 0;
  bool unmapped = false;
  const Al *best_mate = nullptr;
};

void prepare(Mate &m, const smash_sam_rec *rec, uint32_t n) {
  for (uint32_t k = 0; k < n; ++k)
    if (rec[k].pos >= 0) {   // erase off-chromosome mappings (query.cpp:243-250)
      Al a;
      a.r = rec[k];
      a.qpos = rec[k].qpos;
      m.al.push_back(a);
    }
  const size_t na = m.al.size();
  if (!na) return;
  std::vector<int> idx(na);
  for (size_t i = 0; i < na; ++i) idx[i] = int(i);
  auto merge_less = [&](int x, int y) {   // to_merge (query.cpp:201-217)
    const smash_sam_rec &a = m.al[x].r, &b = m.al[y].r;
    if (a.rc != b.rc) return a.rc < b.rc;
    if (a.tid != b.tid) return a.tid < b.tid;
    if (a.pos != b.pos) return a.pos < b.pos;
    return a.prefix < b.prefix;
  };
  std::stable_sort(idx.begin(), idx.end(), merge_less);
  std::string cig;
  uint64_t last_end = 0;
  uint32_t gm = 0;
  uint64_t gu = 0;
  int64_t gq = INT64_MAX;
  std::vector<const smash_sam_rec *> gb;
  char buf[48];
  for (size_t i = 0; i < na; ++i) {
    Al &a = m.al[idx[i]];
    const Al *nx = i + 1 < na ? &m.al[idx[i + 1]] : nullptr;
    ++gm;
    gu += a.r.len;
    gq = std::min(gq, a.qpos);
    if (a.r.prefix) {
      snprintf(buf, sizeof buf, "%lu%c", (unsigned long)(a.r.prefix - last_end),
               last_end ? 'M' : 'S');
      cig += buf;
    }
    snprintf(buf, sizeof buf, "%u=", unsigned(a.r.len));
    cig += buf;
    gb.push_back(&a.r);
    if (!nx || nx->r.pos != a.r.pos || nx->r.tid != a.r.tid || nx->r.rc != a.r.rc) {
      if (a.r.suffix) {
        snprintf(buf, sizeof buf, "%uS", unsigned(a.r.suffix));
        cig += buf;
      }
      a.cigar.swap(cig);
      a.blocks.swap(gb);
      a.n_matches = gm;
      a.n_unique = gu;
      a.qpos = gq;
      cig.clear();
      gb.clear();
      last_end = 0;
      gm = 0;
      gu = 0;
      gq = INT64_MAX;
    } else {
      last_end = uint64_t(a.r.prefix) + a.r.len;   // merged away: n_matches stays 0
    }
  }
  // to_print (query.cpp:219-229): qpos, then rc.  Ties are common under
  // -maxmatch (one segment, many loci) and the reference breaks them with
  // std::sort's introsort over the to_merge order (query.cpp:292): the same
  // std::sort over the same sequence reproduces its order exactly
  std::sort(idx.begin(), idx.end(), [&](int x, int y) {
    const Al &a = m.al[x], &b = m.al[y];
    if (a.qpos != b.qpos) return a.qpos < b.qpos;
    return a.r.rc < b.r.rc;
  });
  m.best = idx.front();
  int prev = -1;
  for (int i : idx) {
    Al &a = m.al[i];
    if (!a.n_matches) continue;
    a.hi = int(m.printed.size());
    m.printed.push_back(i);
    if (prev >= 0) {
      a.prev = prev;
      m.al[prev].next = i;
    }
    prev = i;
  }
}

std::string rev_comp(const char *s) {   // fasta.cpp:26-60
  std::string o(s);
  std::reverse(o.begin(), o.end());
  for (char &ch : o) {
    switch (ch) {
      case 'a': ch = 't'; break;
      case 'c': ch = 'g'; break;
      case 'g': ch = 'c'; break;
      case 't': ch = 'a'; break;
      case 'r': ch = 'y'; break;
      case 'y': ch = 'r'; break;
      case 'm': ch = 'k'; break;
      case 'k': ch = 'm'; break;
      case 'b': ch = 'v'; break;
      case 'd': ch = 'h'; break;
      case 'h': ch = 'd'; break;
      case 'v': ch = 'b'; break;
      case 'A': ch = 'T'; break;
      case 'C': ch = 'G'; break;
      case 'G': ch = 'C'; break;
      case 'T': ch = 'A'; break;
      case 'R': ch = 'Y'; break;
      case 'Y': ch = 'R'; break;
      case 'M': ch = 'K'; break;
      case 'K': ch = 'M'; break;
      case 'B': ch = 'V'; break;
      case 'D': ch = 'H'; break;
      case 'H': ch = 'D'; break;
      case 'V': ch = 'B'; break;
      default: break;
    }
  }
  return o;
}

void appendf(std::string &o, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
void appendf(std::string &o, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  const int n = vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (n < int(sizeof buf)) {
    o.append(buf, size_t(n));
    return;
  }
  std::string big(size_t(n) + 1, '\0');
  va_start(ap, fmt);
  vsnprintf(&big[0], big.size(), fmt, ap);
  va_end(ap);
  o.append(big.data(), size_t(n));
}

}  // namespace
}  // namespace smash

using namespace smash;

static_assert(sizeof(smash_sam_rec) == 40, "smash_sam_rec layout (smashgpu.SAM_REC)");

static int sam_records(const smash_index *ix, const uint8_t *d_reads, uint64_t stride,
                       const uint16_t *d_lens, uint32_t len, uint64_t n_reads,
                       const uint64_t *d_match, uint32_t cap_per_read, const uint32_t *d_n_match,
                       const uint64_t *d_rec_off, const uint32_t *d_tag_offsets,
                       smash_sam_rec *d_out, void *stream) {
  if (!ix || !d_reads || !d_match || !d_n_match || !d_out || !cap_per_read ||
      (!d_lens && (len == 0 || len > 255 || stride < len)) || (d_lens && stride < 255)) {
    set_error("smash_sam_records: bad arguments");
    return SMASH_ERR_ARG;
  }
  if (d_tag_offsets && !ix->d_map) {
    set_error("smash_sam_records: tag offsets given but the index has no map.bin");
    return SMASH_ERR_ARG;
  }
  if (n_reads == 0) return SMASH_OK;
  const uint64_t slots = n_reads * cap_per_read;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(k_sam_recs, dim3(unsigned((slots + kSB - 1) / kSB)), dim3(kSB), 0, s,
                     d_match, d_n_match, cap_per_read, n_reads, d_reads, stride, d_lens, len,
                     ix->d_text, ix->N, ix->d_startpos, ix->d_sizes, ix->n_seq,
                     ix->rcref ? 1 : 0, d_tag_offsets, ix->d_map, ix->map_bytes, d_rec_off, d_out);
  SMASH_HIP(hipGetLastError());
  return SMASH_OK;
}

extern "C" int smash_sam_records(const smash_index *ix, const uint8_t *d_reads, uint64_t stride,
                                 const uint16_t *d_lens, uint32_t len, uint64_t n_reads,
                                 const uint64_t *d_match, uint32_t cap_per_read,
                                 const uint32_t *d_n_match, const uint32_t *d_tag_offsets,
                                 smash_sam_rec *d_out, void *stream) {
  return sam_records(ix, d_reads, stride, d_lens, len, n_reads, d_match, cap_per_read, d_n_match,
                     nullptr, d_tag_offsets, d_out, stream);
}

extern "C" int smash_sam_records_packed(const smash_index *ix, const uint8_t *d_reads,
                                        uint64_t stride, const uint16_t *d_lens, uint32_t len,
                                        uint64_t n_reads, const uint64_t *d_match,
                                        uint32_t cap_per_read, const uint32_t *d_n_match,
                                        const uint64_t *d_rec_off, const uint32_t *d_tag_offsets,
                                        smash_sam_rec *d_out, void *stream) {
  if (!d_rec_off) {
    set_error("smash_sam_records_packed: no record offsets");
    return SMASH_ERR_ARG;
  }
  return sam_records(ix, d_reads, stride, d_lens, len, n_reads, d_match, cap_per_read, d_n_match,
                     d_rec_off, d_tag_offsets, d_out, stream);
}

extern "C" int smash_sam_format(const char *const *contigs, uint32_t n_contig,
                                const smash_sam_rec *h_rec,
                                const uint32_t *h_n, uint32_t cap_per_read, uint64_t n_reads,
                                const char *const *names, const char *const *seqs,
                                const char *const *quals, const char *const *optionals,
                                int nomap, int tag, const uint8_t *h_small_chr,
                                char **out_text, uint64_t *out_len, int32_t *tag_error) {
  if (!contigs || !h_rec || !h_n || !names || !seqs || !out_text || !out_len) {
    set_error("smash_sam_format: bad arguments");
    return SMASH_ERR_ARG;
  }
  // packed records (smash_sam_records_packed): read r's h_n[r] records
  // follow read r-1's; else read r's start at r * cap_per_read.  The cap is
  // the search's slots per read in both layouts (0: packed, unchecked): a
  // count above it means the read's match list was cut, which no layout can
  // format (and packed offsets would run past the records written)
  const bool packed = cap_per_read == 0 || (cap_per_read & SMASH_SAM_PACKED);
  const uint32_t cap = cap_per_read & ~uint32_t(SMASH_SAM_PACKED);
  std::vector<uint64_t> roff(n_reads);
  for (uint64_t r = 0, acc = 0; r < n_reads; ++r) {
    roff[r] = packed ? acc : r * cap;
    acc += h_n[r];
  }
  if (tag_error) *tag_error = 0;
  std::string o;
  o.reserve(n_reads * 256);
  for (uint64_t r = 0; r < n_reads; ++r) {   // every record's contig must be named
    if (cap && h_n[r] > cap) {
      set_error("smash_sam_format: a read has more matches than cap_per_read");
      return SMASH_ERR_ARG;
    }
    for (uint32_t k = 0; k < h_n[r]; ++k)
      if (h_rec[roff[r] + k].tid >= n_contig) {
        set_error("smash_sam_format: record contig out of range");
        return SMASH_ERR_ARG;
      }
  }
  auto contig = [&](uint32_t tid) -> const char * { return contigs[tid]; };
  uint64_t i = 0;
  while (i < n_reads) {
    // Pair::run: queries alternate read1/read2 (query.cpp:486-505)
    const uint64_t nq = std::min<uint64_t>(2, n_reads - i);
    Mate mt[2];
    for (uint64_t k = 0; k < nq; ++k) {
      Mate &m = mt[k];
      const char *nm = names[i + k];
      const size_t nl = strlen(nm);
      if (nl >= 2 && nm[nl - 2] == ':' && (nm[nl - 1] == '0' || nm[nl - 1] == '1'))
        m.flag = nm[nl - 1] == '0' ? 65u : 129u;   // Aligner::reset (query.cpp:186-199)
      prepare(m, h_rec + roff[i + k], h_n[i + k]);
      if (m.printed.empty() && nomap) {   // set_nomap (query.cpp:308-320)
        m.unmapped = true;
        m.flag |= 4u;
      }
    }
    auto n_align = [](const Mate &m) { return m.printed.size() + (m.unmapped ? 1 : 0); };
    auto best_of = [](const Mate &m) -> const Al * {
      return m.printed.empty() ? nullptr : &m.al[size_t(m.best)];
    };
    if (nq == 2 && (mt[0].flag & 64u) && (mt[1].flag & 128u)) {   // has_mate + set_mate
      for (int k = 0; k < 2; ++k) {
        Mate &m = mt[k];
        const Mate &other = mt[1 - k];
        if (n_align(m) && n_align(other)) {
          if (best_of(other)) {
            m.best_mate = best_of(other);
          } else {
            m.flag |= 8u;
            m.best_mate = best_of(m);
          }
        }
      }
    }
    for (uint64_t k = 0; k < nq; ++k) {
      const Mate &m = mt[k];
      std::string name = names[i + k];
      if ((m.flag & 192u) && name.size() >= 2) name.resize(name.size() - 2);
      const char *seq = seqs[i + k];
      const std::string qual =
          quals && quals[i + k] ? std::string(quals[i + k]) : std::string(strlen(seq), '!');
      const char *opt = optionals && optionals[i + k] ? optionals[i + k] : "";
      std::vector<const Al *> lines;
      if (m.unmapped) lines.push_back(nullptr);
      for (int p : m.printed) lines.push_back(&m.al[size_t(p)]);
      for (const Al *a : lines) {
        if (!a) {
          if (m.best_mate)
            appendf(o, "%s\t%u\t%s\t%ld\t0\t*", name.c_str(), m.flag, contig(m.best_mate->r.tid),
                    long(m.best_mate->r.pos + 1));
          else
            appendf(o, "%s\t%u\t*\t0\t0\t*", name.c_str(), m.flag);
        } else {
          appendf(o, "%s\t%u\t%s\t%ld\t50\t%s", name.c_str(),
                  m.flag | (a->r.rc ? 16u : 0u) | (a->hi ? 256u : 0u), contig(a->r.tid),
                  long(a->r.pos + 1), a->cigar.c_str());
        }
        if (m.best_mate)
          appendf(o, "\t%s\t%ld\t0", contig(m.best_mate->r.tid), long(m.best_mate->r.pos + 1));
        else
          o += "\t*\t0\t0";
        if (a && a->r.rc) {
          o += '\t';
          o += rev_comp(seq);
          o += '\t';
          o.append(qual.rbegin(), qual.rend());
        } else {
          o += '\t';
          o += seq;
          o += '\t';
          o += qual;
        }
        if (a) {
          appendf(o, "\tXM:i:%u\tXU:i:%lu\tXE:i:%u\tXS:A:%c\tNH:i:%lu\tHI:i:%d", a->n_matches,
                  (unsigned long)a->n_unique, a->r.xe, a->r.rc ? '-' : '+',
                  (unsigned long)n_align(m), a->hi);
          if (a->prev >= 0) {
            const Al &p = m.al[size_t(a->prev)];
            appendf(o, "\tcc:Z:%s\tcp:i:%ld\txo:A:%c\txc:Z:%s", contig(p.r.tid),
                    long(p.r.pos + 1), p.r.rc == a->r.rc ? '=' : '!', p.cigar.c_str());
          }
          if (a->next >= 0) {
            const Al &n = m.al[size_t(a->next)];
            appendf(o, "\tCC:Z:%s\tCP:i:%ld\tXO:A:%c\tXC:Z:%s", contig(n.r.tid),
                    long(n.r.pos + 1), n.r.rc == a->r.rc ? '=' : '!', n.cigar.c_str());
          }
        } else {
          o += "\tXM:i:0\tNH:i:0";
        }
        o += opt;
        if (tag && a) {   // mappability_tag: L/R of the first 10 '=' blocks
          const bool small = h_small_chr && h_small_chr[a->r.tid];
          int u = 0;
          for (const smash_sam_rec *b : a->blocks) {
            const uint32_t left = uint32_t(b->left), right = uint32_t(b->right);
            if (u < 10) appendf(o, "\tL%d:i:%u\tR%d:i:%u", u, left, u, right);
            if (!small && tag_error && *tag_error == 0) {
              if (left > b->len) *tag_error = SMASH_ERR_TAG_LEFT;
              else if (right > b->len) *tag_error = SMASH_ERR_TAG_RIGHT;
            }
            ++u;
          }
        }
        o += '\n';
      }
    }
    i += nq;
  }
  char *buf = static_cast<char *>(malloc(o.size() + 1));
  if (!buf) {
    set_error("smash_sam_format: out of host memory");
    return SMASH_ERR_NOMEM;
  }
  memcpy(buf, o.data(), o.size());
  buf[o.size()] = 0;
  *out_text = buf;
  *out_len = o.size();
  return SMASH_OK;
}

extern "C" void smash_sam_free(char *text) { free(text); }
