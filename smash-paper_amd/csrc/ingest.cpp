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
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "../../include/smash_gpu.h"

namespace smash {
void set_error(const std::string &msg);
}
using smash::set_error;

namespace {

struct Reader {
  std::vector<std::string> paths;
  size_t next_path = 0;
  gzFile f = nullptr;
  std::vector<char> buf = std::vector<char>(1 << 22);
  size_t beg = 0, fill = 0;   // unread bytes buf[beg, fill)
  std::string msg;   // error text (set_error is per thread; the caller reports it)

  ~Reader() {
    if (f) gzclose(f);
  }
  // refill from the current file (opening the next at EOF); false at the end
  bool more(int &err) {
    for (;;) {
      if (!f) {
        if (next_path >= paths.size()) return false;
        f = gzopen(paths[next_path].c_str(), "rb");
        if (!f) {
          msg = ("cannot open " + paths[next_path]);
          err = SMASH_ERR_IO;
          return false;
        }
        gzbuffer(f, 1 << 20);
        ++next_path;
      }
      if (beg) {
        memmove(buf.data(), buf.data() + beg, fill - beg);
        fill -= beg;
        beg = 0;
      }
      if (fill == buf.size()) buf.resize(buf.size() * 2);
      const int n = gzread(f, buf.data() + fill, unsigned(buf.size() - fill));
      if (n < 0) {
        msg = ("read error in " + paths[next_path - 1]);
        err = SMASH_ERR_IO;
        return false;
      }
      if (n > 0) {
        fill += size_t(n);
        return true;
      }
      gzclose(f);
      f = nullptr;
      // a file that does not end in '\n' ends its last line (as getline does)
      if (fill > beg && buf[fill - 1] != '\n') {
        if (fill == buf.size()) buf.resize(buf.size() * 2);
        buf[fill++] = '\n';
        return true;
      }
    }
  }
  // one line without the trailing \r\n; false at the end of the last file
  bool line(std::string &out, int &err) {
    out.clear();
    size_t scan = beg;
    for (;;) {
      const char *nl = static_cast<const char *>(memchr(buf.data() + scan, '\n', fill - scan));
      if (nl) {
        size_t e = size_t(nl - buf.data());
        out.assign(buf.data() + beg, e - beg);
        beg = e + 1;
        while (!out.empty() && out.back() == '\r') out.pop_back();
        return true;
      }
      scan = fill - beg;   // offset after the memmove in more()
      if (!more(err)) {
        if (fill > beg) {   // unreachable: more() terminates a last line
          out.assign(buf.data() + beg, fill - beg);
          beg = fill;
          return true;
        }
        return false;
      }
    }
  }
  // fastqs_to_sam record: name, bases; false at the end
  bool record(std::string &name, std::string &bases, int &err) {
    std::string l;
    for (;;) {
      if (!line(l, err)) return false;
      size_t b = 0, e = l.size();
      while (b < e && isspace(uint8_t(l[b]))) ++b;
      while (e > b && isspace(uint8_t(l[e - 1]))) --e;
      if (b == e) continue;
      const char mark = l[b];
      if (mark != '@' && mark != '>') {
        msg = ("Fastq @ parse error: " + l.substr(0, 40));
        err = SMASH_ERR_IO;
        return false;
      }
      size_t t = b + 1;
      while (t < e && isspace(uint8_t(l[t]))) ++t;
      size_t te = t;
      while (te < e && !isspace(uint8_t(l[te]))) ++te;
      if (t == te) {
        msg = ("Problem reading read name");
        err = SMASH_ERR_IO;
        return false;
      }
      name.assign(l, t, te - t);
      if (!line(bases, err)) bases.clear();
      if (err) return false;
      if (mark == '@') {
        std::string plus, qual;
        if (!line(plus, err) || plus.find_first_not_of(" \t") == std::string::npos ||
            plus[plus.find_first_not_of(" \t")] != '+') {
          if (!err) {
            msg = ("Fastq + parse error");
            err = SMASH_ERR_IO;
          }
          return false;
        }
        line(qual, err);
        if (err) return false;
      }
      return true;
    }
  }
};

// samtools sort -n (bam_sort.c strnum_cmp; samtools is absent from the
// reference and unpinned: this follows samtools 1.x): bytes compare one by
// one; where both sides are at a digit, leading zeros are skipped, matching
// digits walked, and the longer digit run wins, else the first differing
// digit; a non-digit on either side compares the two bytes.  Names are
// NUL-terminated within their n bytes.
int strnum_cmp(const char *a, size_t na, const char *b, size_t nb) {
  auto at = [](const char *s, size_t n, size_t i) -> int {
    return i < n ? static_cast<unsigned char>(s[i]) : 0;
  };
  auto isd = [](int c) { return c >= '0' && c <= '9'; };
  size_t i = 0, j = 0;
  while (at(a, na, i) && at(b, nb, j)) {
    const int ca = at(a, na, i), cb = at(b, nb, j);
    if (!isd(ca) || !isd(cb)) {
      if (ca != cb) return ca - cb;
      ++i;
      ++j;
    } else {
      while (at(a, na, i) == '0') ++i;
      while (at(b, nb, j) == '0') ++j;
      while (isd(at(a, na, i)) && at(a, na, i) == at(b, nb, j)) ++i, ++j;
      const int diff = at(a, na, i) - at(b, nb, j);
      while (isd(at(a, na, i)) && isd(at(b, nb, j))) ++i, ++j;
      if (isd(at(a, na, i))) return 1;
      if (isd(at(b, nb, j))) return -1;
      if (diff) return diff;
    }
  }
  return at(a, na, i) ? 1 : at(b, nb, j) ? -1 : 0;
}

uint8_t g_lut[256];
struct LutInit {
  LutInit() {
    for (int c = 0; c < 256; ++c) g_lut[c] = uint8_t(c >= 'A' && c <= 'Z' ? c + 32 : c);
    g_lut[uint8_t('N')] = uint8_t('z');   // replaceN, then lowercase
  }
} g_lut_init;

}  // namespace

struct smash_fastq {
  Reader r1, r2;
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

namespace {
// up to `want` records of one mate list: names (read 1 only) and bases, flat
struct Chunk {
  std::vector<char> bases, names;
  std::vector<uint64_t> boff, noff;   // n + 1 offsets each
  bool end = false;
  int err = 0;
  void parse(Reader &r, uint64_t want, bool keep_names) {
    bases.clear();
    names.clear();
    boff.assign(1, 0);
    noff.assign(1, 0);
    end = false;
    std::string nm, b;
    for (uint64_t i = 0; i < want; ++i) {
      if (!r.record(nm, b, err)) {
        end = true;
        return;
      }
      bases.insert(bases.end(), b.begin(), b.end());
      boff.push_back(bases.size());
      if (keep_names) names.insert(names.end(), nm.begin(), nm.end());
      noff.push_back(names.size());
    }
  }
  uint64_t size() const { return boff.size() - 1; }
};
}  // namespace

extern "C" int smash_fastq_read(smash_fastq *f, uint64_t max_pairs, uint32_t *len,
                                uint8_t *h_reads, char *h_names, uint32_t name_stride,
                                uint64_t *n_pairs) {
  if (!f || !len || !h_reads || !n_pairs || (h_names && name_stride < 2)) {
    set_error("smash_fastq_read: bad arguments");
    return SMASH_ERR_ARG;
  }
  *n_pairs = 0;
  uint64_t q = 0;
  Chunk c1, c2;
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
      for (uint32_t j = 0; j < *len; ++j) d[j] = g_lut[uint8_t(a[j])];
      for (uint32_t j = 0; j < *len; ++j) d[*len + j] = g_lut[uint8_t(b[j])];
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
