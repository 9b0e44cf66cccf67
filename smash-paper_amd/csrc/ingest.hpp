// smash-paper_amd/csrc/ingest.hpp -- the FASTQ/FASTA reader shared by the
// batch reader (ingest.cpp, smash_fastq_read) and the file-fed counting
// pipeline (feed.hip, smash_count_fastq).  Host code.
//
// Records follow fastqs_to_sam.cpp:48-96: blank lines before a record are
// skipped, a record starts with '@' (4 lines: name, bases, '+' line,
// qualities) or '>' (2 lines: name, bases); the name is the first token after
// the marker; a missing bases line at the end of input is an empty read; a
// missing or malformed '+' line is an error.  Lines lose their trailing "\r".
// Records are parsed in place in the reader's buffer (views valid until the
// next record() call), so a read costs a few memchr calls and one copy.
#pragma once

#include <zlib.h>

#include <cctype>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/smash_gpu.h"

namespace smash {
namespace ingest {

struct View {
  const char *p = nullptr;
  size_t n = 0;
};

struct Reader {
  std::vector<std::string> paths;
  size_t next_path = 0;
  gzFile f = nullptr;
  std::vector<char> buf = std::vector<char>(1 << 22);
  size_t beg = 0, fill = 0;   // unread bytes buf[beg, fill)
  std::string msg;            // error text (set_error is per thread; the caller reports it)

  Reader() = default;
  Reader(const Reader &) = delete;
  Reader &operator=(const Reader &) = delete;
  ~Reader() {
    if (f) gzclose(f);
  }

  // compact [beg, fill) to the front (*shift = bytes dropped) and read more,
  // opening the next file at the end of one; false at the end of the last
  bool more(int &err, size_t &shift) {
    shift = 0;
    for (;;) {
      if (!f) {
        if (next_path >= paths.size()) return false;
        f = gzopen(paths[next_path].c_str(), "rb");
        if (!f) {
          msg = "cannot open " + paths[next_path];
          err = SMASH_ERR_IO;
          return false;
        }
        gzbuffer(f, 1 << 20);
        ++next_path;
      }
      if (beg) {
        memmove(buf.data(), buf.data() + beg, fill - beg);
        fill -= beg;
        shift += beg;
        beg = 0;
      }
      if (fill == buf.size()) buf.resize(buf.size() * 2);
      const int n = gzread(f, buf.data() + fill, unsigned(buf.size() - fill));
      if (n < 0) {
        msg = "read error in " + paths[next_path - 1];
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

  // the line starting at offset pos (>= beg): [s, e) without "\n" and
  // trailing "\r", pos moved past it; a refill shifts pos and adj[0..nadj)
  // (offsets of this record's earlier lines).  false: no further line.
  bool next_line(size_t &pos, size_t &s, size_t &e, int &err, size_t *adj, int nadj) {
    size_t scan = pos;
    for (;;) {
      const void *nl = scan < fill ? memchr(buf.data() + scan, '\n', fill - scan) : nullptr;
      if (nl) {
        s = pos;
        e = size_t(static_cast<const char *>(nl) - buf.data());
        pos = e + 1;
        while (e > s && buf[e - 1] == '\r') --e;
        return true;
      }
      const size_t seen = fill;
      size_t shift = 0;
      if (!more(err, shift)) return false;
      pos -= shift;
      scan = seen - shift;
      for (int k = 0; k < nadj; ++k) adj[k] -= shift;
    }
  }

  // the next record's name and bases (views into buf); false at the end of
  // input or on an error (err set, msg says what)
  bool record(View &name, View &bases, int &err) {
    for (;;) {
      size_t pos = beg, s = 0, e = 0;
      if (!next_line(pos, s, e, err, nullptr, 0)) return false;
      size_t b = s, t = e;
      while (b < t && isspace(uint8_t(buf[b]))) ++b;
      while (t > b && isspace(uint8_t(buf[t - 1]))) --t;
      if (b == t) {   // blank line
        beg = pos;
        continue;
      }
      const char mark = buf[b];
      if (mark != '@' && mark != '>') {
        msg = "Fastq @ parse error: " + std::string(buf.data() + b, std::min<size_t>(t - b, 40));
        err = SMASH_ERR_IO;
        return false;
      }
      size_t nb = b + 1;
      while (nb < t && isspace(uint8_t(buf[nb]))) ++nb;
      size_t ne = nb;
      while (ne < t && !isspace(uint8_t(buf[ne]))) ++ne;
      if (nb == ne) {
        msg = "Problem reading read name";
        err = SMASH_ERR_IO;
        return false;
      }
      size_t keep[4] = {nb, ne, 0, 0};
      size_t bs = 0, be = 0;
      if (next_line(pos, bs, be, err, keep, 2)) {
        keep[2] = bs;
        keep[3] = be;
      } else {
        if (err) return false;
        keep[2] = keep[3] = pos;   // no bases line: an empty read
      }
      if (mark == '@') {
        size_t ps = 0, pe = 0;
        bool ok = next_line(pos, ps, pe, err, keep, 4);
        if (ok) {
          while (ps < pe && (buf[ps] == ' ' || buf[ps] == '\t')) ++ps;
          ok = ps < pe && buf[ps] == '+';
        }
        if (!ok) {
          if (!err) {
            msg = "Fastq + parse error";
            err = SMASH_ERR_IO;
          }
          return false;
        }
        size_t qs = 0, qe = 0;
        next_line(pos, qs, qe, err, keep, 4);   // qualities (may be missing at the end)
        if (err) return false;
      }
      name = View{buf.data() + keep[0], keep[1] - keep[0]};
      bases = View{buf.data() + keep[2], keep[3] - keep[2]};
      beg = pos;
      return true;
    }
  }
};

// up to `want` records of one mate list: bases and (read 1) names, flat;
// buffers keep their capacity across calls
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
    View nm, b;
    for (uint64_t i = 0; i < want; ++i) {
      if (!r.record(nm, b, err)) {
        end = true;
        return;
      }
      const size_t o = bases.size();
      bases.resize(o + b.n);
      if (b.n) memcpy(bases.data() + o, b.p, b.n);
      boff.push_back(bases.size());
      if (keep_names) {
        const size_t q = names.size();
        names.resize(q + nm.n);
        memcpy(names.data() + q, nm.p, nm.n);
      }
      noff.push_back(names.size());
    }
  }
  uint64_t size() const { return boff.size() - 1; }
};

// samtools sort -n (bam_sort.c strnum_cmp; samtools is absent from the
// reference and unpinned: this follows samtools 1.x): bytes compare one by
// one; where both sides are at a digit, leading zeros are skipped, matching
// digits walked, and the longer digit run wins, else the first differing
// digit; a non-digit on either side compares the two bytes.  Names end at
// their length or at a NUL.
inline int strnum_cmp(const char *a, size_t na, const char *b, size_t nb) {
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

// replaceN (N -> Z, fastqs_to_sam.cpp:74 with argc == 4), then the
// NewQuery::extend lowercasing (query.cpp:125-144)
struct Lut {
  uint8_t t[256];
  Lut() {
    for (int c = 0; c < 256; ++c) t[c] = uint8_t(c >= 'A' && c <= 'Z' ? c + 32 : c);
    t[uint8_t('N')] = uint8_t('z');
  }
};
inline const uint8_t *lut() {
  static const Lut l;
  return l.t;
}

}  // namespace ingest
}  // namespace smash
