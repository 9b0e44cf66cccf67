// smash-paper_amd/csrc/fastq_par.hpp -- the parallel FASTQ reader behind
// smash_count_fastq (feed.hip) and smash_fastq_read_parallel (ingest.cpp).
// Host code.
//
// The front of smash_mapping.sh:19 (zcat r1s | fastqs_to_sam ...) reads each
// mate list on one thread (fastqs_to_sam.cpp:29-111).  Here every byte range
// of every file is indexed at once: in strict 4-line FASTQ ('@' name line,
// bases, '+' line, qualities; no blank lines) a record start is the only line
// that begins with '@' and is followed, two lines down, by a line beginning
// with '+' (a quality line may begin with '@', but two lines below it is the
// next record's bases line), so a thread that starts at an arbitrary byte
// finds the first record of its range by itself.  Plain files are mapped;
// gzip files are inflated whole, one thread per file (SMASH passes lists of
// lane files).  Then pair i is record i of list 1 and record i of list 2
// (zip: the shorter list ends the pairs), parsed and converted by any thread.
// Input that is not strict 4-line FASTQ (FASTA records, blank lines, a '+'
// line not in column 0, a truncated last record) makes index() return false:
// the streaming reader (ingest.hpp, fastqs_to_sam.cpp:48-96 semantics) takes
// it from the start.  On strict input both readers give the same pairs.
#pragma once

#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ingest.hpp"

namespace smash {
namespace ingest {

// run f(t) for t in [0, T) on T threads (the caller's thread is one)
template <class F>
void run_threads(uint32_t T, F f) {
  if (T <= 1) {
    f(0u);
    return;
  }
  std::vector<std::thread> th;
  for (uint32_t t = 1; t < T; ++t) th.emplace_back([&, t] { f(t); });
  f(0u);
  for (auto &x : th) x.join();
}

// one input file, its bytes in memory: mapped (plain) or inflated (gzip)
struct Source {
  std::string path;
  const char *p = nullptr;
  size_t n = 0;
  void *map = nullptr;
  size_t maplen = 0;
  std::vector<char> buf;
  char *raw = nullptr;   // an inflated file (malloc'd: never zero-filled, only written once)
  Source() = default;
  Source(const Source &) = delete;
  Source &operator=(const Source &) = delete;
  ~Source() {
    if (map) munmap(map, maplen);
    free(raw);
  }
};

// libdeflate (the image's libdeflate0 package: whole-buffer gzip decoding,
// ~2-3x zlib's inflate on FASTQ), bound at run time; absent, zlib reads the
// file.  Only the three entry points below are used (libdeflate 1.x ABI).
struct Deflate {
  void *(*alloc)() = nullptr;
  void (*release)(void *) = nullptr;
  int (*gzip_ex)(void *, const void *, size_t, void *, size_t, size_t *, size_t *) = nullptr;
  Deflate() {
    void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    alloc = reinterpret_cast<void *(*)()>(dlsym(h, "libdeflate_alloc_decompressor"));
    release = reinterpret_cast<void (*)(void *)>(dlsym(h, "libdeflate_free_decompressor"));
    gzip_ex = reinterpret_cast<int (*)(void *, const void *, size_t, void *, size_t, size_t *,
                                       size_t *)>(dlsym(h, "libdeflate_gzip_decompress_ex"));
    if (!alloc || !release || !gzip_ex) alloc = nullptr;
  }
  bool ok() const { return alloc != nullptr; }
};
inline const Deflate &deflate() {
  static const Deflate d;
  return d;
}

// a gzip file (every member, concatenated) into s.raw with libdeflate; the
// output is sized from the last member's ISIZE and grown on demand.  false:
// why (an error), or why empty: libdeflate is absent (use zlib)
inline bool inflate_libdeflate(Source &s, const unsigned char *in, size_t size, std::string &why) {
  const Deflate &D = deflate();
  if (!D.ok()) return false;
  void *dec = D.alloc();
  if (!dec) return false;
  const size_t isize = size >= 4 ? size_t(in[size - 4]) | size_t(in[size - 3]) << 8 |
                                       size_t(in[size - 2]) << 16 | size_t(in[size - 1]) << 24
                                 : 0;
  size_t cap = std::max<size_t>({isize + 1, size * 4, size_t(1) << 16});
  char *out = static_cast<char *>(malloc(cap + 1));
  size_t in_off = 0, fill = 0;
  bool ok = out != nullptr;
  while (ok && in_off + 2 <= size && in[in_off] == 0x1f && in[in_off + 1] == 0x8b) {
    size_t used = 0, got = 0;
    const int r = D.gzip_ex(dec, in + in_off, size - in_off, out + fill, cap - fill, &used, &got);
    if (r == 3) {   // LIBDEFLATE_INSUFFICIENT_SPACE: larger output, the member again
      cap *= 2;
      char *o2 = static_cast<char *>(realloc(out, cap + 1));
      if (!o2) {
        ok = false;
        break;
      }
      out = o2;
      continue;
    }
    if (r != 0) {   // LIBDEFLATE_BAD_DATA / SHORT_OUTPUT
      why = "corrupt gzip data in " + s.path;
      ok = false;
      break;
    }
    in_off += used;
    fill += got;
  }
  D.release(dec);
  if (!ok) {
    if (why.empty()) why = "out of host memory inflating " + s.path;
    free(out);
    return false;
  }
  // (trailing bytes that are no gzip member are ignored, as gzip -dc does)
  if (fill && out[fill - 1] != '\n') out[fill++] = '\n';
  s.raw = out;
  s.p = out;
  s.n = fill;
  return true;
}

// open one file: one that starts with the gzip magic is inflated into memory
// (zlib reads concatenated members), another is mapped; a file whose last
// byte is not '\n' is copied with one appended (every line of every record
// then ends in '\n').  false: why says what failed.
inline bool load_source(Source &s, std::string &why) {
  const int fd = open(s.path.c_str(), O_RDONLY);
  if (fd < 0) {
    why = "cannot open " + s.path;
    return false;
  }
  struct stat stt;
  unsigned char magic[2] = {0, 0};
  const bool ok = fstat(fd, &stt) == 0 && (stt.st_size < 2 || pread(fd, magic, 2, 0) == 2);
  if (!ok) {
    close(fd);
    why = "cannot read " + s.path;
    return false;
  }
  const size_t size = size_t(stt.st_size);
  if (size >= 2 && magic[0] == 0x1f && magic[1] == 0x8b) {
    if (deflate().ok()) {
      void *m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      close(fd);
      if (m == MAP_FAILED) {
        why = "cannot map " + s.path;
        return false;
      }
      madvise(m, size, MADV_SEQUENTIAL);
      const bool ok = inflate_libdeflate(s, static_cast<const unsigned char *>(m), size, why);
      munmap(m, size);
      return ok;
    }
    close(fd);
    gzFile g = gzopen(s.path.c_str(), "rb");
    if (!g) {
      why = "cannot open " + s.path;
      return false;
    }
    gzbuffer(g, 1 << 20);
    s.buf.resize(std::max<size_t>(size * 4, 1 << 20));
    size_t fill = 0;
    for (;;) {
      if (fill == s.buf.size()) s.buf.resize(s.buf.size() * 2);
      const size_t want = std::min<size_t>(s.buf.size() - fill, size_t(1) << 30);
      const int r = gzread(g, s.buf.data() + fill, unsigned(want));
      if (r < 0) {
        why = "read error in " + s.path;
        gzclose(g);
        return false;
      }
      if (r == 0) break;
      fill += size_t(r);
    }
    gzclose(g);
    s.buf.resize(fill);
    if (fill && s.buf.back() != '\n') s.buf.push_back('\n');
    s.p = s.buf.data();
    s.n = s.buf.size();
    return true;
  }
  if (size == 0) {
    close(fd);
    return true;
  }
  void *m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (m == MAP_FAILED) {
    why = "cannot map " + s.path;
    return false;
  }
  s.map = m;
  s.maplen = size;
  s.p = static_cast<const char *>(m);
  s.n = size;
  if (s.p[size - 1] != '\n') {   // (rare) give the last line its newline
    s.buf.assign(s.p, s.p + size);
    s.buf.push_back('\n');
    munmap(m, size);
    s.map = nullptr;
    s.p = s.buf.data();
    s.n = s.buf.size();
  }
  return true;
}

// open every path (load_source), in parallel
inline bool load_sources(const std::vector<std::string> &paths, uint32_t T,
                         std::vector<std::unique_ptr<Source>> &out, std::string &msg, int &err) {
  out.clear();
  for (const auto &p : paths) {
    out.emplace_back(new Source);
    out.back()->path = p;
  }
  std::atomic<size_t> next{0};
  std::atomic<int> bad{0};
  std::vector<std::string> why(out.size());
  run_threads(std::min<uint32_t>(T, uint32_t(out.size())), [&](uint32_t) {
    for (size_t k; (k = next++) < out.size();)
      if (!load_source(*out[k], why[k])) bad = 1;
  });
  if (bad) {
    for (auto &w : why)
      if (!w.empty()) {
        msg = w;
        break;
      }
    err = SMASH_ERR_IO;
    return false;
  }
  return true;
}

// end of the line starting at p (the '\n'), inside [p, e)
inline const char *line_end(const char *p, const char *e) {
  const void *q = memchr(p, '\n', size_t(e - p));
  return q ? static_cast<const char *>(q) : nullptr;
}

// the longest name or bases line the parallel reader takes (parse() finds
// line ends within it); a longer one is "not strict": the streaming reader
// takes the input and reports it by its own rules
constexpr size_t kMaxLine = size_t(1) << 16;

// one strict record at r (r[0] == '@'): the end of its fourth line (its
// '\n'); nullptr = not strict
inline const char *strict_record(const char *r, const char *e) {
  if (r >= e || r[0] != '@') return nullptr;
  const char *l1 = line_end(r, e);
  if (!l1 || size_t(l1 - r) >= kMaxLine) return nullptr;
  const char *l2 = line_end(l1 + 1, e);
  if (!l2 || size_t(l2 - l1) > kMaxLine || l2 + 1 >= e || l2[1] != '+') return nullptr;
  const char *l3 = line_end(l2 + 1, e);
  return l3 ? line_end(l3 + 1, e) : nullptr;   // nullptr: no qualities line
}

// the first record start in [b, e) of a source's bytes [s0, send), or e
inline const char *resync(const char *s0, const char *send, const char *b, const char *e) {
  const char *q = b;
  if (q > s0 && q[-1] != '\n') {
    const char *x = line_end(q, send);
    if (!x) return e;
    q = x + 1;
  }
  while (q < e) {
    if (q[0] == '@') {   // '@' line: a name iff the line two below begins with '+'
      const char *l1 = line_end(q, send);
      const char *l2 = l1 ? line_end(l1 + 1, send) : nullptr;
      if (!l2) return e;
      if (l2 + 1 < send && l2[1] == '+') return q;
      q = l1 + 1;
      continue;
    }
    const char *x = line_end(q, send);
    if (!x) return e;
    q = x + 1;
  }
  return e;
}

// record starts of one mate list (its files in order), T threads over ranges
// of ~32 MB; false: not strict 4-line FASTQ
inline bool index_records(const std::vector<std::unique_ptr<Source>> &src, uint32_t T,
                          std::vector<const char *> &rec) {
  struct Range {
    const Source *s;
    size_t b, e;
    std::vector<const char *> r;
  };
  std::vector<Range> rg;
  const size_t step = size_t(32) << 20;
  for (const auto &sp : src)
    for (size_t b = 0; b < sp->n; b += step) rg.push_back(Range{sp.get(), b, std::min(sp->n, b + step), {}});
  std::atomic<size_t> next{0};
  std::atomic<int> bad{0};
  run_threads(std::min<uint32_t>(T, uint32_t(std::max<size_t>(rg.size(), 1))), [&](uint32_t) {
    for (size_t k; (k = next++) < rg.size() && !bad;) {
      Range &x = rg[k];
      const char *s0 = x.s->p, *send = s0 + x.s->n;
      const char *e = s0 + x.e;
      const char *r = x.b == 0 ? s0 : resync(s0, send, s0 + x.b, e);
      x.r.reserve(size_t(x.e - x.b) / 256);
      while (r < e) {
        const char *end = strict_record(r, send);
        if (!end) {
          bad = 1;
          break;
        }
        x.r.push_back(r);
        r = end + 1;
      }
    }
  });
  if (bad) return false;
  size_t tot = 0;
  for (auto &x : rg) tot += x.r.size();
  rec.resize(tot);
  std::vector<size_t> at(rg.size() + 1, 0);
  for (size_t k = 0; k < rg.size(); ++k) at[k + 1] = at[k] + rg[k].r.size();
  next = 0;
  run_threads(T, [&](uint32_t) {
    for (size_t k; (k = next++) < rg.size();)
      std::copy(rg[k].r.begin(), rg[k].r.end(), rec.begin() + long(at[k]));
  });
  return true;
}

// a strict record's name (first token after '@', ingest.hpp Reader::record)
// and bases (the line, less trailing '\r')
struct Rec {
  const char *name;
  uint32_t nn;
  const char *seq;
  uint32_t sn;
};
inline Rec parse(const char *r) {
  // (every line of an indexed record ends in '\n' within kMaxLine bytes)
  const char *l1 = static_cast<const char *>(memchr(r, '\n', kMaxLine));
  const char *nb = r + 1;
  while (nb < l1 && isspace(uint8_t(*nb))) ++nb;
  const char *ne = nb;
  while (ne < l1 && !isspace(uint8_t(*ne))) ++ne;
  const char *b = l1 + 1;
  const char *l2 = static_cast<const char *>(memchr(b, '\n', kMaxLine));
  const char *be = l2;
  while (be > b && be[-1] == '\r') --be;
  return Rec{nb, uint32_t(ne - nb), b, uint32_t(be - b)};
}

// replaceN + lowercasing (ingest.hpp lut), written so the compiler
// vectorises it (byte compares and selects, no table)
inline void convert(uint8_t *d, const char *s, uint32_t n) {
  for (uint32_t j = 0; j < n; ++j) {
    const uint8_t c = uint8_t(s[j]);
    const uint8_t lo = (c >= 'A' && c <= 'Z') ? uint8_t(c + 32) : c;
    d[j] = c == 'N' ? uint8_t('z') : lo;
  }
}

// the two lists, indexed: pairs = min(records of list 1, of list 2)
struct PairIndex {
  std::vector<std::unique_ptr<Source>> s1, s2;
  std::vector<const char *> r1, r2;
  uint64_t n = 0;
  // open and index both lists; returns SMASH_OK, SMASH_ERR_UNSUPPORTED (not
  // strict 4-line FASTQ: use the streaming reader) or an I/O error (msg)
  int build(const std::vector<std::string> &p1, const std::vector<std::string> &p2, uint32_t T,
            std::string &msg) {
    int err = 0;
    std::vector<std::string> all(p1);
    all.insert(all.end(), p2.begin(), p2.end());
    std::vector<std::unique_ptr<Source>> src;
    if (!load_sources(all, T, src, msg, err)) return err;
    for (size_t k = 0; k < src.size(); ++k) (k < p1.size() ? s1 : s2).push_back(std::move(src[k]));
    if (!index_records(s1, T, r1) || !index_records(s2, T, r2))
      return SMASH_ERR_UNSUPPORTED;
    n = std::min(r1.size(), r2.size());
    return SMASH_OK;
  }
};

// the pairs to emit, in order: input pair idx[k] for output k (idx empty: k
// itself); pairs whose two mates have no bases are dropped
struct Plan {
  uint64_t n_out = 0;
  std::vector<uint64_t> idx;
  uint32_t L = 0;
};

// Plan the emission of all indexed pairs (fastqs_to_sam.cpp:80 + the
// samtools sort -n order), with the checks of the streaming readers (feed.hip
// check_pairs / produce_stream, ingest.cpp smash_fastq_read):
//  * both mates empty: dropped; one empty: error (the first such pair);
//  * every mate has L bases (L = 0: the first kept pair's length, <= 255);
//  * order: check_order -- every kept pair's read-1 name >= the previous
//    kept pair's under strnum_cmp, else error; sort -- kept pairs stably
//    ordered by read-1 name.
// All of it on T threads, before any pair is emitted.  Returns SMASH_OK or
// an error code with msg.
inline int plan_pairs(const PairIndex &px, uint32_t T, uint32_t L, bool check_order, bool sort,
                      Plan &pl, std::string &msg) {
  const uint64_t n = px.n;
  pl = Plan();
  const bool given = L != 0;   // (the messages of the streaming readers)
  if (!L) {   // the first kept pair's length
    for (uint64_t i = 0; i < n; ++i) {
      const Rec a = parse(px.r1[i]), b = parse(px.r2[i]);
      if (a.sn == 0 && b.sn == 0) continue;
      L = a.sn ? a.sn : b.sn;
      break;
    }
    if (L > 255) {
      msg = "reads longer than 255 bases";
      return SMASH_ERR_UNSUPPORTED;
    }
  }
  pl.L = L;
  const uint32_t R = std::max<uint32_t>(1, std::min<uint64_t>(T * 4, (n + 4095) / 4096));
  std::vector<uint64_t> kept(R, 0), first_bad(R, ~0ull), disorder(R, ~0ull);
  std::vector<uint64_t> first_kept(R, ~0ull), last_kept(R, ~0ull);
  std::vector<int> kind(R, 0);
  std::vector<uint8_t> drop(n, 0);
  std::atomic<uint32_t> next{0};
  run_threads(std::min(T, R), [&](uint32_t) {
    for (uint32_t r; (r = next++) < R;) {
      const uint64_t lo = n * r / R, hi = n * (r + 1) / R;
      const char *pn = nullptr;
      uint32_t pl_ = 0;
      // (the range's results in locals, stored once: the per-range slots
      // share cache lines)
      uint64_t kp = 0, fb = ~0ull, fk = ~0ull, lk = ~0ull, dis = ~0ull;
      int kd = 0;
      for (uint64_t i = lo; i < hi; ++i) {
        const Rec a = parse(px.r1[i]), b = parse(px.r2[i]);
        int e = 0;
        if (a.sn == 0 && b.sn == 0) {
          drop[i] = 1;
          continue;
        }
        if (a.sn == 0 || b.sn == 0) e = 1;
        else if (a.sn != L || b.sn != L) e = 2;
        if (e && fb == ~0ull) {
          fb = i;
          kd = e;
        }
        ++kp;
        if (fk == ~0ull) fk = i;
        lk = i;
        if (check_order && pn && dis == ~0ull && strnum_cmp(pn, pl_, a.name, a.nn) > 0) dis = i;
        pn = a.name;
        pl_ = a.nn;
      }
      kept[r] = kp;
      first_bad[r] = fb;
      kind[r] = kd;
      first_kept[r] = fk;
      last_kept[r] = lk;
      disorder[r] = dis;
    }
  });
  auto name_of = [&](uint64_t i) {
    const Rec a = parse(px.r1[i]);
    return std::string(a.name, a.nn);
  };
  for (uint32_t r = 0; r < R; ++r)
    if (first_bad[r] != ~0ull) {
      msg = kind[r] == 1 ? "one mate of a pair has no bases (" + name_of(first_bad[r]) + ")"
            : given ? "every mate must have the pipeline's read length, " + std::to_string(L) +
                          " (" + name_of(first_bad[r]) + ")"
                    : "all mates must have the same length (" + name_of(first_bad[r]) + ")";
      return SMASH_ERR_ARG;
    }
  uint64_t tot = 0, prev = ~0ull;
  for (uint32_t r = 0; r < R; ++r) {
    tot += kept[r];
    if (check_order && first_kept[r] != ~0ull) {
      if (prev != ~0ull && disorder[r] == ~0ull) {   // the range's first against the last before
        const Rec a = parse(px.r1[prev]), b = parse(px.r1[first_kept[r]]);
        if (strnum_cmp(a.name, a.nn, b.name, b.nn) > 0) disorder[r] = first_kept[r];
      }
      if (disorder[r] != ~0ull) {
        msg = "pairs are not in samtools sort -n order at read " + name_of(disorder[r]) +
              " (use sort_names = 1)";
        return SMASH_ERR_ARG;
      }
    }
    if (last_kept[r] != ~0ull) prev = last_kept[r];
  }
  pl.n_out = tot;
  if (tot != n) {   // drops: the kept pairs' indices
    pl.idx.resize(tot);
    std::vector<uint64_t> at(R + 1, 0);
    for (uint32_t r = 0; r < R; ++r) at[r + 1] = at[r] + kept[r];
    next = 0;
    run_threads(std::min(T, R), [&](uint32_t) {
      for (uint32_t r; (r = next++) < R;) {
        uint64_t o = at[r];
        for (uint64_t i = n * r / R, hi = n * (r + 1) / R; i < hi; ++i)
          if (!drop[i]) pl.idx[o++] = i;
      }
    });
  }
  if (!sort || tot < 2) return SMASH_OK;
  // samtools sort -n: stable by read-1 name (strnum_cmp); already in order
  // (the usual case) costs one parallel pass
  struct NameV {
    const char *p;
    uint32_t n;
  };
  std::vector<NameV> nm(tot);
  std::vector<uint64_t> ord(tot);
  next = 0;
  std::atomic<int> unsorted{0};
  run_threads(std::min(T, R), [&](uint32_t) {
    for (uint32_t r; (r = next++) < R;) {
      const uint64_t lo = tot * r / R, hi = tot * (r + 1) / R;
      for (uint64_t k = lo; k < hi; ++k) {
        const Rec a = parse(px.r1[pl.idx.empty() ? k : pl.idx[k]]);
        nm[k] = NameV{a.name, a.nn};
        ord[k] = pl.idx.empty() ? k : pl.idx[k];
      }
    }
  });
  next = 0;
  run_threads(std::min(T, R), [&](uint32_t) {
    for (uint32_t r; (r = next++) < R;) {
      const uint64_t lo = std::max<uint64_t>(1, tot * r / R), hi = tot * (r + 1) / R;
      for (uint64_t k = lo; k < hi && !unsorted; ++k)
        if (strnum_cmp(nm[k - 1].p, nm[k - 1].n, nm[k].p, nm[k].n) > 0) unsorted = 1;
    }
  });
  if (!unsorted) return SMASH_OK;
  // T sorted runs (stable), then pairwise merges (std::merge keeps the first
  // run's element on ties: stable)
  std::vector<uint64_t> pos(tot);
  for (uint64_t k = 0; k < tot; ++k) pos[k] = k;
  auto less = [&](uint64_t x, uint64_t y) {
    return strnum_cmp(nm[x].p, nm[x].n, nm[y].p, nm[y].n) < 0;
  };
  const uint32_t runs = std::max<uint32_t>(1, std::min<uint64_t>(T, tot / 1024 + 1));
  std::vector<uint64_t> cut(runs + 1);
  for (uint32_t r = 0; r <= runs; ++r) cut[r] = tot * r / runs;
  run_threads(runs, [&](uint32_t r) {
    std::stable_sort(pos.begin() + long(cut[r]), pos.begin() + long(cut[r + 1]), less);
  });
  std::vector<uint64_t> tmp(tot);
  for (uint32_t w = 1; w < runs; w *= 2) {
    std::vector<std::pair<uint32_t, uint32_t>> jobs;
    for (uint32_t a = 0; a < runs; a += 2 * w) jobs.emplace_back(a, std::min(runs, a + 2 * w));
    std::atomic<size_t> jn{0};
    run_threads(std::min<uint32_t>(T, uint32_t(jobs.size())), [&](uint32_t) {
      for (size_t j; (j = jn++) < jobs.size();) {
        const uint64_t b = cut[jobs[j].first], m = cut[std::min(runs, jobs[j].first + w)],
                       e = cut[jobs[j].second];
        std::merge(pos.begin() + long(b), pos.begin() + long(m), pos.begin() + long(m),
                   pos.begin() + long(e), tmp.begin() + long(b), less);
      }
    });
    pos.swap(tmp);
  }
  pl.idx.resize(tot);
  for (uint64_t k = 0; k < tot; ++k) pl.idx[k] = ord[pos[k]];
  return SMASH_OK;
}

// output pairs [k0, k1) of the plan into out (2 * L bytes per pair: read 1,
// read 2, prepared) and, with names, read-1 names (stride bytes, NUL padded;
// false if one does not fit), T threads
inline bool pack_pairs(const PairIndex &px, const Plan &pl, uint64_t k0, uint64_t k1, uint8_t *out,
                       char *names, uint32_t stride, uint32_t T, uint32_t row = 0) {
  const uint32_t L = pl.L;
  const uint64_t RW = row ? row : L;   // bytes per mate row (the bytes past L: left as they are)
  const uint64_t n = k1 - k0;
  const uint32_t R = std::max<uint32_t>(1, std::min<uint64_t>(T * 4, (n + 4095) / 4096));
  std::atomic<uint32_t> next{0};
  std::atomic<int> bad{0};
  run_threads(std::min(T, R), [&](uint32_t) {
    for (uint32_t r; (r = next++) < R;) {
      for (uint64_t k = k0 + n * r / R, hi = k0 + n * (r + 1) / R; k < hi; ++k) {
        const uint64_t i = pl.idx.empty() ? k : pl.idx[k];
        const Rec a = parse(px.r1[i]), b = parse(px.r2[i]);
        uint8_t *d = out + (k - k0) * 2 * RW;
        convert(d, a.seq, L);
        convert(d + RW, b.seq, L);
        if (names) {
          if (a.nn >= stride) {
            bad = 1;
            continue;
          }
          char *o = names + (k - k0) * stride;
          memcpy(o, a.name, a.nn);
          memset(o + a.nn, 0, stride - a.nn);
        }
      }
    }
  });
  return !bad;
}

}  // namespace ingest
}  // namespace smash
