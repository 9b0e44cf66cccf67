// smash-paper_amd/csrc/fastq_shard.cpp -- rank-local FASTQ ingest for the
// multi-GPU driver.  Host code.
//
// The reference streams `zcat r1 lanes` and `zcat r2 lanes` into
// fastqs_to_sam | mummer (smash_mapping.sh:19), whose reader threads hold one
// ring of queries at a time (query.cpp:614-740).  Across W ranks the global
// pair order is (step, rank, pair) (dist.py), so rank r's batch of step s is
// pairs [s W B + r B, + B) -- spread over every file.  Here no rank reads the
// whole input:
//
//  pass 1 (scan): both mate lists are cut into segments -- plain files into
//    64 MB byte ranges, gzip files whole -- dealt to the ranks (largest
//    first, to the least loaded rank).  Each rank scans only its segments,
//    on its threads: the records that start in the segment (the strict
//    4-line FASTQ rule of fastq_par.hpp), the empty ones, the read-1 names at
//    the ends and any order break inside.  A gzip file is inflated once, in
//    bounded buffers, and leaves restart points every 32 MB of output at
//    deflate block boundaries (zlib's zran scheme: compressed offset, the
//    bits of the boundary byte, the 32 KB window before it) with the first
//    record start after each point and the records before it.
//  exchange: each rank's scan is one blob; the caller all-gathers the blobs.
//  open: every rank merges the blobs into the same plan (records per
//    segment, pairs = the shorter list, pairs whose two mates are empty
//    dropped, the order of the read-1 names checked across segments).
//  pass 2 (pack): a range of planned pairs is read by `threads` cursors that
//    each start at their first pair: a plain segment is mapped and its
//    records skipped from the segment's first one, a gzip file is inflated
//    from the restart point before the pair.  Only the bytes of the pairs
//    asked for (plus at most one segment or restart span before each
//    cursor's first pair) are read.
//
// Host memory per rank: the buffers of the cursors (~8 MB each), the restart
// windows of every gzip file (32 KB per 32 MB of FASTQ), the caller's pinned
// batches; never a whole file.  Input that is not strict 4-line FASTQ, whose
// last line has no newline, or (sort_names) is not in samtools sort -n order
// gets SMASH_ERR_UNSUPPORTED: the caller takes smash_fastq_index instead.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "fastq_par.hpp"
#include "ingest.hpp"

namespace smash {
void set_error(const std::string &msg);
}
using smash::set_error;
using smash::ingest::kMaxLine;
using smash::ingest::line_end;
using smash::ingest::resync;
using smash::ingest::run_threads;
using smash::ingest::strict_record;
using smash::ingest::strnum_cmp;

namespace {

// plain file segment; gzip restart point spacing (output bytes).  Tests set
// SMASH_SHARD_SEG_BYTES / SMASH_SHARD_AP_SPAN to exercise many of both on
// small files (every rank must use the same values: they shape the plan)
uint64_t env_u64(const char *name, uint64_t dflt) {
  const char *e = getenv(name);
  const long long v = e && *e ? atoll(e) : 0;
  return v > 0 ? uint64_t(v) : dflt;
}
constexpr uint32_t kWin = 32768;                      // deflate window
constexpr uint64_t kMagic = 0x3144524148534d53ull;    // "SMSHARD1"
constexpr size_t kInChunk = size_t(4) << 20;
// a strict record longer than this is refused (kMaxLine bounds the name and
// bases lines; the '+' and quality lines are not bounded by the strict rule)
constexpr size_t kMaxRecord = size_t(1) << 22;

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double>(b - a).count();
}

struct FileInfo {
  std::string path;
  uint64_t size = 0;
  bool gz = false;
};

struct Ap {   // gzip restart point
  uint64_t in = 0;       // compressed offset: the point follows byte in - 1 (bits of it unused)
  uint32_t bits = 0;
  uint32_t member = 0;   // 1: a gzip member header starts at `in` (no window)
  uint64_t out = 0;      // uncompressed offset of the point
  uint64_t rec_out = 0;  // the first record start at or after `out`
  uint64_t rec_idx = 0;  // the file's records before rec_out
  std::string win;
};

struct SegResult {
  uint32_t status = 0;   // SMASH_OK, SMASH_ERR_UNSUPPORTED (not strict), SMASH_ERR_IO
  std::string msg;
  uint64_t n = 0;        // records starting in the segment
  uint32_t first_len = 0;                 // bases of its first non-empty record
  std::vector<uint64_t> empty;            // local indices of records without bases
  // read-1 order: the first / last non-empty record (local index, name) and
  // the first local order break among non-empty records (~0: none)
  uint64_t first_i = ~0ull, last_i = ~0ull, break_i = ~0ull;
  std::string first_name, last_name, break_name;
  std::vector<Ap> aps;
  uint64_t bytes_in = 0, bytes_out = 0;   // compressed read, FASTQ bytes scanned
};

struct Segment {
  uint32_t list = 0, file = 0;
  uint64_t b = 0, e = 0;   // byte range (gzip: the whole file)
  uint64_t cost = 0;
  uint32_t owner = 0;
};

struct Lists {
  std::vector<FileInfo> f[2];
  std::vector<Segment> seg;   // list 0's in file order, then list 1's
  uint64_t seg_bytes = env_u64("SMASH_SHARD_SEG_BYTES", uint64_t(64) << 20);
  uint64_t ap_span = env_u64("SMASH_SHARD_AP_SPAN", uint64_t(32) << 20);
};

int load_lists(const char *const *r1, uint32_t n1, const char *const *r2, uint32_t n2,
               uint32_t world, Lists &L, std::string &msg) {
  for (int m = 0; m < 2; ++m) {
    const char *const *p = m ? r2 : r1;
    const uint32_t n = m ? n2 : n1;
    for (uint32_t i = 0; i < n; ++i) {
      FileInfo fi;
      fi.path = p[i];
      const int fd = open(p[i], O_RDONLY);
      struct stat st;
      if (fd < 0 || fstat(fd, &st) != 0) {
        if (fd >= 0) close(fd);
        msg = "cannot open " + fi.path;
        return SMASH_ERR_IO;
      }
      fi.size = uint64_t(st.st_size);
      unsigned char mg[2] = {0, 0};
      fi.gz = fi.size >= 2 && pread(fd, mg, 2, 0) == 2 && mg[0] == 0x1f && mg[1] == 0x8b;
      close(fd);
      L.f[m].push_back(fi);
    }
  }
  for (uint32_t m = 0; m < 2; ++m)
    for (uint32_t i = 0; i < L.f[m].size(); ++i) {
      const FileInfo &fi = L.f[m][i];
      if (fi.gz) {
        L.seg.push_back(Segment{m, i, 0, fi.size, 4 * fi.size, 0});
      } else {
        for (uint64_t b = 0; b < fi.size; b += L.seg_bytes)
          L.seg.push_back(Segment{m, i, b, std::min(fi.size, b + L.seg_bytes),
                                  std::min(fi.size, b + L.seg_bytes) - b, 0});
      }
    }
  // deal: largest first to the least loaded rank (ties: the lower index)
  std::vector<size_t> ord(L.seg.size());
  for (size_t k = 0; k < ord.size(); ++k) ord[k] = k;
  std::stable_sort(ord.begin(), ord.end(),
                   [&](size_t a, size_t b) { return L.seg[a].cost > L.seg[b].cost; });
  std::vector<uint64_t> load(world, 0);
  for (size_t k : ord) {
    uint32_t r = 0;
    for (uint32_t q = 1; q < world; ++q)
      if (load[q] < load[r]) r = q;
    L.seg[k].owner = r;
    load[r] += L.seg[k].cost + 1;
  }
  return SMASH_OK;
}

// a read-only mapping of a whole file
struct Mapping {
  const char *p = nullptr;
  size_t n = 0;
  Mapping() = default;
  Mapping(const Mapping &) = delete;
  Mapping &operator=(const Mapping &) = delete;
  ~Mapping() { reset(); }
  void reset() {
    if (p) munmap(const_cast<char *>(p), n);
    p = nullptr;
    n = 0;
  }
  bool map(const std::string &path, size_t size) {
    reset();
    if (!size) return true;
    const int fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) return false;
    void *m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return false;
    p = static_cast<const char *>(m);
    n = size;
    return true;
  }
};

// the per-record bookkeeping of a scan (order of the non-empty records' names)
struct ScanAcc {
  SegResult &r;
  explicit ScanAcc(SegResult &x) : r(x) {}
  void record(const char *rec) {
    const smash::ingest::Rec x = smash::ingest::parse(rec);
    const uint64_t i = r.n++;
    if (x.sn == 0) {
      r.empty.push_back(i);
      return;
    }
    if (r.first_i == ~0ull) {
      r.first_i = i;
      r.first_len = x.sn;
      r.first_name.assign(x.name, x.nn);
    } else if (r.break_i == ~0ull &&
               strnum_cmp(r.last_name.data(), r.last_name.size(), x.name, x.nn) > 0) {
      r.break_i = i;
      r.break_name.assign(x.name, x.nn);
    }
    r.last_i = i;
    r.last_name.assign(x.name, x.nn);
  }
};

void scan_plain(const FileInfo &fi, const Segment &sg, SegResult &r) {
  Mapping mp;
  if (!mp.map(fi.path, fi.size)) {
    r.status = SMASH_ERR_IO;
    r.msg = "cannot map " + fi.path;
    return;
  }
  const char *s0 = mp.p, *send = mp.p + mp.n;
  if (send[-1] != '\n') {
    r.status = SMASH_ERR_UNSUPPORTED;
    r.msg = fi.path + ": last line has no newline";
    return;
  }
  const char *e = s0 + sg.e;
  const char *q = sg.b == 0 ? s0 : resync(s0, send, s0 + sg.b, e);
  ScanAcc acc(r);
  while (q < e) {
    const char *end = strict_record(q, send);
    if (!end) {
      r.status = SMASH_ERR_UNSUPPORTED;
      r.msg = fi.path + ": not strict 4-line FASTQ";
      return;
    }
    acc.record(q);
    q = end + 1;
  }
  r.bytes_out = uint64_t(std::min(q, send) - (sg.b == 0 ? s0 : s0 + sg.b));
}

// zlib inflate of one gzip file from a restart point, members in sequence
struct Inflater {
  int fd = -1;
  z_stream zs;
  bool init = false, raw = false, done = false;
  std::vector<unsigned char> in;
  uint64_t in_file = 0;   // file offset of in[0]
  uint64_t consumed_base = 0;
  uint64_t out_abs = 0;   // uncompressed offset of the next output byte
  uint64_t read_bytes = 0;
  std::string err;

  ~Inflater() { close_(); }
  void close_() {
    if (init) inflateEnd(&zs);
    init = false;
    if (fd >= 0) close(fd);
    fd = -1;
  }
  // compressed bytes consumed from the file start
  uint64_t consumed() const { return in_file + (zs.next_in - in.data()); }
  bool fill() {
    const uint64_t at = consumed();
    if (zs.avail_in) memmove(in.data(), zs.next_in, zs.avail_in);
    const size_t keep = zs.avail_in;
    const ssize_t got = read(fd, in.data() + keep, in.size() - keep);
    if (got < 0) {
      err = "read error";
      return false;
    }
    read_bytes += uint64_t(got);
    in_file = at;
    zs.next_in = in.data();
    zs.avail_in = unsigned(keep + size_t(got));
    return true;
  }
  bool open_at(const std::string &path, const Ap &ap) {
    close_();
    in.resize(kInChunk);
    fd = open(path.c_str(), O_RDONLY);
    if (fd < 0) {
      err = "cannot open " + path;
      return false;
    }
    memset(&zs, 0, sizeof(zs));
    raw = !ap.member;
    if (inflateInit2(&zs, raw ? -15 : 47) != Z_OK) {
      err = "inflateInit2 failed";
      return false;
    }
    init = true;
    done = false;
    const uint64_t start = ap.in - (ap.bits ? 1 : 0);
    if (lseek(fd, off_t(start), SEEK_SET) < 0) {
      err = "seek failed";
      return false;
    }
    in_file = start;
    zs.next_in = in.data();
    zs.avail_in = 0;
    if (!fill()) return false;
    if (ap.bits) {
      if (!zs.avail_in) {
        err = "truncated gzip";
        return false;
      }
      const int c = zs.next_in[0];
      zs.next_in++;
      zs.avail_in--;
      if (inflatePrime(&zs, int(ap.bits), c >> (8 - ap.bits)) != Z_OK) {
        err = "inflatePrime failed";
        return false;
      }
    }
    if (raw && !ap.win.empty() &&
        inflateSetDictionary(&zs, reinterpret_cast<const Bytef *>(ap.win.data()),
                             uInt(ap.win.size())) != Z_OK) {
      err = "inflateSetDictionary failed";
      return false;
    }
    out_abs = ap.out;
    return true;
  }
  // up to cap bytes into dst; *n produced; flush Z_BLOCK stops at block ends
  // (the scan's restart points).  false: error (err).  At the end of the
  // file's last member `done` is set.
  bool step(char *dst, size_t cap, size_t *n, int flush) {
    *n = 0;
    if (done) return true;
    zs.next_out = reinterpret_cast<Bytef *>(dst);
    zs.avail_out = uInt(cap);
    for (;;) {
      if (!zs.avail_in && !fill()) return false;
      if (!zs.avail_in) {   // input ended inside a member
        if (zs.avail_out != cap) break;
        err = "truncated gzip";
        return false;
      }
      const int ret = inflate(&zs, flush);
      if (ret == Z_STREAM_END) {
        if (raw) {   // the member's 8-byte trailer (a raw restart does not read it)
          for (int k = 0; k < 8; ++k) {
            if (!zs.avail_in && !fill()) return false;
            if (!zs.avail_in) {
              err = "truncated gzip trailer";
              return false;
            }
            zs.next_in++;
            zs.avail_in--;
          }
        }
        if (zs.avail_in < 2 && !fill()) return false;
        if (zs.avail_in < 2 || zs.next_in[0] != 0x1f || zs.next_in[1] != 0x8b) {
          done = true;   // (trailing bytes that are no gzip member are ignored, as gzip -dc does)
          break;
        }
        if (inflateReset2(&zs, 47) != Z_OK) {
          err = "inflateReset2 failed";
          return false;
        }
        raw = false;
        member_start = true;
        break;
      }
      if (ret != Z_OK && ret != Z_BUF_ERROR) {
        err = std::string("inflate: ") + (zs.msg ? zs.msg : "error");
        return false;
      }
      if (!zs.avail_out) break;
      if (flush == Z_BLOCK && (zs.data_type & 128)) break;
    }
    *n = cap - zs.avail_out;
    out_abs += *n;
    return true;
  }
  bool member_start = false;
};

// the last kWin output bytes (a ring)
struct History {
  std::vector<char> ring = std::vector<char>(kWin);
  uint64_t total = 0;   // bytes ever pushed
  void push(const char *p, size_t n) {
    if (n >= kWin) {
      p += n - kWin;
      total += n - kWin;
      n = kWin;
    }
    const size_t at = size_t(total % kWin);
    const size_t a = std::min<size_t>(n, kWin - at);
    memcpy(ring.data() + at, p, a);
    memcpy(ring.data(), p + a, n - a);
    total += n;
  }
  std::string last(uint64_t k) const {   // the last min(k, kWin, total) bytes
    const size_t m = size_t(std::min<uint64_t>({k, uint64_t(kWin), total}));
    std::string s(m, '\0');
    for (size_t i = 0; i < m; ++i) s[i] = ring[size_t((total - m + i) % kWin)];
    return s;
  }
};

void scan_gz(const FileInfo &fi, uint64_t ap_span, SegResult &r) {
  Inflater z;
  Ap first;   // the file start: a member header at offset 0
  first.member = 1;
  if (!z.open_at(fi.path, first)) {
    r.status = SMASH_ERR_IO;
    r.msg = fi.path + ": " + z.err;
    return;
  }
  r.aps.push_back(first);
  std::vector<size_t> pending{0};   // restart points without their record yet
  History hist;
  uint64_t member_out0 = 0;   // output offset where the current member began
  std::vector<char> buf(size_t(8) << 20);
  size_t beg = 0, fill = 0;
  uint64_t buf_abs = 0;       // uncompressed offset of buf[0]
  ScanAcc acc(r);
  uint64_t last_ap = 0;
  bool ended = false;
  for (;;) {
    // parse the complete records in buf[beg, fill)
    while (beg < fill) {
      const char *q = buf.data() + beg, *e = buf.data() + fill;
      const char *end = strict_record(q, e);
      if (!end) {
        if (!ended && size_t(e - q) < kMaxRecord) break;   // more bytes needed
        r.status = SMASH_ERR_UNSUPPORTED;
        r.msg = fi.path + (ended ? ": truncated last record or no final newline"
                                 : ": not strict 4-line FASTQ");
        return;
      }
      const uint64_t at = buf_abs + beg;
      while (!pending.empty() && r.aps[pending.front()].out <= at) {
        r.aps[pending.front()].rec_out = at;
        r.aps[pending.front()].rec_idx = r.n;
        pending.erase(pending.begin());
      }
      acc.record(q);
      beg = size_t(end + 1 - buf.data());
    }
    if (ended) break;
    if (beg) {   // compact
      memmove(buf.data(), buf.data() + beg, fill - beg);
      fill -= beg;
      buf_abs += beg;
      beg = 0;
    }
    if (fill == buf.size()) buf.resize(buf.size() * 2);
    size_t n = 0;
    if (!z.step(buf.data() + fill, buf.size() - fill, &n, Z_BLOCK)) {
      r.status = SMASH_ERR_IO;
      r.msg = fi.path + ": " + z.err;
      return;
    }
    hist.push(buf.data() + fill, n);
    fill += n;
    if (z.done) {
      ended = true;
      continue;
    }
    if (z.member_start) {   // a new member: a restart point without a window
      z.member_start = false;
      member_out0 = z.out_abs;
      if (z.out_abs - last_ap >= ap_span) {
        Ap a;
        a.in = z.consumed();
        a.member = 1;
        a.out = z.out_abs;
        pending.push_back(r.aps.size());
        r.aps.push_back(a);
        last_ap = z.out_abs;
      }
    } else if ((z.zs.data_type & 128) && !(z.zs.data_type & 64) && z.out_abs - last_ap >= ap_span) {
      Ap a;   // a deflate block boundary inside the member
      a.in = z.consumed();
      a.bits = uint32_t(z.zs.data_type & 7);
      a.out = z.out_abs;
      a.win = hist.last(z.out_abs - member_out0);
      pending.push_back(r.aps.size());
      r.aps.push_back(a);
      last_ap = z.out_abs;
    }
  }
  if (fill && buf[fill - 1] != '\n') {
    r.status = SMASH_ERR_UNSUPPORTED;
    r.msg = fi.path + ": last line has no newline";
    return;
  }
  // points after the last record: no record follows them
  for (size_t k : pending) {
    r.aps[k].rec_out = buf_abs + fill;
    r.aps[k].rec_idx = r.n;
  }
  r.bytes_in = z.read_bytes;
  r.bytes_out = buf_abs + fill;
}

// ---- blobs -------------------------------------------------------------------
struct Writer {
  std::string s;
  void u(uint64_t x) { s.append(reinterpret_cast<const char *>(&x), 8); }
  void str(const std::string &x) {
    u(x.size());
    s.append(x);
  }
};
struct ReaderB {
  const char *p, *e;
  bool ok = true;
  uint64_t u() {
    if (e - p < 8) {
      ok = false;
      return 0;
    }
    uint64_t x;
    memcpy(&x, p, 8);
    p += 8;
    return x;
  }
  std::string str() {
    const uint64_t n = u();
    if (!ok || uint64_t(e - p) < n) {
      ok = false;
      return std::string();
    }
    std::string x(p, size_t(n));
    p += n;
    return x;
  }
};

uint64_t fingerprint(const Lists &L) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t x) { h = (h ^ x) * 1099511628211ull; };
  mix(L.seg_bytes);
  mix(L.ap_span);
  for (int m = 0; m < 2; ++m) {
    mix(L.f[m].size());
    for (const auto &f : L.f[m]) {
      mix(f.size);
      mix(f.gz);
    }
  }
  return h;
}

void put_result(Writer &w, uint64_t id, const SegResult &r) {
  w.u(id);
  w.u(r.status);
  w.str(r.msg);
  w.u(r.n);
  w.u(r.first_len);
  w.u(r.empty.size());
  for (uint64_t x : r.empty) w.u(x);
  w.u(r.first_i);
  w.u(r.last_i);
  w.u(r.break_i);
  w.str(r.first_name);
  w.str(r.last_name);
  w.str(r.break_name);
  w.u(r.aps.size());
  for (const Ap &a : r.aps) {
    w.u(a.in);
    w.u(a.bits);
    w.u(a.member);
    w.u(a.out);
    w.u(a.rec_out);
    w.u(a.rec_idx);
    w.str(a.win);
  }
  w.u(r.bytes_in);
  w.u(r.bytes_out);
}

bool get_result(ReaderB &rd, uint64_t &id, SegResult &r) {
  id = rd.u();
  r.status = uint32_t(rd.u());
  r.msg = rd.str();
  r.n = rd.u();
  r.first_len = uint32_t(rd.u());
  const uint64_t ne = rd.u();
  if (!rd.ok || ne > r.n) return false;
  r.empty.resize(ne);
  for (auto &x : r.empty) x = rd.u();
  r.first_i = rd.u();
  r.last_i = rd.u();
  r.break_i = rd.u();
  r.first_name = rd.str();
  r.last_name = rd.str();
  r.break_name = rd.str();
  const uint64_t na = rd.u();
  if (!rd.ok || na > (uint64_t(1) << 32)) return false;
  r.aps.resize(na);
  for (Ap &a : r.aps) {
    a.in = rd.u();
    a.bits = uint32_t(rd.u());
    a.member = uint32_t(rd.u());
    a.out = rd.u();
    a.rec_out = rd.u();
    a.rec_idx = rd.u();
    a.win = rd.str();
  }
  r.bytes_in = rd.u();
  r.bytes_out = rd.u();
  return rd.ok;
}

}  // namespace

// ---- the plan and its cursors --------------------------------------------------
struct smash_fastq_shards {
  Lists L;
  std::vector<SegResult> res;          // per segment
  std::vector<uint64_t> seg_first;     // global record index (within its list) of a segment's first
  std::vector<uint32_t> list_seg[2];   // segment ids of each list, in order
  std::vector<uint64_t> file_first[2]; // records before each file of a list
  uint64_t n_in = 0, n_out = 0;        // input pairs (zip), planned pairs
  std::vector<uint64_t> dropped;       // input pairs whose two mates are empty (sorted)
  uint32_t len = 0, threads = 1;
  std::mutex mu;
  smash_shard_stats st{};
};

namespace {

// records of list m, sequentially from input record i
struct Cursor {
  smash_fastq_shards *h;
  int m;
  uint32_t file = 0;
  bool gz = false;
  Mapping mp;
  const char *cur = nullptr, *end = nullptr;   // plain: the mapping; gz: buf[beg, fill)
  Inflater z;
  std::vector<char> buf;
  size_t beg = 0, fill = 0;
  std::string err;
  uint64_t bytes_out = 0, bytes_in = 0;

  const Segment &seg(uint32_t s) const { return h->L.seg[s]; }
  const FileInfo &fi() const { return h->L.f[m][file]; }

  bool open_file_at_start(uint32_t f) {
    file = f;
    gz = fi().gz;
    if (!gz) {
      if (!mp.map(fi().path, fi().size)) {
        err = "cannot map " + fi().path;
        return false;
      }
      cur = mp.p;
      end = mp.p + mp.n;
      return true;
    }
    Ap a;
    a.member = 1;
    return open_gz(a, 0);
  }
  bool open_gz(const Ap &a, uint64_t skip_to) {
    mp.reset();
    if (!z.open_at(fi().path, a)) {
      err = fi().path + ": " + z.err;
      return false;
    }
    if (buf.empty()) buf.resize(size_t(8) << 20);
    beg = fill = 0;
    // drop the output before skip_to (the record start)
    uint64_t abs = a.out;
    while (abs < skip_to) {
      size_t n = 0;
      const size_t want = size_t(std::min<uint64_t>(buf.size(), skip_to - abs));
      if (!z.step(buf.data(), want, &n, Z_NO_FLUSH)) {
        err = fi().path + ": " + z.err;
        return false;
      }
      if (!n && z.done) break;
      z.member_start = false;
      abs += n;
    }
    cur = end = buf.data();
    return true;
  }
  // position at input record i (i < the list's records)
  bool seek(uint64_t i) {
    const auto &ls = h->list_seg[m];
    // the segment holding record i: the first whose end is past i
    size_t lo = 0, hi = ls.size();
    while (lo < hi) {
      const size_t mid = (lo + hi) / 2;
      const uint32_t s = ls[mid];
      if (h->seg_first[s] + h->res[s].n <= i) lo = mid + 1;
      else hi = mid;
    }
    if (lo == ls.size()) {
      err = "record index past the list";
      return false;
    }
    const uint32_t s = ls[lo];
    uint64_t skip = i - h->seg_first[s];
    file = seg(s).file;
    gz = fi().gz;
    if (!gz) {
      if (!mp.map(fi().path, fi().size)) {
        err = "cannot map " + fi().path;
        return false;
      }
      const char *s0 = mp.p, *send = mp.p + mp.n;
      cur = seg(s).b == 0 ? s0 : resync(s0, send, s0 + seg(s).b, s0 + seg(s).e);
      end = send;
    } else {
      const auto &aps = h->res[s].aps;
      size_t k = 0;   // the last restart point with rec_idx <= skip
      for (size_t j = 1; j < aps.size(); ++j)
        if (aps[j].rec_idx <= skip) k = j;
      if (!open_gz(aps[k], aps[k].rec_out)) return false;
      skip -= aps[k].rec_idx;
    }
    for (; skip; --skip) {
      const char *r = next_record();
      if (!r) {
        if (err.empty()) err = "fewer records than the scan counted";
        return false;
      }
    }
    return true;
  }
  // the next record's start (valid until the next call), nullptr at the end
  // of the list or on error (err)
  const char *next_record() {
    for (;;) {
      if (!gz) {
        if (cur < end) {
          const char *e = strict_record(cur, end);
          if (!e) {
            err = fi().path + ": not strict 4-line FASTQ";
            return nullptr;
          }
          const char *r = cur;
          bytes_out += uint64_t(e + 1 - cur);
          cur = e + 1;
          return r;
        }
      } else {
        for (;;) {
          const char *e = cur < end ? strict_record(cur, end) : nullptr;
          if (e) {
            const char *r = cur;
            bytes_out += uint64_t(e + 1 - cur);
            cur = e + 1;
            return r;
          }
          if (z.done) {
            if (cur < end) {
              err = fi().path + ": truncated last record";
              return nullptr;
            }
            break;
          }
          if (size_t(end - cur) >= kMaxRecord) {
            err = fi().path + ": not strict 4-line FASTQ";
            return nullptr;
          }
          // refill: keep [cur, end), inflate more after it
          const size_t keep = size_t(end - cur);
          if (keep && cur != buf.data()) memmove(buf.data(), cur, keep);
          fill = keep;
          if (fill == buf.size()) buf.resize(buf.size() * 2);
          size_t n = 0;
          if (!z.step(buf.data() + fill, buf.size() - fill, &n, Z_NO_FLUSH)) {
            err = fi().path + ": " + z.err;
            return nullptr;
          }
          z.member_start = false;
          fill += n;
          cur = buf.data();
          end = buf.data() + fill;
        }
      }
      // end of this file: the next one of the list
      bytes_in += gz ? z.read_bytes : 0;
      if (file + 1 >= h->L.f[m].size()) return nullptr;
      if (!open_file_at_start(file + 1)) return nullptr;
    }
  }
  void finish() {
    if (gz) bytes_in += z.read_bytes;
    z.read_bytes = 0;
  }
};

}  // namespace

extern "C" int smash_fastq_shard_scan(const char *const *r1, uint32_t n1, const char *const *r2,
                                      uint32_t n2, uint32_t world, uint32_t rank,
                                      uint32_t threads, void **blob, uint64_t *blob_bytes) {
  if (!r1 || !r2 || !n1 || !n2 || !world || rank >= world || !blob || !blob_bytes) {
    set_error("smash_fastq_shard_scan: bad arguments");
    return SMASH_ERR_ARG;
  }
  const auto t0 = Clock::now();
  Lists L;
  std::string msg;
  if (int rc = load_lists(r1, n1, r2, n2, world, L, msg)) {
    set_error("smash_fastq_shard_scan: " + msg);
    return rc;
  }
  std::vector<uint32_t> mine;
  for (uint32_t s = 0; s < L.seg.size(); ++s)
    if (L.seg[s].owner == rank) mine.push_back(s);
  std::vector<SegResult> res(mine.size());
  std::atomic<size_t> next{0};
  run_threads(std::max<uint32_t>(1, std::min<uint32_t>(threads ? threads : 1, uint32_t(mine.size()))),
              [&](uint32_t) {
                for (size_t k; (k = next++) < mine.size();) {
                  const Segment &sg = L.seg[mine[k]];
                  const FileInfo &fi = L.f[sg.list][sg.file];
                  if (fi.gz) scan_gz(fi, L.ap_span, res[k]);
                  else scan_plain(fi, sg, res[k]);
                }
              });
  Writer w;
  w.u(kMagic);
  w.u(world);
  w.u(rank);
  w.u(fingerprint(L));
  w.u(L.seg.size());
  w.u(mine.size());
  for (size_t k = 0; k < mine.size(); ++k) put_result(w, mine[k], res[k]);
  uint64_t t_us = uint64_t(secs(t0, Clock::now()) * 1e6);
  w.u(t_us);
  char *out = static_cast<char *>(malloc(w.s.size()));
  if (!out) {
    set_error("smash_fastq_shard_scan: out of host memory");
    return SMASH_ERR_NOMEM;
  }
  memcpy(out, w.s.data(), w.s.size());
  *blob = out;
  *blob_bytes = w.s.size();
  return SMASH_OK;
}

extern "C" void smash_fastq_shard_free_blob(void *blob) { free(blob); }

extern "C" int smash_fastq_shard_open(const char *const *r1, uint32_t n1, const char *const *r2,
                                      uint32_t n2, uint32_t world, uint32_t rank,
                                      const void *const *blobs, const uint64_t *blob_bytes,
                                      uint32_t threads, uint32_t *len, int sort_names,
                                      smash_fastq_shards **out, uint64_t *n_pairs) {
  if (!r1 || !r2 || !n1 || !n2 || !world || rank >= world || !blobs || !blob_bytes || !len ||
      !out || !n_pairs) {
    set_error("smash_fastq_shard_open: bad arguments");
    return SMASH_ERR_ARG;
  }
  auto h = std::make_unique<smash_fastq_shards>();
  h->threads = threads ? threads : 1;
  std::string msg;
  if (int rc = load_lists(r1, n1, r2, n2, world, h->L, msg)) {
    set_error("smash_fastq_shard_open: " + msg);
    return rc;
  }
  const uint64_t fp = fingerprint(h->L);
  const size_t S = h->L.seg.size();
  h->res.resize(S);
  std::vector<uint8_t> have(S, 0);
  for (uint32_t r = 0; r < world; ++r) {
    ReaderB rd{static_cast<const char *>(blobs[r]), static_cast<const char *>(blobs[r]) + blob_bytes[r]};
    if (rd.u() != kMagic || rd.u() != world || rd.u() != r || rd.u() != fp || rd.u() != S) {
      set_error("smash_fastq_shard_open: blob " + std::to_string(r) +
                " is not a scan of these files by rank " + std::to_string(r) + " of " +
                std::to_string(world));
      return SMASH_ERR_ARG;
    }
    const uint64_t k = rd.u();
    for (uint64_t j = 0; j < k && rd.ok; ++j) {
      uint64_t id = 0;
      SegResult x;
      if (!get_result(rd, id, x) || id >= S || have[id] || h->L.seg[id].owner != r) {
        set_error("smash_fastq_shard_open: malformed blob " + std::to_string(r));
        return SMASH_ERR_ARG;
      }
      h->res[id] = std::move(x);
      have[id] = 1;
    }
    const double t = double(rd.u()) * 1e-6;
    if (!rd.ok) {
      set_error("smash_fastq_shard_open: malformed blob " + std::to_string(r));
      return SMASH_ERR_ARG;
    }
    if (r == rank) {
      h->st.scan_s = t;
      for (size_t s = 0; s < S; ++s)
        if (h->L.seg[s].owner == r) {
          h->st.scan_bytes_in += h->res[s].bytes_in ? h->res[s].bytes_in
                                                    : (h->L.f[h->L.seg[s].list][h->L.seg[s].file].gz
                                                           ? 0 : h->res[s].bytes_out);
          h->st.scan_bytes += h->res[s].bytes_out;
          ++h->st.scan_segments;
        }
    }
  }
  for (size_t s = 0; s < S; ++s) {
    if (!have[s]) {
      set_error("smash_fastq_shard_open: segment " + std::to_string(s) + " was not scanned");
      return SMASH_ERR_ARG;
    }
    if (h->res[s].status) {
      set_error("smash_fastq_shard_open: " + h->res[s].msg);
      return int(h->res[s].status);
    }
  }
  for (const auto &f : h->L.f[0]) h->st.input_bytes += f.size;
  for (const auto &f : h->L.f[1]) h->st.input_bytes += f.size;
  // records per list and segment
  h->seg_first.assign(S, 0);
  uint64_t tot[2] = {0, 0};
  for (uint32_t s = 0; s < S; ++s) {
    const uint32_t m = h->L.seg[s].list;
    h->list_seg[m].push_back(s);
    h->seg_first[s] = tot[m];
    tot[m] += h->res[s].n;
  }
  h->n_in = std::min(tot[0], tot[1]);
  // pairs whose two mates are empty are dropped (fastqs_to_sam.cpp:80)
  std::vector<uint64_t> e[2];
  for (uint32_t s = 0; s < S; ++s)
    for (uint64_t x : h->res[s].empty) e[h->L.seg[s].list].push_back(h->seg_first[s] + x);
  for (int m = 0; m < 2; ++m) std::sort(e[m].begin(), e[m].end());
  std::set_intersection(e[0].begin(), e[0].end(), e[1].begin(), e[1].end(),
                        std::back_inserter(h->dropped));
  while (!h->dropped.empty() && h->dropped.back() >= h->n_in) h->dropped.pop_back();
  h->n_out = h->n_in - h->dropped.size();
  // read-1 order (samtools sort -n) over the non-empty mate-1 records of the
  // pairs: inside every segment (scanned) and across segment boundaries
  {
    const std::string *prev = nullptr;
    for (uint32_t s : h->list_seg[0]) {
      const SegResult &x = h->res[s];
      const uint64_t g0 = h->seg_first[s];
      if (x.first_i == ~0ull || g0 + x.first_i >= h->n_in) continue;
      std::string bad;
      if (prev && strnum_cmp(prev->data(), prev->size(), x.first_name.data(), x.first_name.size()) > 0)
        bad = x.first_name;
      else if (x.break_i != ~0ull && g0 + x.break_i < h->n_in)
        bad = x.break_name;
      if (!bad.empty()) {
        if (sort_names) {
          set_error("smash_fastq_shard_open: pairs are not in samtools sort -n order (" + bad +
                    "): sorting needs the whole input (smash_fastq_index)");
          return SMASH_ERR_UNSUPPORTED;
        }
        set_error("smash_fastq_shard_open: pairs are not in samtools sort -n order at read " + bad +
                  " (use sort_names = 1)");
        return SMASH_ERR_ARG;
      }
      prev = &x.last_name;
    }
  }
  // read length: the given one, else the first non-empty read-1 record's
  uint32_t L0 = *len;
  if (!L0)
    for (uint32_t s : h->list_seg[0])
      if (h->res[s].first_i != ~0ull) {
        L0 = h->res[s].first_len;
        break;
      }
  if (L0 > 255) {
    set_error("smash_fastq_shard_open: reads longer than 255 bases");
    return SMASH_ERR_UNSUPPORTED;
  }
  h->len = L0;
  *len = L0;
  *n_pairs = h->n_out;
  *out = h.release();
  return SMASH_OK;
}

extern "C" int smash_fastq_shard_pack(smash_fastq_shards *h, uint64_t k0, uint64_t k1,
                                      uint8_t *h_reads) {
  if (!h || k1 < k0 || k1 > h->n_out || (k1 > k0 && !h_reads)) {
    set_error("smash_fastq_shard_pack: bad arguments");
    return SMASH_ERR_ARG;
  }
  if (k1 == k0) return SMASH_OK;
  const auto t0 = Clock::now();
  const uint32_t L = h->len;
  const uint64_t n = k1 - k0;
  // planned pair k -> input pair: k + the dropped pairs at or before it
  auto input_of = [&](uint64_t k) {
    uint64_t i = k;
    for (;;) {
      const uint64_t d = uint64_t(std::upper_bound(h->dropped.begin(), h->dropped.end(), i) -
                                  h->dropped.begin());
      if (k + d == i) return i;
      i = k + d;
    }
  };
  const uint32_t T = std::max<uint32_t>(1, std::min<uint64_t>(h->threads, (n + 65535) / 65536));
  std::vector<std::string> errs(T);
  std::vector<uint64_t> err_at(T, ~0ull);
  std::atomic<uint64_t> bin{0}, bout{0};
  run_threads(T, [&](uint32_t t) {
    const uint64_t a = k0 + n * t / T, b = k0 + n * (t + 1) / T;
    if (a == b) return;
    Cursor c1{h, 0}, c2{h, 1};
    uint64_t i = input_of(a);
    if (!c1.seek(i) || !c2.seek(i)) {
      errs[t] = !c1.err.empty() ? c1.err : c2.err;
      err_at[t] = a;
      return;
    }
    size_t dj = size_t(std::lower_bound(h->dropped.begin(), h->dropped.end(), i) - h->dropped.begin());
    for (uint64_t k = a; k < b; ++i) {
      const char *ra = c1.next_record(), *rb = c2.next_record();
      if (!ra || !rb) {
        errs[t] = !c1.err.empty() ? c1.err : !c2.err.empty() ? c2.err : "input ended early";
        err_at[t] = k;
        return;
      }
      if (dj < h->dropped.size() && h->dropped[dj] == i) {   // both mates empty
        ++dj;
        continue;
      }
      const smash::ingest::Rec x = smash::ingest::parse(ra), y = smash::ingest::parse(rb);
      if (x.sn == 0 || y.sn == 0 || x.sn != L || y.sn != L) {
        errs[t] = (x.sn == 0 || y.sn == 0)
                      ? "one mate of a pair has no bases (" + std::string(x.name, x.nn) + ")"
                      : "every mate must have the pipeline's read length, " + std::to_string(L) +
                            " (" + std::string(x.name, x.nn) + ")";
        err_at[t] = k;
        return;
      }
      uint8_t *d = h_reads + (k - k0) * 2 * L;
      smash::ingest::convert(d, x.seq, L);
      smash::ingest::convert(d + L, y.seq, L);
      ++k;
    }
    c1.finish();
    c2.finish();
    bin += c1.bytes_in + c2.bytes_in;
    bout += c1.bytes_out + c2.bytes_out;
  });
  {
    std::lock_guard<std::mutex> g(h->mu);
    h->st.pack_s += secs(t0, Clock::now());
    h->st.pack_bytes += bout.load();
    h->st.pack_bytes_in += bin.load();
    h->st.pack_pairs += n;
  }
  uint32_t w = T;
  for (uint32_t t = 0; t < T; ++t)
    if (err_at[t] != ~0ull && (w == T || err_at[t] < err_at[w])) w = t;
  if (w != T) {
    set_error("smash_fastq_shard_pack: " + errs[w]);
    return SMASH_ERR_ARG;
  }
  return SMASH_OK;
}

extern "C" int smash_fastq_shard_stats(smash_fastq_shards *h, smash_shard_stats *st) {
  if (!h || !st) return SMASH_ERR_ARG;
  std::lock_guard<std::mutex> g(h->mu);
  *st = h->st;
  return SMASH_OK;
}

extern "C" void smash_fastq_shard_close(smash_fastq_shards *h) { delete h; }
