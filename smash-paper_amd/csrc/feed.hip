// smash-paper_amd/csrc/feed.hip -- file-fed counting: the FASTQ/FASTA read
// lists of both mates -> pinned host batches -> H2D -> smash_count_batch,
// with parsing, copies and compute overlapped.
//
// This is the front of smash_mapping.sh:19-25 (zcat | fastqs_to_sam |
// samtools sort -n | memsam ...) feeding the device pipeline, organised like
// the reference's reader threads feeding its workers (query.cpp:614-740):
//   * producer: the two mate lists are parsed on two threads (ingest.hpp,
//     zlib for gzip), zipped into a pinned host batch by `threads` workers
//     (replaceN + lowercasing, pair checks as smash_fastq_read);
//   * consumer (the calling thread): per batch, an H2D copy on a copy stream
//     into one of two device buffers, then smash_count_batch on the compute
//     stream once the copy's event fires; the copy of batch b+1 runs under
//     the compute of batch b, the parse of b+2 under both.
// Pair order: the pipeline wants pairs in `samtools sort -n` order.  With
// sort_names = 0 the input must already be in that order (checked on the
// read-1 names as they stream; an out-of-order pair is SMASH_ERR_ARG, counts
// then partial); with sort_names = 1 every pair is read first (host memory),
// ordered by strnum_cmp (stable), and then streamed through the same
// copy / compute overlap.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <numeric>
#include <thread>

#include "common.hpp"
#include "fastq_par.hpp"
#include "ingest.hpp"

using smash::ingest::Chunk;
using smash::ingest::Reader;
using smash::ingest::strnum_cmp;

namespace smash {
uint32_t pipe_read_len(const smash_pipeline *p);
uint32_t pipe_stride(const smash_pipeline *p);
uint64_t pipe_max_pairs(const smash_pipeline *p);
int pipe_device(const smash_pipeline *p);
void *&pipe_feed(smash_pipeline *p, void (*freer)(void *));
}  // namespace smash

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double>(b - a).count();
}

// run f(lo, hi) over [0, n) on up to T threads
template <class F>
void par_for(uint64_t n, uint32_t T, F f) {
  if (T <= 1 || n < 4096) {
    f(uint64_t(0), n);
    return;
  }
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < T; ++t) {
    const uint64_t lo = n * t / T, hi = n * (t + 1) / T;
    th.emplace_back([&, lo, hi] { f(lo, hi); });
  }
  for (auto &x : th) x.join();
}

struct Slot {
  uint8_t *h = nullptr;   // pinned [2 * max_pairs * L] (FeedBufs)
  uint64_t n = 0;
  bool last = false;
  int state = 0;          // 0 free, 1 filled
};

// the pinned slots, device buffers, events and copy stream of the feed,
// owned by the pipeline between calls (pipe_feed)
struct FeedBufs {
  uint64_t bytes = 0;
  uint8_t *h[3] = {nullptr, nullptr, nullptr};
  uint8_t *d[2] = {nullptr, nullptr};
  hipEvent_t copied[2] = {nullptr, nullptr}, done[2] = {nullptr, nullptr};
  hipStream_t xs = nullptr;
  ~FeedBufs() {
    if (xs) (void)hipStreamSynchronize(xs);
    for (int k = 0; k < 2; ++k) {
      if (d[k]) (void)hipFree(d[k]);
      if (copied[k]) (void)hipEventDestroy(copied[k]);
      if (done[k]) (void)hipEventDestroy(done[k]);
    }
    for (auto *x : h)
      if (x) (void)hipHostFree(x);
    if (xs) (void)hipStreamDestroy(xs);
  }
  bool alloc(uint64_t b) {
    bytes = b;
    bool ok = hipStreamCreateWithFlags(&xs, hipStreamNonBlocking) == hipSuccess;
    for (int k = 0; k < 2 && ok; ++k)
      ok = hipMalloc(&d[k], b) == hipSuccess &&
           hipEventCreateWithFlags(&copied[k], hipEventDisableTiming) == hipSuccess &&
           hipEventCreateWithFlags(&done[k], hipEventDisableTiming) == hipSuccess;
    for (auto *&x : h) {
      ok = ok && hipHostMalloc(reinterpret_cast<void **>(&x), b, hipHostMallocDefault) == hipSuccess;
      if (ok) memset(x, 0, b);   // the rows' pads stay zero: packing writes only [0, L) of a row
    }
    return ok;
  }
};
void free_feed(void *f) { delete static_cast<FeedBufs *>(f); }

struct Feed {
  smash_pipeline *p;
  uint32_t L, T;
  uint32_t S;   // bytes per mate row in the batches (the pipeline's read stride)
  uint64_t B;
  Reader r1, r2;
  Chunk c1, c2;
  std::string prev_name;   // read-1 name of the last pair streamed (order check)
  bool have_prev = false;
  // shared state
  std::mutex mu;
  std::condition_variable cv;
  Slot slot[3];
  uint64_t next_slot = 0;  // the producers fill slot[next_slot % 3] in turn (one may hand over)
  int err = 0;
  std::string msg;
  double ingest_s = 0;
  double index_s = 0;      // parallel path: map / inflate + index + checks, before batch 0
  bool parallel = false;   // the parallel producer ran

  void fail(int e, const std::string &m) {
    std::lock_guard<std::mutex> g(mu);
    if (!err) {
      err = e;
      msg = m;
    }
    cv.notify_all();
  }
  bool failed() {
    std::lock_guard<std::mutex> g(mu);
    return err != 0;
  }

  // parse up to `want` pairs (both lists on two threads); n pairs ready in
  // c1 / c2; false at error
  bool parse(uint64_t want, uint64_t &n, bool &end) {
    std::thread t([&] { c2.parse(r2, want, false); });
    c1.parse(r1, want, true);
    t.join();
    if (c1.err || c2.err) {
      fail(c1.err ? c1.err : c2.err, c1.err ? r1.msg : r2.msg);
      return false;
    }
    n = std::min(c1.size(), c2.size());
    end = c1.end || c2.end;   // zip(): the shorter list ends the pairs
    return true;
  }

  // pair checks of pairs [0, n) of c1 / c2 (both mates empty: dropped, one
  // empty: error, other lengths: error); keep[i] = pair kept
  bool check_pairs(uint64_t n, std::vector<uint8_t> &keep) {
    keep.assign(n, 1);
    std::atomic<int> bad{0};
    std::atomic<uint64_t> where{~0ull};
    par_for(n, T, [&](uint64_t lo, uint64_t hi) {
      for (uint64_t i = lo; i < hi; ++i) {
        const uint64_t la = c1.boff[i + 1] - c1.boff[i], lb = c2.boff[i + 1] - c2.boff[i];
        int e = 0;
        if (la == 0 && lb == 0) keep[i] = 0;
        else if (la == 0 || lb == 0) e = 1;
        else if (la != L || lb != L) e = 2;
        if (e) {
          uint64_t w = where.load();
          while (i < w && !where.compare_exchange_weak(w, i)) {
          }
          bad = 1;
        }
      }
    });
    if (!bad) return true;
    const uint64_t i = where.load();
    const std::string na(c1.names.data() + c1.noff[i], c1.noff[i + 1] - c1.noff[i]);
    const uint64_t la = c1.boff[i + 1] - c1.boff[i], lb = c2.boff[i + 1] - c2.boff[i];
    if (la == 0 || lb == 0)
      fail(SMASH_ERR_ARG, "smash_count_fastq: one mate of a pair has no bases (" + na + ")");
    else
      fail(SMASH_ERR_ARG, "smash_count_fastq: every mate must have the pipeline's read length (" +
                              na + ")");
    return false;
  }

  // streaming producer (input already in name order)
  void produce_stream() {
    const uint8_t *lut = smash::ingest::lut();
    std::vector<uint8_t> keep;
    std::vector<uint64_t> dst;
    for (;;) {
      Slot &s = slot[next_slot++ % 3];
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return s.state == 0 || err; });
        if (err) return;
      }
      const auto t0 = Clock::now();
      uint64_t n = 0;
      bool end = false;
      if (!parse(B, n, end) || !check_pairs(n, keep)) return;
      // destination pair index of each kept pair, and the order check
      dst.resize(n);
      uint64_t k = 0;
      for (uint64_t i = 0; i < n; ++i) dst[i] = keep[i] ? k++ : ~0ull;
      std::atomic<uint64_t> disorder{~0ull};
      par_for(n, T, [&](uint64_t lo, uint64_t hi) {
        const char *prev = nullptr;
        size_t pn = 0;
        for (uint64_t i = lo; i < hi; ++i) {
          if (!keep[i]) continue;
          const char *nm = c1.names.data() + c1.noff[i];
          const size_t nn = c1.noff[i + 1] - c1.noff[i];
          if (!prev && i > 0) {   // the kept pair before this range
            for (uint64_t j = i; j-- > 0;)
              if (keep[j]) {
                prev = c1.names.data() + c1.noff[j];
                pn = c1.noff[j + 1] - c1.noff[j];
                break;
              }
          }
          if (!prev && have_prev) {
            prev = prev_name.data();
            pn = prev_name.size();
          }
          if (prev && strnum_cmp(prev, pn, nm, nn) > 0) {
            uint64_t w = disorder.load();
            while (i < w && !disorder.compare_exchange_weak(w, i)) {
            }
            break;
          }
          prev = nm;
          pn = nn;
          const uint8_t *a = reinterpret_cast<const uint8_t *>(c1.bases.data() + c1.boff[i]);
          const uint8_t *bb = reinterpret_cast<const uint8_t *>(c2.bases.data() + c2.boff[i]);
          uint8_t *d = s.h + dst[i] * 2 * S;
          for (uint32_t j = 0; j < L; ++j) d[j] = lut[a[j]];
          for (uint32_t j = 0; j < L; ++j) d[S + j] = lut[bb[j]];
        }
      });
      if (disorder.load() != ~0ull) {
        const uint64_t i = disorder.load();
        fail(SMASH_ERR_ARG,
             "smash_count_fastq: pairs are not in samtools sort -n order at read " +
                 std::string(c1.names.data() + c1.noff[i], c1.noff[i + 1] - c1.noff[i]) +
                 " (use sort_names = 1)");
        return;
      }
      for (uint64_t i = n; i-- > 0;)
        if (keep[i]) {
          prev_name.assign(c1.names.data() + c1.noff[i], c1.noff[i + 1] - c1.noff[i]);
          have_prev = true;
          break;
        }
      {
        std::lock_guard<std::mutex> g(mu);
        ingest_s += secs(t0, Clock::now());
        s.n = k;
        s.last = end;
        s.state = 1;
      }
      cv.notify_all();
      if (end) return;
    }
  }

  // parallel producer (fastq_par.hpp): every file mapped / inflated and
  // indexed by byte range, the pairs checked, ordered (sort_names) or checked
  // for order, all on T threads; then batches packed on T threads.  false:
  // the input is not strict 4-line FASTQ (nothing consumed: the streaming
  // producers take it from the start)
  bool produce_parallel(bool sort_names) {
    namespace I = smash::ingest;
    const auto t0 = Clock::now();
    I::PairIndex px;
    std::string m;
    int rc = px.build(r1.paths, r2.paths, T, m);
    if (rc == SMASH_ERR_UNSUPPORTED) return false;
    I::Plan pl;
    if (rc == SMASH_OK) rc = I::plan_pairs(px, T, L, !sort_names, sort_names, pl, m);
    if (rc != SMASH_OK) {
      fail(rc, "smash_count_fastq: " + m);
      return true;
    }
    {
      std::lock_guard<std::mutex> g(mu);
      ingest_s += secs(t0, Clock::now());
      index_s = secs(t0, Clock::now());
      parallel = true;
    }
    for (uint64_t k0 = 0;;) {
      Slot &s = slot[next_slot++ % 3];
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return s.state == 0 || err; });
        if (err) return true;
      }
      const auto t1 = Clock::now();
      const uint64_t k = std::min(B, pl.n_out - k0);
      I::pack_pairs(px, pl, k0, k0 + k, s.h, nullptr, 0, T, S);
      k0 += k;
      const bool end = k0 >= pl.n_out;
      {
        std::lock_guard<std::mutex> g(mu);
        ingest_s += secs(t1, Clock::now());
        s.n = k;
        s.last = end;
        s.state = 1;
      }
      cv.notify_all();
      if (end) return true;
    }
  }

  // streaming parallel producer for gzip lane lists (input in name order):
  // worker threads inflate (or map) the files of both lists in the order the
  // pairs need them -- the two lists interleaved by cumulative size, at most
  // 2 T files ahead of the packer -- and index each file's records as it
  // lands; the packer fills the pinned batches from the files already
  // indexed, so inflation overlaps packing, copies and compute (the whole-
  // input parallel producer inflates every file before batch 0).  A file
  // freed once its last record is packed.  Returns false if it does not
  // apply (nothing consumed: the caller's producers take the input); if a
  // later file is not strict 4-line FASTQ, the streaming producer takes over
  // at the next pair.
  bool produce_files() {
    namespace I = smash::ingest;
    const std::vector<std::string> *pl[2] = {&r1.paths, &r2.paths};
    bool any_gz = false;
    std::vector<uint64_t> fsz[2];
    for (int m = 0; m < 2; ++m)
      for (const auto &path : *pl[m]) {
        struct stat st;
        unsigned char mg[2] = {0, 0};
        const int fd = open(path.c_str(), O_RDONLY);
        if (fd < 0 || fstat(fd, &st) != 0) {
          if (fd >= 0) close(fd);
          return false;   // (the other producers report it)
        }
        if (st.st_size >= 2 && pread(fd, mg, 2, 0) == 2 && mg[0] == 0x1f && mg[1] == 0x8b)
          any_gz = true;
        close(fd);
        fsz[m].push_back(uint64_t(st.st_size));
      }
    if (!any_gz) return false;
    const auto t0 = Clock::now();
    struct F {
      std::unique_ptr<I::Source> s;
      std::vector<const char *> rec;
      int st = -1;   // -1 pending, 0 indexed, 1 not strict, 2 I/O error
      std::string why;
    };
    std::vector<F> files[2];
    files[0].resize(pl[0]->size());
    files[1].resize(pl[1]->size());
    // loading order: the lists interleaved by cumulative size
    std::vector<std::pair<int, size_t>> order;
    {
      size_t i[2] = {0, 0};
      uint64_t c[2] = {0, 0};
      while (i[0] < fsz[0].size() || i[1] < fsz[1].size()) {
        const int m = i[1] >= fsz[1].size() ? 0 : i[0] >= fsz[0].size() ? 1 : (c[0] <= c[1] ? 0 : 1);
        c[m] += fsz[m][i[m]];
        order.emplace_back(m, i[m]++);
      }
    }
    std::vector<size_t> pos_in_order[2];
    pos_in_order[0].resize(fsz[0].size());
    pos_in_order[1].resize(fsz[1].size());
    for (size_t j = 0; j < order.size(); ++j) pos_in_order[order[j].first][order[j].second] = j;
    std::mutex fm;
    std::condition_variable fcv;
    // jobs claimed; a loader claims job j only while j < need + ahead, need
    // = the latest loading position of the packer's current files (the
    // packer never waits for a file no loader may claim)
    size_t next_job = 0, need = 0;
    bool stop = false;
    const size_t ahead = std::max<size_t>(4, 2 * size_t(T));
    auto loader = [&] {
      for (;;) {
        size_t j;
        {
          std::unique_lock<std::mutex> g(fm);
          fcv.wait(g, [&] { return stop || next_job >= order.size() || next_job < need + ahead; });
          if (stop || next_job >= order.size()) return;
          j = next_job++;
        }
        F &f = files[order[j].first][order[j].second];
        auto src = std::make_unique<I::Source>();
        src->path = (*pl[order[j].first])[order[j].second];
        std::string why;
        int st = 0;
        std::vector<const char *> rec;
        if (!I::load_source(*src, why)) {
          st = 2;
        } else {
          const char *q = src->p, *e = src->p + src->n;
          rec.reserve(src->n / 256);
          while (q < e) {
            const char *end = I::strict_record(q, e);
            if (!end) {
              st = 1;
              break;
            }
            rec.push_back(q);
            q = end + 1;
          }
        }
        std::lock_guard<std::mutex> g(fm);
        f.s = std::move(src);
        f.rec.swap(rec);
        f.why = why;
        f.st = st;
        fcv.notify_all();
      }
    };
    std::vector<std::thread> pool;
    for (uint32_t t = 0; t < std::max<uint32_t>(1, T); ++t) pool.emplace_back(loader);
    auto shutdown = [&] {
      {
        std::lock_guard<std::mutex> g(fm);
        stop = true;
      }
      fcv.notify_all();
      for (auto &x : pool) x.join();
    };
    auto release = [&](int m, size_t i) {
      std::lock_guard<std::mutex> g(fm);
      files[m][i].s.reset();
      std::vector<const char *>().swap(files[m][i].rec);
    };
    // cursors: file, record within it
    size_t fi[2] = {0, 0}, ri[2] = {0, 0};
    std::vector<std::pair<int, size_t>> done_files;   // read past, records maybe still in a run
    bool ready[2] = {false, false};   // the cursor's file is loaded (its fields are final)
    auto set_need = [&] {
      size_t x = 0;
      for (int m = 0; m < 2; ++m)
        if (fi[m] < files[m].size()) x = std::max(x, pos_in_order[m][fi[m]]);
      std::lock_guard<std::mutex> g(fm);
      need = x;
      fcv.notify_all();
    };
    // the cursor's file with records left: 0 ok, 1 list ended, 2 not strict
    // (hand over), 3 I/O error
    auto avail = [&](int m) -> int {
      for (;;) {
        if (fi[m] >= files[m].size()) return 1;
        F &f = files[m][fi[m]];
        if (!ready[m]) {
          std::unique_lock<std::mutex> g(fm);
          fcv.wait(g, [&] { return f.st != -1; });
          ready[m] = true;
        }
        if (f.st == 1) return 2;
        if (f.st == 2) {
          fail(SMASH_ERR_IO, "smash_count_fastq: " + f.why);
          return 3;
        }
        if (ri[m] < f.rec.size()) return 0;
        done_files.emplace_back(m, fi[m]);   // freed once the run holding its records is packed
        ++fi[m];
        ri[m] = 0;
        ready[m] = false;
        set_need();
      }
    };
    auto release_done = [&] {
      for (auto &x : done_files) release(x.first, x.second);
      done_files.clear();
    };
    std::vector<uint8_t> keep;
    std::vector<uint64_t> dst;
    uint64_t emitted = 0;
    bool first = true;
    for (;;) {
      Slot &s = slot[next_slot++ % 3];
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return s.state == 0 || err; });
        if (err) {
          shutdown();
          return true;
        }
      }
      const auto t1 = Clock::now();
      uint64_t k = 0;   // pairs in the slot
      int why = 0;      // how the input ended: 0 not yet, 1 end, 2 not strict, 3 error
      while (k < B && !why) {
        // a run of pairs inside the two cursors' current files: record ri0 +
        // i of one, ri1 + i of the other
        const int x = avail(0);
        const int y = x ? 0 : avail(1);
        why = x ? x : y;
        if (why == 3) {
          shutdown();
          return true;
        }
        if (why == 2 && first && emitted == 0 && k == 0) {
          shutdown();   // nothing consumed: the other producers take it all
          --next_slot;  // (from this slot on)
          return false;
        }
        if (why) break;
        const F &f0 = files[0][fi[0]], &f1 = files[1][fi[1]];
        const uint64_t n = std::min<uint64_t>({B - k, f0.rec.size() - ri[0], f1.rec.size() - ri[1]});
        const char *const *pa = f0.rec.data() + ri[0];
        const char *const *pb = f1.rec.data() + ri[1];
        keep.resize(n);
        dst.resize(n);
        // checks (one empty mate, read length), drops, order; then convert
        std::atomic<int> bad{0};
        std::atomic<uint64_t> where{~0ull}, disorder{~0ull};
        par_for(n, T, [&](uint64_t lo, uint64_t hi) {
          for (uint64_t i = lo; i < hi; ++i) {
            const I::Rec x = I::parse(pa[i]), y = I::parse(pb[i]);
            keep[i] = !(x.sn == 0 && y.sn == 0);
            if (keep[i] && (x.sn == 0 || y.sn == 0 || x.sn != L || y.sn != L)) {
              uint64_t w = where.load();
              while (i < w && !where.compare_exchange_weak(w, i)) {
              }
              bad = 1;
            }
          }
        });
        if (bad) {
          const I::Rec x = I::parse(pa[where]), y = I::parse(pb[where]);
          const std::string na(x.name, x.nn);
          fail(SMASH_ERR_ARG, (x.sn == 0 || y.sn == 0)
                                  ? "smash_count_fastq: one mate of a pair has no bases (" + na + ")"
                                  : "smash_count_fastq: every mate must have the pipeline's read "
                                    "length (" + na + ")");
          shutdown();
          return true;
        }
        uint64_t kk = 0;
        for (uint64_t i = 0; i < n; ++i) dst[i] = keep[i] ? kk++ : ~0ull;
        par_for(n, T, [&](uint64_t lo, uint64_t hi) {
          const char *prev = nullptr;
          size_t pn = 0;
          for (uint64_t i = lo; i < hi; ++i) {
            if (!keep[i]) continue;
            const I::Rec x = I::parse(pa[i]), y = I::parse(pb[i]);
            if (!prev) {   // the kept pair before this range
              for (uint64_t j = i; j-- > 0;)
                if (keep[j]) {
                  const I::Rec z = I::parse(pa[j]);
                  prev = z.name;
                  pn = z.nn;
                  break;
                }
              if (!prev && have_prev) {
                prev = prev_name.data();
                pn = prev_name.size();
              }
            }
            if (prev && strnum_cmp(prev, pn, x.name, x.nn) > 0) {
              uint64_t w = disorder.load();
              while (i < w && !disorder.compare_exchange_weak(w, i)) {
              }
              break;
            }
            prev = x.name;
            pn = x.nn;
            uint8_t *d = s.h + (k + dst[i]) * 2 * S;
            I::convert(d, x.seq, L);
            I::convert(d + S, y.seq, L);
          }
        });
        if (disorder.load() != ~0ull) {
          const I::Rec x = I::parse(pa[disorder.load()]);
          fail(SMASH_ERR_ARG, "smash_count_fastq: pairs are not in samtools sort -n order at read " +
                                  std::string(x.name, x.nn) + " (use sort_names = 1)");
          shutdown();
          return true;
        }
        for (uint64_t i = n; i-- > 0;)
          if (keep[i]) {
            const I::Rec x = I::parse(pa[i]);
            prev_name.assign(x.name, x.nn);
            have_prev = true;
            break;
          }
        k += kk;
        ri[0] += n;
        ri[1] += n;
        release_done();   // the runs' records before this one are converted
      }
      const bool end = why != 0;
      {
        std::lock_guard<std::mutex> g(mu);
        ingest_s += secs(t1, Clock::now());
        if (first) index_s = secs(t0, Clock::now());
        parallel = true;
        s.n = k;
        s.last = end && why != 2;
        s.state = 1;
      }
      cv.notify_all();
      first = false;
      emitted += k;
      if (why == 2) {
        // a file that is not strict: the streaming producer takes over at
        // the next pair (each list from its current file, the records
        // before the cursor skipped: on the strict files before, both
        // readers see the same records)
        shutdown();
        for (int m = 0; m < 2; ++m) {
          Reader &rd = m ? r2 : r1;
          std::vector<std::string> rest(pl[m]->begin() + long(std::min(fi[m], pl[m]->size())),
                                        pl[m]->end());
          rd.paths.swap(rest);
          rd.next_path = 0;
          I::View nm, bs;
          int e = 0;
          for (size_t q = 0; q < ri[m]; ++q)
            if (!rd.record(nm, bs, e)) {
              fail(e ? e : SMASH_ERR_IO, "smash_count_fastq: " + rd.msg);
              return true;
            }
        }
        produce_stream();
        return true;
      }
      if (end) {
        shutdown();
        return true;
      }
    }
  }

  void produce(bool sort_names) {
    if (!sort_names && produce_files()) return;
    if (produce_parallel(sort_names)) return;
    if (sort_names) produce_sorted();
    else produce_stream();
  }

  // buffered producer: read all, order by name, stream batches
  void produce_sorted() {
    const uint8_t *lut = smash::ingest::lut();
    const auto t0 = Clock::now();
    std::vector<uint8_t> reads;        // [2 * pairs * L], converted
    std::vector<char> names;
    std::vector<uint64_t> noff(1, 0);
    std::vector<uint8_t> keep;
    for (;;) {
      uint64_t n = 0;
      bool end = false;
      if (!parse(B, n, end) || !check_pairs(n, keep)) return;
      for (uint64_t i = 0; i < n; ++i) {
        if (!keep[i]) continue;
        const size_t o = reads.size();
        reads.resize(o + 2 * L);
        const uint8_t *a = reinterpret_cast<const uint8_t *>(c1.bases.data() + c1.boff[i]);
        const uint8_t *bb = reinterpret_cast<const uint8_t *>(c2.bases.data() + c2.boff[i]);
        for (uint32_t j = 0; j < L; ++j) reads[o + j] = lut[a[j]];
        for (uint32_t j = 0; j < L; ++j) reads[o + L + j] = lut[bb[j]];
        names.insert(names.end(), c1.names.data() + c1.noff[i], c1.names.data() + c1.noff[i + 1]);
        noff.push_back(names.size());
      }
      if (end) break;
    }
    const uint64_t np = noff.size() - 1;
    std::vector<uint64_t> perm(np);
    std::iota(perm.begin(), perm.end(), uint64_t(0));
    std::stable_sort(perm.begin(), perm.end(), [&](uint64_t x, uint64_t y) {
      return strnum_cmp(names.data() + noff[x], noff[x + 1] - noff[x], names.data() + noff[y],
                        noff[y + 1] - noff[y]) < 0;
    });
    {
      std::lock_guard<std::mutex> g(mu);
      ingest_s += secs(t0, Clock::now());
    }
    for (uint64_t q0 = 0;;) {
      Slot &s = slot[next_slot++ % 3];
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return s.state == 0 || err; });
        if (err) return;
      }
      const auto t1 = Clock::now();
      const uint64_t k = std::min(B, np - q0);
      par_for(k, T, [&](uint64_t lo, uint64_t hi) {
        for (uint64_t i = lo; i < hi; ++i) {
          memcpy(s.h + i * 2 * S, reads.data() + perm[q0 + i] * 2 * L, L);
          memcpy(s.h + i * 2 * S + S, reads.data() + perm[q0 + i] * 2 * L + L, L);
        }
      });
      q0 += k;
      const bool end = q0 >= np;
      {
        std::lock_guard<std::mutex> g(mu);
        ingest_s += secs(t1, Clock::now());
        s.n = k;
        s.last = end;
        s.state = 1;
      }
      cv.notify_all();
      if (end) return;
    }
  }
};

}  // namespace

extern "C" int smash_count_fastq(smash_pipeline *p, const char *const *r1, uint32_t n1,
                                 const char *const *r2, uint32_t n2, int sort_names,
                                 uint32_t threads, uint64_t *d_counts, smash_feed_stats *st,
                                 void *stream) {
  if (!p || !r1 || !r2 || n1 == 0 || n2 == 0 || !d_counts) {
    smash::set_error("smash_count_fastq: bad arguments");
    return SMASH_ERR_ARG;
  }
  const auto t_start = Clock::now();
  auto f = std::make_unique<Feed>();
  f->p = p;
  f->L = smash::pipe_read_len(p);
  f->S = smash::pipe_stride(p);
  f->B = smash::pipe_max_pairs(p);
  // SMASH_FEED_BATCH: pairs per file-fed batch below the pipeline's
  // max_pairs (the device buffers are 2 x 2 B x stride bytes)
  if (const char *fb_env = std::getenv("SMASH_FEED_BATCH")) {
    const uint64_t b = std::strtoull(fb_env, nullptr, 10);
    if (b > 0 && b < f->B) f->B = b;
  }
  f->T = threads ? threads : 1;
  for (uint32_t i = 0; i < n1; ++i) f->r1.paths.emplace_back(r1[i]);
  for (uint32_t i = 0; i < n2; ++i) f->r2.paths.emplace_back(r2[i]);
  const uint64_t bytes = 2 * f->B * f->S;
  SMASH_HIP(hipSetDevice(smash::pipe_device(p)));
  hipStream_t cs = static_cast<hipStream_t>(stream);
  void *&fb_slot = smash::pipe_feed(p, free_feed);
  if (fb_slot && static_cast<FeedBufs *>(fb_slot)->bytes != bytes) {
    free_feed(fb_slot);
    fb_slot = nullptr;
  }
  if (!fb_slot) {
    auto *nb = new FeedBufs;
    if (!nb->alloc(bytes)) {
      delete nb;
      smash::set_error("smash_count_fastq: cannot allocate the batch buffers");
      return SMASH_ERR_NOMEM;
    }
    fb_slot = nb;
  }
  FeedBufs &fb = *static_cast<FeedBufs *>(fb_slot);
  hipStream_t xs = fb.xs;
  uint8_t **dbuf = fb.d;
  hipEvent_t *copied = fb.copied, *done = fb.done;
  for (int k = 0; k < 3; ++k) f->slot[k].h = fb.h[k];
  int rc = SMASH_OK;
  uint64_t pairs = 0, batches = 0;
  double wait_s = 0;
  std::thread prod;
  auto cleanup = [&] {
    if (prod.joinable()) {
      f->fail(f->err ? f->err : SMASH_ERR_IO, f->msg.empty() ? "stopped" : f->msg);
      prod.join();
    }
    if (xs) (void)hipStreamSynchronize(xs);
    if (cs) (void)hipStreamSynchronize(cs);
  };
  do {
    prod = std::thread([&] { f->produce(sort_names != 0); });
    for (uint64_t b = 0;; ++b) {
      Slot &s = f->slot[b % 3];
      const auto w0 = Clock::now();
      {
        std::unique_lock<std::mutex> g(f->mu);
        f->cv.wait(g, [&] { return s.state == 1 || f->err; });
        if (f->err) break;
      }
      wait_s += secs(w0, Clock::now());
      const int d = int(b & 1);
      if (s.n) {
        // the copy into dbuf[d] waits for the compute that last read it
        if (b >= 2 && hipStreamWaitEvent(xs, done[d], 0) != hipSuccess) { rc = SMASH_ERR_HIP; break; }
        if (hipMemcpyAsync(dbuf[d], s.h, 2 * s.n * f->S, hipMemcpyHostToDevice, xs) != hipSuccess ||
            hipEventRecord(copied[d], xs) != hipSuccess) {
          rc = SMASH_ERR_HIP;
          break;
        }
        // the key set grows (doubling) before a batch could overflow it: the
        // pairs of a gzip input are not counted before it is inflated
        if ((rc = smash::ensure_keys(p, s.n, cs)) != SMASH_OK) break;
        // the batch's search waits for its copy only (not for the previous
        // batch's post stage on cs): it can start under that batch's search
        if ((rc = smash::count_batch_ev(p, dbuf[d], s.n, d_counts, cs, copied[d])) != SMASH_OK)
          break;
        if (hipEventRecord(done[d], cs) != hipSuccess ||
            hipEventSynchronize(copied[d]) != hipSuccess) {   // the pinned slot is free again
          rc = SMASH_ERR_HIP;
          break;
        }
        pairs += s.n;
        ++batches;
      }
      const bool last = s.last;
      {
        std::lock_guard<std::mutex> g(f->mu);
        s.state = 0;
        s.n = 0;
      }
      f->cv.notify_all();
      if (last) break;
    }
    if (rc == SMASH_OK && hipStreamSynchronize(cs) != hipSuccess) rc = SMASH_ERR_HIP;
    if (prod.joinable()) prod.join();
    if (rc == SMASH_OK && f->err) {
      smash::set_error(f->msg);
      rc = f->err;
    }
  } while (false);
  if (rc == SMASH_ERR_HIP) smash::set_error("smash_count_fastq: HIP error");
  cleanup();
  if (st) {
    st->pairs = pairs;
    st->batches = batches;
    st->wall_s = secs(t_start, Clock::now());
    st->ingest_s = f->ingest_s;
    st->wait_s = wait_s;
    st->read_len = f->L;
    st->parallel = f->parallel ? 1u : 0u;
    st->index_s = f->index_s;
  }
  return rc;
}
