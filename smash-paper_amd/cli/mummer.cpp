// smash-paper_amd/cli/mummer.cpp -- the reference's `mummer` (memsam) command
// line over libsmashgpu's C ABI: the same flags (mummer.cpp:77-150), the same
// inputs and the same outputs, with the index, the search and the per-match
// records on the MI355X.
//
//   mummer [options] REF.fa QUERY...
//     index   REF.fa.bin/ cache loaded (smash_index_load) or, when absent,
//             built on the device and saved (longSA.cpp:94-210)
//     -mappability  REF.fa OUT: map.bin to OUT (longSA::show_mappability,
//             index_setup.sh:22)
//     queries SAM (-samin), FASTQ (-fastq) or FASTA records (QueryReader::run,
//             query.cpp:614-687), mates alternating read 1 / read 2 (Pair::run,
//             query.cpp:481-516); search MAM (default, -mumreference,
//             -mumcand), MUM (-mum) or MEM (-maxmatch), -l min length, -n
//     -samout the mapout SAM lines (query.cpp:331-403) into mapout/, one file
//             per batch with the fasta.cpp:243-252 header, lines in MemSam
//             order (memsam.h:136-158); without -samout the reference writes
//             header-only files (query.cpp:404-412 never ends a line) and so
//             does this
//   -qthreads, -verbose, -cached, -normalmem, -minblock are accepted; query
//   parallelism is the device's.  Errors: "Error" + the message on stderr,
//   exit status 1 (mummer.cpp:55-66).
#include <getopt.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/smash_gpu.h"

namespace {

struct Fail : std::runtime_error {
  using std::runtime_error::runtime_error;
};
// raised where the reference's worker thread throws (memsam.h:148-150,
// MemSam::chromosomes.at): Pair::runner_thread prints e.what() alone and
// exits 1 (query.cpp:522-535), without main's "Error" line
struct ThreadFail : Fail {
  using Fail::Fail;
};

void ck(int rc, const char *what) {
  if (rc != SMASH_OK) throw Fail(std::string(what) + ": " + smash_last_error());
}
void hk(hipError_t e, const char *what) {
  if (e != hipSuccess) throw Fail(std::string(what) + ": " + hipGetErrorString(e));
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Args {
  uint32_t min_len = 20;
  int type = SMASH_MODE_MAM;
  bool nucleotides_only = false, sam_out = false, verbose = false, nomap = false;
  bool rcref = false, fastq = false, sam_in = false, mappability = false;
  int qthreads = 2;
  std::string ref;
  std::vector<std::string> input;
};

[[noreturn]] void usage(const char *prog) {
  std::fprintf(stderr,
               "Usage: %s [options] <reference-file> <query-file> ...\n"
               "Implemented MUMmer v3 options:\n"
               "-mum           compute maximal matches that are unique in both sequences\n"
               "-mumreference  compute maximal matches that are unique in the reference-\n"
               "               sequence but not necessarily in the query-sequence (default)\n"
               "-mumcand       same as -mumreference\n"
               "-maxmatch      compute all maximal matches regardless of their uniqueness\n"
               "-l             set the minimum length of a match\n"
               "               if not set, the default value is 20\n"
               "-n             match only the characters a, c, g, or t\n"
               "\n"
               "Additional options:\n"
               "-verbose       output diagnostics and progress to stderr\n"
               "-samin         input in SAM format\n"
               "-samout        output in basic SAM format\n"
               "-qthreads      number of threads to use for queries (the device runs them)\n"
               "-nomap         output unmapped reads too (only when -samout)\n"
               "-rcref         reverse complement reference\n"
               "-fastq         fastq input\n"
               "-mappability   output mappability measures only\n"
               "-minblock      accepted, unused (as in the reference)\n"
               "-cached        accepted (no effect: the index is resident in HBM)\n"
               "-normalmem     accepted (no effect)\n",
               prog);
  std::exit(1);
}

// mummer.cpp:73-153
Args parse(int argc, char **argv) {
  static option opts[] = {{"l", 1, nullptr, 0},         {"mumreference", 0, nullptr, 0},
                          {"maxmatch", 0, nullptr, 0},  {"mum", 0, nullptr, 0},
                          {"mumcand", 0, nullptr, 0},   {"n", 0, nullptr, 0},
                          {"qthreads", 1, nullptr, 0},  {"samout", 0, nullptr, 0},
                          {"verbose", 0, nullptr, 0},   {"nomap", 0, nullptr, 0},
                          {"rcref", 0, nullptr, 0},     {"fastq", 0, nullptr, 0},
                          {"samin", 0, nullptr, 0},     {"mappability", 0, nullptr, 0},
                          {"cached", 0, nullptr, 0},    {"normalmem", 0, nullptr, 0},
                          {"minblock", 1, nullptr, 0},  {nullptr, 0, nullptr, 0}};
  Args a;
  for (;;) {
    int li = -1;
    const int c = getopt_long_only(argc, argv, "", opts, &li);
    if (c == -1) break;
    if (c == '?') {
      std::fprintf(stderr, "Invalid arguments.\n");
      usage(argv[0]);
    }
    switch (li) {
      case 0: a.min_len = uint32_t(std::atol(optarg)); break;
      case 1: case 4: a.type = SMASH_MODE_MAM; break;
      case 2: a.type = SMASH_MODE_MEM; break;
      case 3: a.type = SMASH_MODE_MUM; break;
      case 5: a.nucleotides_only = true; break;
      case 6: a.qthreads = std::atoi(optarg); break;
      case 7: a.sam_out = true; break;
      case 8: a.verbose = true; break;
      case 9: a.nomap = true; break;
      case 10: a.rcref = true; break;
      case 11: a.fastq = true; break;
      case 12: a.sam_in = true; break;
      case 13: a.mappability = true; break;
      default: break;   // -cached, -normalmem, -minblock
    }
  }
  const int left = argc - optind;
  if (left < 2) {
    std::fprintf(stderr, "There are too few arguments\n");
    usage(argv[0]);
  }
  if (a.fastq && a.sam_in) throw Fail("-fastq cannot be used with -samin");
  if (a.nomap && !a.sam_out) throw Fail("-nomap can only be used with -sam_out");
  if (a.mappability && !a.rcref) throw Fail("-mappability requires -rcref");
  a.ref = argv[optind];
  for (int i = optind + 1; i < argc; ++i) a.input.emplace_back(argv[i]);
  return a;
}

bool exists(const std::string &p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0;
}

// ---- the index: REF.fa.bin/ cache or a device build + save ------------------
struct Index {
  smash_index *h = nullptr;
  std::vector<std::string> names;   // 2 per contig with -rcref, else 1
  std::vector<uint64_t> sizes;
  bool rcref = true;
  ~Index() {
    if (h) smash_index_free(h);
  }
};

void load_or_build(const Args &a, Index &ix) {
  const std::string dir = a.ref + ".bin/";
  const std::string rc = a.rcref ? "rc1" : "rc0";   // fasta.cpp:98, longSA.cpp:103
  ix.rcref = a.rcref;
  const double t0 = now_s();
  if (exists(dir + rc + ".i4.index.bin") || exists(dir + rc + ".i8.index.bin")) {
    if (a.verbose) std::fprintf(stderr, "# loading index binary\n");
    ck(smash_index_load_layout(a.ref.c_str(), a.rcref ? 1 : 0, 0, &ix.h), "smash_index_load");
    // names and sizes from rc?.ref.bin (fasta.cpp:221-233)
    std::ifstream f(dir + rc + ".ref.bin", std::ios::binary);
    auto rd = [&]() {
      uint64_t v = 0;
      f.read(reinterpret_cast<char *>(&v), 8);
      return v;
    };
    rd();
    rd();
    const uint64_t n = rd();
    for (uint64_t i = 0; i < n; ++i) {
      rd();
      ix.sizes.push_back(rd());
      const uint64_t L = rd();
      std::string s(L, '\0');
      f.read(&s[0], std::streamsize(L));
      ix.names.push_back(s);
    }
    if (!f) throw Fail("cannot read " + dir + rc + ".ref.bin");
  } else {
    if (!exists(a.ref)) throw Fail("reference file not found: " + a.ref);
    if (a.verbose) std::fprintf(stderr, "# building the index on the device\n");
    uint8_t *text = nullptr;
    uint64_t N = 0, *sp = nullptr, *sz = nullptr;
    uint32_t ns = 0;
    char **nm = nullptr;
    ck(smash_text_from_fasta_layout(a.ref.c_str(), a.rcref ? 1 : 0, &text, &N, &ns, &sp, &sz,
                                    &nm),
       "smash_text_from_fasta");
    for (uint32_t i = 0; i < ns; ++i) {
      ix.names.emplace_back(nm[i]);
      ix.sizes.push_back(sz[i]);
    }
    const int rcode = smash_index_create_layout(text, N, ns, sp, sz, nm, a.rcref ? 1 : 0, 0, &ix.h);
    smash_text_free(text, ns, sp, sz, nm);
    ck(rcode, "smash_index_create");
    struct stat st;
    stat(a.ref.c_str(), &st);
    ck(smash_index_save(ix.h, a.ref.c_str(), uint64_t(st.st_size)), "smash_index_save");
  }
  if (a.verbose)
    std::fprintf(stderr, "# constructed index in %.0f seconds\n", now_s() - t0);
}

// ---- queries (QueryReader::run, query.cpp:614-687) --------------------------
struct Query {
  std::string name, seq, qual, opt;   // qual empty: '!' per base (Aligner::run)
};

// NewQuery::extend (query.cpp:125-144): trailing spaces cut, spaces dropped
std::string extend(const std::string &line) {
  size_t end = line.size();
  while (end && line[end - 1] == ' ') --end;
  std::string o;
  o.reserve(end);
  for (size_t i = 0; i < end; ++i)
    if (line[i] != ' ') o.push_back(line[i]);
  return o;
}

class Reader {
 public:
  Reader(const std::string &path, const Args &a) : a_(a), in_(path) {
    if (!in_) throw Fail("unable to open " + path);
  }
  // false at the end of the input
  bool next(Query &q) {
    std::string line;
    while (std::getline(in_, line)) {
      if (line.empty()) continue;
      q = Query();
      if (a_.sam_in) {
        if (line[0] == '@') continue;   // header lines (fastqs_to_sam writes none)
        std::istringstream in(line);
        std::string ref, pos, mapq, cigar, mref, mpos, tlen, o;
        unsigned flag = 0;
        in >> q.name >> flag >> ref >> pos >> mapq >> cigar >> mref >> mpos >> tlen >> q.seq >>
            q.qual;
        if (flag & 64u) q.name += ":0";
        else if (flag & 128u) q.name += ":1";
        q.seq = extend(q.seq);
        while (in >> o) q.opt += "\t" + o;
        if (q.qual.empty()) throw Fail("empty errors");
        return true;
      }
      const char start = a_.fastq ? '@' : '>';
      if (line[0] != start)
        throw Fail(std::string("missing query start character ") + start + "in input line" + line);
      size_t b = 1, e = line.size();   // trim (util.h)
      while (b < e && line[b] == ' ') ++b;
      while (e > b && line[e - 1] == ' ') --e;
      for (size_t i = b; i < e; ++i) {
        if (line[i] == ' ') {   // illumina mate info after the name
          if (i + 1 != e) {
            if (line[i + 1] == '1') q.name += ":0";
            else if (line[i + 1] == '2') q.name += ":1";
          }
          break;
        }
        q.name += line[i];
      }
      if (!std::getline(in_, line) || line.empty()) throw Fail("empty sequence");
      q.seq = extend(line);
      if (a_.fastq) {
        std::getline(in_, line);
        std::getline(in_, line);
        if (line.empty()) throw Fail("empty errors");
        q.qual = line;
      }
      return true;
    }
    return false;
  }

 private:
  const Args &a_;
  std::ifstream in_;
};

// ---- output: OutputSorter (query.cpp:448-468) + MemSam order ----------------
struct Sorter {
  std::map<std::string, uint64_t> chrom;   // Pairs::Pairs (query.cpp:546-552)
  std::string header;
  std::string tag;
  int seq = 0;
  explicit Sorter(const Index &ix) {
    // the absolute-position map steps over descr by 2 with or without
    // -rcref (query.cpp:547-551): without it every second contig is missing
    // and a line on one of them ends the run with "map::at", as it does there
    uint64_t off = 0;
    for (size_t i = 0; i < ix.names.size(); i += 2) {
      chrom[ix.names[i]] = off;
      off += ix.sizes[i];
    }
    chrom["*"] = off;
    header = "@HD\tVN:1.0\tSO:unsorted\n";   // Sequence::sam_header (fasta.cpp:243-252)
    for (size_t i = 0; i < ix.names.size(); i += ix.rcref ? 2 : 1)
      header += "@SQ\tSN:" + ix.names[i] + "\tLN:" + std::to_string(ix.sizes[i]) + "\n";
    header += "@PG\tID:longMEM\tPN:longMEM\tVN:0.5\n";
    tag = std::to_string(uint64_t(getpid()));
  }
  static const char *field(const char *l, int k) {
    while (k--) l = std::strchr(l, '\t') + 1;
    return l;
  }
  struct Key {
    uint64_t abspos;
    std::string name;
    unsigned mate;
    const char *line;
    size_t len;
  };
  // one file per call: the header, then the lines in MemSam order
  void flush(const char *text, uint64_t n) {
    mkdir("mapout", 0777);
    std::vector<Key> keys;
    const char *p = text, *end = text + n;
    while (p < end) {
      const char *nl = static_cast<const char *>(std::memchr(p, '\n', size_t(end - p)));
      const size_t len = size_t((nl ? nl + 1 : end) - p);
      Key k;
      k.line = p;
      k.len = len;
      const char *f1 = field(p, 1), *f2 = field(p, 2), *f3 = field(p, 3);
      k.name.assign(p, size_t(f1 - 1 - p));
      const unsigned flag = unsigned(std::atoi(f1));
      k.mate = flag & (64u | 128u | 16u);
      const auto c = chrom.find(std::string(f2, size_t(f3 - 1 - f2)));
      if (c == chrom.end()) throw ThreadFail("map::at");   // MemSam::chromosomes.at
      k.abspos = uint64_t(std::atol(f3)) + c->second;
      keys.push_back(std::move(k));
      p += len;
    }
    std::sort(keys.begin(), keys.end(), [](const Key &a, const Key &b) {
      if (a.abspos != b.abspos) return a.abspos < b.abspos;
      if (a.name != b.name) return a.name < b.name;
      if (a.mate == b.mate) throw ThreadFail("flags equal");   // memsam.h:148-150
      return a.mate < b.mate;
    });
    const std::string path = "mapout/mapout" + tag + "." + std::to_string(++seq) + ".txt";
    FILE *o = std::fopen(path.c_str(), "wb");
    if (!o) throw Fail("Problem opening out file");
    std::fputs(header.c_str(), o);
    for (const Key &k : keys) std::fwrite(k.line, 1, k.len, o);
    std::fclose(o);
  }
};

// ---- one batch: search + records on the device, lines on the host ----------
struct Device {
  uint8_t *reads = nullptr;
  uint16_t *lens = nullptr;
  uint64_t *match = nullptr;
  smash_match *mrec = nullptr;
  uint32_t *n = nullptr;
  smash_sam_rec *rec = nullptr;
  uint64_t *off = nullptr;
  size_t reads_cap = 0, lens_cap = 0, match_cap = 0, mrec_cap = 0, n_cap = 0, rec_cap = 0,
         off_cap = 0;
  template <class T>
  static void grow(T *&p, size_t &cap, size_t want) {
    if (want <= cap) return;
    if (p) (void)hipFree(p);
    p = nullptr;
    hk(hipMalloc(reinterpret_cast<void **>(&p), want * sizeof(T)), "hipMalloc");
    cap = want;
  }
  ~Device() {
    for (void *p : {(void *)reads, (void *)lens, (void *)match, (void *)mrec, (void *)n,
                    (void *)rec, (void *)off})
      if (p) (void)hipFree(p);
  }
};

void run_batch(const Args &a, const Index &ix, Device &d, Sorter &out,
               const std::vector<Query> &qs, const std::vector<const char *> &contigs) {
  const uint64_t n = qs.size();
  if (!n) return;
  uint32_t L = uint32_t(qs[0].seq.size());
  bool fixed = true;
  for (const Query &q : qs) {
    if (q.seq.empty()) throw Fail("empty sequence");
    if (q.seq.size() > 255)
      throw Fail("query " + q.name + " longer than 255 bases (device batches hold <= 255)");
    fixed = fixed && q.seq.size() == L;
  }
  const uint64_t stride = fixed ? L : 256;
  std::vector<uint8_t> h(n * stride, 0);
  std::vector<uint16_t> hl(n);
  for (uint64_t i = 0; i < n; ++i) {
    const std::string &s = qs[i].seq;
    hl[i] = uint16_t(s.size());
    for (size_t j = 0; j < s.size(); ++j) {
      char c = char(std::tolower(static_cast<unsigned char>(s[j])));   // NewQuery::extend
      if (a.nucleotides_only && c != 'a' && c != 'c' && c != 'g' && c != 't') c = '~';
      h[i * stride + j] = uint8_t(c);
    }
  }
  Device::grow(d.reads, d.reads_cap, h.size());
  hk(hipMemcpy(d.reads, h.data(), h.size(), hipMemcpyHostToDevice), "hipMemcpy");
  const uint16_t *dl = nullptr;
  if (!fixed) {
    Device::grow(d.lens, d.lens_cap, n);
    hk(hipMemcpy(d.lens, hl.data(), 2 * n, hipMemcpyHostToDevice), "hipMemcpy");
    dl = d.lens;
    L = 255;
  }
  Device::grow(d.n, d.n_cap, n);
  uint32_t cap = (fixed ? L : 255) >= a.min_len ? (fixed ? L : 255) - a.min_len + 1 : 1;
  if (a.type == SMASH_MODE_MEM) {
    // every MEM occurrence is a record: grow the per-read capacity to the
    // largest count, then pack into the u64 match words (reads <= 255 bp)
    std::vector<uint32_t> cnt(n);
    for (;;) {
      Device::grow(d.mrec, d.mrec_cap, n * cap);
      ck(smash_match_batch(ix.h, SMASH_MODE_MEM, a.min_len, d.reads, stride, dl, fixed ? L : 0,
                           n, d.mrec, cap, d.n, nullptr),
         "smash_match_batch");
      hk(hipMemcpy(cnt.data(), d.n, 4 * n, hipMemcpyDeviceToHost), "hipMemcpy");
      const uint32_t mx = *std::max_element(cnt.begin(), cnt.end());
      if (mx <= cap) break;
      cap = mx;
    }
    std::vector<smash_match> m(n * cap);
    hk(hipMemcpy(m.data(), d.mrec, m.size() * sizeof(smash_match), hipMemcpyDeviceToHost),
       "hipMemcpy");
    std::vector<uint64_t> w(n * cap, 0);
    for (uint64_t i = 0; i < n; ++i)
      for (uint32_t k = 0; k < cnt[i]; ++k) {
        const smash_match &x = m[i * cap + k];
        w[i * cap + k] = (x.ref & 0xFFFFFFFFFFFFull) | (uint64_t(x.query & 0xFF) << 48) |
                         (uint64_t(x.len & 0xFF) << 56);
      }
    Device::grow(d.match, d.match_cap, w.size());
    hk(hipMemcpy(d.match, w.data(), 8 * w.size(), hipMemcpyHostToDevice), "hipMemcpy");
  } else {
    Device::grow(d.match, d.match_cap, n * cap);
    ck(smash_map_batch(ix.h, a.type, a.min_len, d.reads, stride, dl, fixed ? L : 0, n, d.match,
                       cap, d.n, nullptr),
       "smash_map_batch");
  }
  // records packed read after read (smash_sam_records_packed): the table is
  // as large as the matches found, not n * cap
  std::vector<uint32_t> cnt(n);
  hk(hipMemcpy(cnt.data(), d.n, 4 * n, hipMemcpyDeviceToHost), "hipMemcpy");
  std::vector<uint64_t> off(n);
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (cnt[i] > cap) throw Fail("a query has more matches than the record cap");
    off[i] = total;
    total += cnt[i];
  }
  Device::grow(d.off, d.off_cap, n);
  hk(hipMemcpy(d.off, off.data(), 8 * n, hipMemcpyHostToDevice), "hipMemcpy");
  Device::grow(d.rec, d.rec_cap, total ? total : 1);
  ck(smash_sam_records_packed(ix.h, d.reads, stride, dl, fixed ? L : 0, n, d.match, cap, d.n,
                              d.off, nullptr, d.rec, nullptr),
     "smash_sam_records_packed");
  hk(hipDeviceSynchronize(), "hipDeviceSynchronize");
  if (!a.sam_out) return;   // query.cpp:404-412: the non-SAM lines are never ended
  std::vector<smash_sam_rec> rec(total);
  hk(hipMemcpy(rec.data(), d.rec, total * sizeof(smash_sam_rec), hipMemcpyDeviceToHost),
     "hipMemcpy");
  std::vector<const char *> names(n), seqs(n), quals(n), opts(n);
  for (uint64_t i = 0; i < n; ++i) {
    names[i] = qs[i].name.c_str();
    seqs[i] = qs[i].seq.c_str();
    quals[i] = qs[i].qual.empty() ? nullptr : qs[i].qual.c_str();
    opts[i] = qs[i].opt.c_str();
  }
  char *text = nullptr;
  uint64_t len = 0;
  int32_t terr = 0;
  ck(smash_sam_format(contigs.data(), uint32_t(contigs.size()), rec.data(), cnt.data(),
                      SMASH_SAM_PACKED | cap, n,
                      names.data(), seqs.data(), quals.data(), opts.data(), a.nomap ? 1 : 0, 0,
                      nullptr, &text, &len, &terr),
     "smash_sam_format");
  try {
    out.flush(text, len);
  } catch (...) {
    smash_sam_free(text);
    throw;
  }
  smash_sam_free(text);
}

int run(int argc, char **argv) {
  const Args a = parse(argc, argv);
  Index ix;
  load_or_build(a, ix);
  if (a.mappability) {   // longSA::show_mappability -> input[0] (mummer.cpp:48-51)
    smash_index_info info;
    ck(smash_index_query(ix.h, &info), "smash_index_query");
    std::vector<uint8_t> m(info.map_bytes);
    hk(hipMemcpy(m.data(), info.d_map, m.size(), hipMemcpyDeviceToHost), "hipMemcpy");
    FILE *o = std::fopen(a.input[0].c_str(), "wb");
    if (!o || std::fwrite(m.data(), 1, m.size(), o) != m.size())
      throw Fail("Problem writing mappability file " + a.input[0]);
    std::fclose(o);
    return 0;
  }
  std::vector<const char *> contigs;   // per record tid (k_sam_recs)
  for (size_t i = 0; i < ix.names.size(); i += a.rcref ? 2 : 1)
    contigs.push_back(ix.names[i].c_str());
  Sorter out(ix);
  Device d;
  const size_t batch = 1u << 18;   // reads per device batch (even: mates stay together)
  uint64_t total = 0;
  const double t0 = now_s();
  for (const std::string &path : a.input) {
    Reader r(path, a);
    std::vector<Query> qs;
    Query q;
    uint64_t n_path = 0;
    while (r.next(q)) {
      qs.push_back(std::move(q));
      ++n_path;
      if (qs.size() == batch) {
        run_batch(a, ix, d, out, qs, contigs);
        qs.clear();
      }
    }
    run_batch(a, ix, d, out, qs, contigs);
    if (!a.sam_out && !n_path) {}
    if (a.verbose)
      std::fprintf(stderr, "# query reader for %s processed %llu sequences\n", path.c_str(),
                   (unsigned long long)n_path);
    if (!n_path) std::fprintf(stderr, "# no reads processed\n");
    total += n_path;
  }
  if (!a.sam_out) out.flush("", 0);   // the header-only file of the non-SAM mode
  if (a.verbose)
    std::fprintf(stderr, "# ran %llu queries in %.1f seconds\n", (unsigned long long)total,
                 now_s() - t0);
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  try {
    return run(argc, argv);
  } catch (ThreadFail &e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  } catch (std::exception &e) {
    std::fprintf(stderr, "Error\n%s\n", e.what());
    return 1;
  }
}
