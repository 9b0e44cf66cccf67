// smash-paper_amd/csrc/index.hip -- device index lifecycle (smash_gpu.h).
//
// Replaces longSA::longSA (longSA.cpp:94-210) and Sequence::Sequence
// (fasta.cpp:133-285): the index is built on the device (sa_build.hip) or
// loaded from the reference's own cache files, and stays resident in HBM.
#include <sys/stat.h>

#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>

#include "common.hpp"

namespace smash {
// SMASH_IDX_BYTES=8: 8-byte SA/ISA even when N < 2^32 (tests the wide
// search path on small genomes; the reference would pick rc1.i4 there)
static bool force_wide_index() {
  const char *e = getenv("SMASH_IDX_BYTES");
  return e && e[0] == '8';
}

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }
}  // namespace smash

using namespace smash;

extern "C" const char *smash_last_error(void) { return g_err.c_str(); }

namespace {

double now_s() {
  return std::chrono::duration<double>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void free_index(smash_index *ix) {
  if (!ix) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(ix->device);
  dfree(ix->d_text); dfree(ix->d_sa); dfree(ix->d_isa); dfree(ix->d_lcp8);
  dfree(ix->d_ovf); dfree(ix->d_map); dfree(ix->d_startpos); dfree(ix->d_sizes);
  dfree(ix->d_uniq); dfree(ix->d_kmer); dfree(ix->d_bitmap); dfree(ix->d_work); dfree(ix->d_rec);
  dfree(ix->d_nsdir);
  smash::release_uniq_scratch(ix);   // (its scratch and second stream)
  (void)hipSetDevice(cur);
  delete ix;
}

void upload_tables(smash_index *ix, hipStream_t s) {
  if (!ix->d_work) {   // [0] work counter, [1..10] k_mam_sm's sticky probe check
    ix->d_work = dalloc<uint64_t>(16);
    SMASH_HIPX(hipMemsetAsync(ix->d_work, 0, 16 * 8, s));
  }
  ix->d_startpos = dalloc<uint64_t>(ix->n_seq);
  ix->d_sizes = dalloc<uint64_t>(ix->n_seq);
  SMASH_HIPX(hipMemcpyAsync(ix->d_startpos, ix->startpos.data(), 8 * ix->n_seq,
                            hipMemcpyHostToDevice, s));
  SMASH_HIPX(hipMemcpyAsync(ix->d_sizes, ix->sizes.data(), 8 * ix->n_seq,
                            hipMemcpyHostToDevice, s));
}

void account(smash_index *ix) {
  const uint64_t N = ix->N;
  ix->device_bytes = (N + 64) + 2 * N * ix->idx_bytes + (N + 64) + 16 * ix->n_ovf +
                     ix->map_bytes + 16 * ix->n_seq + (N + 64) +
                     (ix->kmer_k ? 16ull << (2 * ix->kmer_k) : 0) +
                     (ix->d_bitmap ? (1ull << (2 * ix->bitmap_b)) / 8 : 0);
}

// u32 exact LCP from lcp8 + overflow (used when map.bin must be computed
// for an index that was loaded from disk)
__global__ void k_lcp_expand(const uint8_t *l8, uint64_t N, uint32_t *lcp) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; r < N; r += stride)
    lcp[r] = l8[r];
}
__global__ void k_lcp_ovf(const uint64_t *ovf, uint64_t n, uint32_t *lcp) {
  const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t a = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; a < n; a += stride) {
    const uint64_t v = ovf[2 * a + 1];
    lcp[ovf[2 * a]] = v > 0xFFFFFFFFull ? 0xFFFFFFFFu : uint32_t(v);
  }
}

bool read_file(const std::string &path, std::vector<uint8_t> &buf) {
  FILE *f = fopen(path.c_str(), "rb");
  if (!f) return false;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  buf.resize(size_t(n));
  size_t got = n ? fread(buf.data(), 1, size_t(n), f) : 0;
  fclose(f);
  return got == size_t(n);
}

bool exists(const std::string &p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0;
}

uint64_t rd64(const uint8_t *&p) {
  uint64_t v;
  memcpy(&v, p, 8);
  p += 8;
  return v;
}

bool write_file(const std::string &path, const void *data, uint64_t n) {
  FILE *f = fopen(path.c_str(), "wb");
  if (!f) return false;
  bool ok = fwrite(data, 1, n, f) == n;
  return fclose(f) == 0 && ok;
}

}  // namespace

extern "C" int smash_index_create_layout(const uint8_t *h_text, uint64_t N,
                                         uint32_t n_seq, const uint64_t *h_startpos,
                                         const uint64_t *h_sizes,
                                         const char *const *names, int rcref, int device,
                                         smash_index **out) {
  if (!h_text || N < 2 || !h_startpos || !h_sizes || !out || n_seq == 0 ||
      (rcref && (n_seq & 1))) {
    set_error("smash_index_create: bad arguments");
    return SMASH_ERR_ARG;
  }
  if (h_text[N - 1] != '$') {
    set_error("smash_index_create: text must end with the '$' sentinel (fasta.cpp:247)");
    return SMASH_ERR_ARG;
  }
  std::unique_ptr<smash_index, void (*)(smash_index *)> ix(new smash_index, free_index);
  try {
    const double t0 = now_s();
    SMASH_HIPX(hipSetDevice(device));
    ix->device = device;
    ix->N = N;
    ix->logN = uint64_t(std::ceil(std::log(double(N)) / std::log(2.0)));
    ix->idx_bytes = (N <= 0xFFFFFFFFull && !force_wide_index()) ? 4 : 8;
    ix->n_seq = n_seq;
    ix->rcref = rcref != 0;
    ix->startpos.assign(h_startpos, h_startpos + n_seq);
    ix->sizes.assign(h_sizes, h_sizes + n_seq);
    if (names)
      for (uint32_t i = 0; i < n_seq; ++i) ix->names.emplace_back(names[i] ? names[i] : "");
    hipStream_t s;
    SMASH_HIPX(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ix->d_text = dalloc<uint8_t>(N + 64);
    SMASH_HIPX(hipMemsetAsync(ix->d_text + N, 0, 64, s));
    SMASH_HIPX(hipMemcpyAsync(ix->d_text, h_text, N, hipMemcpyHostToDevice, s));
    upload_tables(ix.get(), s);
    build_sa_isa(ix.get(), s);
    uint32_t *lcp = build_lcp32(ix.get(), s);
    finish_lcp(ix.get(), lcp, s);
    if (ix->rcref) build_map(ix.get(), lcp, s);   // -mappability requires -rcref (mummer.cpp:145)
    SMASH_HIPX(hipStreamSynchronize(s));
    dfree(lcp);
    build_aux(ix.get(), s);
    pack_index(ix.get(), true, s);   // (after every build step that reads SA / ISA)
    SMASH_HIPX(hipStreamSynchronize(s));
    SMASH_HIPX(hipStreamDestroy(s));
    ix->build_seconds = now_s() - t0;
    account(ix.get());
  } catch (hip_failure &f) {
    set_error(f.what);
    return f.what.find("hipMalloc") != std::string::npos ? SMASH_ERR_NOMEM
                                                         : SMASH_ERR_HIP;
  }
  *out = ix.release();
  return SMASH_OK;
}

extern "C" int smash_index_create(const uint8_t *h_text, uint64_t N, uint32_t n_seq,
                                  const uint64_t *h_startpos, const uint64_t *h_sizes,
                                  const char *const *names, int device, smash_index **out) {
  return smash_index_create_layout(h_text, N, n_seq, h_startpos, h_sizes, names, 1, device, out);
}

extern "C" int smash_index_load_layout(const char *fasta_path, int rcref, int device,
                                       smash_index **out) {
  if (!fasta_path || !out) {
    set_error("smash_index_load: bad arguments");
    return SMASH_ERR_ARG;
  }
  const std::string dir = std::string(fasta_path) + ".bin/";
  const std::string rc = rcref ? "rc1" : "rc0";   // fasta.cpp:98, longSA.cpp:103
  std::vector<uint8_t> refhdr, idxhdr;
  if (!read_file(dir + rc + ".ref.bin", refhdr) || refhdr.size() < 24) {
    set_error("cannot read " + dir + rc + ".ref.bin");
    return SMASH_ERR_IO;
  }
  std::unique_ptr<smash_index, void (*)(smash_index *)> ix(new smash_index, free_index);
  try {
    const double t0 = now_s();
    // rc1.ref.bin (fasta.cpp:265-277)
    const uint8_t *p = refhdr.data();
    const uint8_t *end = p + refhdr.size();
    (void)rd64(p);                           // fasta_size
    const uint64_t N = rd64(p);
    const uint64_t nd = rd64(p);
    for (uint64_t i = 0; i < nd; ++i) {
      if (p + 24 > end) throw hip_failure{"truncated " + rc + ".ref.bin"};
      ix->startpos.push_back(rd64(p));
      ix->sizes.push_back(rd64(p));
      const uint64_t L = rd64(p);
      if (p + L > end) throw hip_failure{"truncated " + rc + ".ref.bin"};
      ix->names.emplace_back(reinterpret_cast<const char *>(p), L);
      p += L;
    }
    ix->N = N;
    ix->n_seq = uint32_t(nd);
    ix->rcref = rcref != 0;
    if (!nd || (rcref && (nd & 1))) throw hip_failure{"bad contig table in " + rc + ".ref.bin"};
    ix->logN = uint64_t(std::ceil(std::log(double(N)) / std::log(2.0)));
    // index flavour: rc?.i4 or rc?.i8 (longSA.cpp:101-107)
    int W = 0;
    for (int w : {4, 8})
      if (!W && exists(dir + rc + ".i" + std::to_string(w) + ".index.bin")) W = w;
    if (!W) throw hip_failure{"no " + rc + ".i{4,8}.index.bin under " + dir};
    const std::string base = dir + rc + ".i" + std::to_string(W) + ".index";
    if (!read_file(base + ".bin", idxhdr) || idxhdr.size() < 48)
      throw hip_failure{"cannot read " + base + ".bin"};
    p = idxhdr.data();
    (void)rd64(p); (void)rd64(p); (void)rd64(p);   // fasta_size, logN, Nm1
    const uint64_t sa_size = rd64(p);
    const uint64_t n_vec = rd64(p);
    const uint64_t n_m = rd64(p);
    if (sa_size != N || n_vec != N) throw hip_failure{"index size mismatch"};
    SMASH_HIPX(hipSetDevice(device));
    ix->device = device;
    ix->idx_bytes = (N <= 0xFFFFFFFFull && !force_wide_index()) ? 4 : 8;
    hipStream_t s;
    SMASH_HIPX(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<uint8_t> buf;
    if (!read_file(dir + rc + ".ref.seq.bin", buf) || buf.size() != N)
      throw hip_failure{"cannot read " + rc + ".ref.seq.bin"};
    ix->d_text = dalloc<uint8_t>(N + 64);
    SMASH_HIPX(hipMemset(ix->d_text + N, 0, 64));
    SMASH_HIPX(hipMemcpy(ix->d_text, buf.data(), N, hipMemcpyHostToDevice));
    for (int which = 0; which < 2; ++which) {
      if (!read_file(base + (which ? ".isa.bin" : ".sa.bin"), buf) || buf.size() != N * W)
        throw hip_failure{"cannot read SA/ISA"};
      void *d = dalloc<uint8_t>(N * ix->idx_bytes);
      if (uint32_t(W) == ix->idx_bytes) {
        SMASH_HIPX(hipMemcpy(d, buf.data(), N * W, hipMemcpyHostToDevice));
      } else {  // i8 file with N < 2^32: narrow on the host
        std::vector<uint32_t> nar(N);
        const uint64_t *src = reinterpret_cast<const uint64_t *>(buf.data());
        for (uint64_t i = 0; i < N; ++i) nar[i] = uint32_t(src[i]);
        SMASH_HIPX(hipMemcpy(d, nar.data(), N * 4, hipMemcpyHostToDevice));
      }
      (which ? ix->d_isa : ix->d_sa) = d;
    }
    if (!read_file(base + ".lcp.vec.bin", buf) || buf.size() != N)
      throw hip_failure{"cannot read lcp.vec.bin"};
    ix->d_lcp8 = dalloc<uint8_t>(N + 64);   // zero pad: 16-byte probes at the last entry
    SMASH_HIPX(hipMemset(ix->d_lcp8 + N, 0, 64));
    SMASH_HIPX(hipMemcpy(ix->d_lcp8, buf.data(), N, hipMemcpyHostToDevice));
    if (!read_file(base + ".lcp.m.bin", buf) || buf.size() != n_m * 16)
      throw hip_failure{"cannot read lcp.m.bin"};
    {
      // item_t{size_t idx; ANINT val} (longSA.h:19-28): mask i4 padding
      std::vector<uint64_t> ovf(2 * (n_m ? n_m : 1));
      const uint64_t *src = reinterpret_cast<const uint64_t *>(buf.data());
      for (uint64_t a = 0; a < n_m; ++a) {
        ovf[2 * a] = src[2 * a];
        ovf[2 * a + 1] = W == 4 ? (src[2 * a + 1] & 0xFFFFFFFFull) : src[2 * a + 1];
      }
      ix->n_ovf = n_m;
      ix->d_ovf = dalloc<uint64_t>(ovf.size());
      SMASH_HIPX(hipMemcpy(ix->d_ovf, ovf.data(), 8 * ovf.size(), hipMemcpyHostToDevice));
    }
    upload_tables(ix.get(), s);
    uint64_t total = 0;
    for (uint32_t c = 0; c < ix->n_seq; c += 2) total += ix->sizes[c];
    if (!ix->rcref) {
      // no map.bin for the forward-only layout (-mappability requires -rcref)
    } else if (read_file(dir + "map.bin", buf) && buf.size() == 2 + 2 * total) {
      ix->map_bytes = buf.size();
      ix->d_map = dalloc<uint8_t>(buf.size());
      SMASH_HIPX(hipMemcpy(ix->d_map, buf.data(), buf.size(), hipMemcpyHostToDevice));
    } else {
      uint32_t *lcp = dalloc<uint32_t>(N);
      k_lcp_expand<<<grid_for(N, 256, 65536), 256, 0, s>>>(ix->d_lcp8, N, lcp);
      if (ix->n_ovf)
        k_lcp_ovf<<<grid_for(ix->n_ovf, 256, 65536), 256, 0, s>>>(ix->d_ovf, ix->n_ovf, lcp);
      build_map(ix.get(), lcp, s);
      SMASH_HIPX(hipStreamSynchronize(s));
      dfree(lcp);
    }
    SMASH_HIPX(hipStreamSynchronize(s));
    build_aux(ix.get(), s);
    pack_index(ix.get(), true, s);
    SMASH_HIPX(hipStreamSynchronize(s));
    SMASH_HIPX(hipStreamDestroy(s));
    ix->build_seconds = now_s() - t0;
    account(ix.get());
  } catch (hip_failure &f) {
    set_error(f.what);
    return f.what.find("hipMalloc") != std::string::npos ? SMASH_ERR_NOMEM : SMASH_ERR_IO;
  }
  *out = ix.release();
  return SMASH_OK;
}

extern "C" int smash_index_load(const char *fasta_path, int device, smash_index **out) {
  return smash_index_load_layout(fasta_path, 1, device, out);
}

extern "C" int smash_index_save(const smash_index *ix, const char *fasta_path,
                                uint64_t fasta_size) {
  if (!ix || !fasta_path) {
    set_error("smash_index_save: bad arguments");
    return SMASH_ERR_ARG;
  }
  try {
    SMASH_HIPX(hipSetDevice(ix->device));
    const std::string dir = std::string(fasta_path) + ".bin/";
    mkdir(dir.c_str(), 0777);
    const uint64_t N = ix->N;
    // flavour mummer would run for this fasta (mummer.cpp:156-183)
    const std::string rc = ix->rcref ? "rc1" : "rc0";
    const int W = (fasta_size * (ix->rcref ? 2 : 1) > 0xFFFFFFFFull - 100000) ? 8 : 4;
    if (W == 4 && ix->idx_bytes == 8) throw hip_failure{"index too large for " + rc + ".i4"};
    std::vector<uint8_t> hdr;
    auto put64 = [&](uint64_t v) {
      const uint8_t *b = reinterpret_cast<const uint8_t *>(&v);
      hdr.insert(hdr.end(), b, b + 8);
    };
    // rc1.ref.bin + rc1.ref.seq.bin (fasta.cpp:265-277)
    put64(fasta_size);
    put64(N);
    put64(ix->n_seq);
    uint64_t maxd = 0;
    for (uint32_t i = 0; i < ix->n_seq; ++i) {
      const std::string nm = i < ix->names.size() ? ix->names[i]
                                                   : ("seq" + std::to_string(ix->rcref ? i / 2 : i));
      put64(ix->startpos[i]);
      put64(ix->sizes[i]);
      put64(nm.size());
      hdr.insert(hdr.end(), nm.begin(), nm.end());
      maxd = std::max<uint64_t>(maxd, nm.size());
    }
    put64(maxd);
    if (!write_file(dir + rc + ".ref.bin", hdr.data(), hdr.size()))
      throw hip_failure{"write " + rc + ".ref.bin"};
    std::vector<uint8_t> buf(N);
    SMASH_HIPX(hipMemcpy(buf.data(), ix->d_text, N, hipMemcpyDeviceToHost));
    if (!write_file(dir + rc + ".ref.seq.bin", buf.data(), N)) throw hip_failure{"write seq"};
    const std::string base = dir + rc + ".i" + std::to_string(W) + ".index";
    // SA / ISA
    for (int which = 0; which < 2; ++which) {
      std::vector<uint8_t> a(N * ix->idx_bytes);
      SMASH_HIPX(hipMemcpy(a.data(), which ? ix->d_isa : ix->d_sa, a.size(), hipMemcpyDeviceToHost));
      if (ix->idx_bytes == 8 && ix->pos_mask != ~0ull) {   // the reference's plain elements
        uint64_t *w = reinterpret_cast<uint64_t *>(a.data());
        for (uint64_t i = 0; i < N; ++i) w[i] &= ix->pos_mask;
      }
      if (uint32_t(W) != ix->idx_bytes) {  // widen u32 -> u64
        std::vector<uint64_t> w(N);
        const uint32_t *src = reinterpret_cast<const uint32_t *>(a.data());
        for (uint64_t i = 0; i < N; ++i) w[i] = src[i];
        if (!write_file(base + (which ? ".isa.bin" : ".sa.bin"), w.data(), 8 * N)) throw hip_failure{"write"};
      } else if (!write_file(base + (which ? ".isa.bin" : ".sa.bin"), a.data(), a.size())) {
        throw hip_failure{"write"};
      }
    }
    SMASH_HIPX(hipMemcpy(buf.data(), ix->d_lcp8, N, hipMemcpyDeviceToHost));
    if (!write_file(base + ".lcp.vec.bin", buf.data(), N)) throw hip_failure{"write lcp.vec"};
    std::vector<uint64_t> ovf(2 * (ix->n_ovf ? ix->n_ovf : 1));
    if (ix->n_ovf)
      SMASH_HIPX(hipMemcpy(ovf.data(), ix->d_ovf, 16 * ix->n_ovf, hipMemcpyDeviceToHost));
    if (!write_file(base + ".lcp.m.bin", ovf.data(), 16 * ix->n_ovf)) throw hip_failure{"write lcp.m"};
    hdr.clear();
    put64(fasta_size);
    put64(ix->logN);
    put64(N - 1);
    put64(N);
    put64(N);
    put64(ix->n_ovf);
    if (!write_file(base + ".bin", hdr.data(), hdr.size())) throw hip_failure{"write index.bin"};
    if (ix->d_map) {
      std::vector<uint8_t> m(ix->map_bytes);
      SMASH_HIPX(hipMemcpy(m.data(), ix->d_map, m.size(), hipMemcpyDeviceToHost));
      if (!write_file(dir + "map.bin", m.data(), m.size())) throw hip_failure{"write map.bin"};
    }
  } catch (hip_failure &f) {
    set_error(f.what);
    return SMASH_ERR_IO;
  }
  return SMASH_OK;
}

extern "C" void smash_index_free(smash_index *ix) { free_index(ix); }

extern "C" int smash_index_query(const smash_index *ix, smash_index_info *o) {
  if (!ix || !o) {
    set_error("smash_index_query: bad arguments");
    return SMASH_ERR_ARG;
  }
  o->N = ix->N;
  o->logN = ix->logN;
  o->idx_bytes = ix->idx_bytes;
  o->n_seq = ix->n_seq;
  o->rcref = ix->rcref ? 1 : 0;
  o->pos_bits = ix->pos_mask == kPkPosMask ? kPkPosBits : 0;
  o->n_lcp_overflow = ix->n_ovf;
  o->map_bytes = ix->map_bytes;
  o->d_text = ix->d_text;
  o->d_sa = ix->d_sa;
  o->d_isa = ix->d_isa;
  o->d_lcp8 = ix->d_lcp8;
  o->d_lcp_ovf = ix->d_ovf;
  o->d_map = ix->d_map;
  o->device_bytes = ix->device_bytes;
  o->build_seconds = ix->build_seconds;
  o->kmer_k = ix->kmer_k;
  o->d_uniq = ix->d_uniq;
  o->d_kmer = ix->d_kmer;
  o->bitmap_b = ix->bitmap_b;
  o->d_bitmap = ix->d_bitmap;
  for (int k = 0; k < 4; ++k) o->in_text[k] = ix->in_text[k];
  return SMASH_OK;
}
