// tools/readgen.hip -- synthetic SMASH read pairs generated ON THE DEVICE from
// the resident doubled text (test / benchmark data, not part of the product).
//
// Same model as tools/synth.py make_reads: each mate is a
// concatenation of segments of uniform length [20, 60] from independent
// loci (intervals of non-N sequence >= 500 bp from N runs and contig ends,
// weighted by length, chrM and '_' contigs excluded) on a random strand;
// 1% uniform substitutions; 0.5% of mates carry one N; 1% of pairs are exact
// copies of an earlier pair.  Reads come out already prepared as the
// pipeline consumes them (lowercase, N -> 'z': fastqs_to_sam replaceN +
// NewQuery::extend).  Counter-based hashing of (seed, pair, mate, segment)
// makes every pair independent of the batch split: pair q is the same bytes
// whether generated alone or in a batch of 25 M.
#include <hip/hip_runtime.h>
#include <zlib.h>

#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

namespace {

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t h4(uint64_t s, uint64_t a, uint64_t b, uint64_t c) {
  return mix(mix(mix(s ^ a) ^ (b * 0xD6E8FEB86659FD93ull)) ^ (c * 0xA0761D6478BD642Full));
}
__device__ __forceinline__ double unit(uint64_t h) { return double(h >> 11) * 0x1.0p-53; }

struct Iv {
  uint64_t a, b;        // forward contig coordinates [a, b)
  uint64_t fwd_base;    // text position of forward base 0 of the contig
  uint64_t rc_end;      // text position of the rc copy + contig size
};

__global__ void k_gen(const uint8_t *__restrict__ text, const Iv *__restrict__ iv,
                      const uint64_t *__restrict__ cum, uint32_t n_iv, uint64_t total,
                      uint64_t seed, uint64_t q0, uint64_t n_pairs, uint32_t L,
                      uint8_t *__restrict__ out) {
  const uint64_t t = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= 2 * n_pairs) return;
  const uint64_t q = q0 + t / 2, mate = t & 1;
  uint64_t src = q;   // 1% exact duplicates of an earlier pair
  if (q > 0 && unit(h4(seed, q, 0xD0, 0)) < 0.01) src = h4(seed, q, 0xD1, 0) % q;
  uint8_t *o = out + t * L;
  uint32_t pos = 0;
  for (uint32_t k = 0; pos < L; ++k) {
    const uint64_t hs = h4(seed, src, mate, 4 * k);
    const uint32_t seglen = 20 + uint32_t(hs % 41);
    const uint64_t u = h4(seed, src, mate, 4 * k + 1) % total;
    uint32_t lo = 0, hi = n_iv;   // interval containing u (upper_bound of cum)
    while (lo < hi) {
      const uint32_t m = (lo + hi) >> 1;
      if (cum[m] <= u) lo = m + 1; else hi = m;
    }
    const Iv v = iv[lo < n_iv ? lo : n_iv - 1];
    const uint64_t span = v.b - v.a > seglen ? v.b - v.a - seglen : 1;
    const uint64_t S = v.a + uint64_t(unit(h4(seed, src, mate, 4 * k + 2)) * double(span));
    const bool rc = h4(seed, src, mate, 4 * k + 3) & 1;
    const uint64_t base = rc ? v.rc_end - S - seglen : v.fwd_base + S;
    for (uint32_t j = 0; j < seglen && pos < L; ++j, ++pos) {
      uint8_t c = text[base + j];
      const uint64_t hm = h4(seed ^ 0x5B, src, mate, pos);
      if (unit(hm) < 0.01) {   // substitution to one of the other three bases
        const uint32_t ci = c == 'a' ? 0 : c == 'c' ? 1 : c == 'g' ? 2 : 3;
        c = "acgt"[(ci + 1 + uint32_t((hm >> 7) % 3)) & 3];
      }
      o[pos] = c;
    }
  }
  const uint64_t hn = h4(seed ^ 0x4E, src, mate, 0);
  if (unit(hn) < 0.005) o[(hn >> 20) % L] = 'z';
}

}  // namespace

// Pairs [q0, q0 + n_pairs) into d_out[2 * n_pairs * L] (mate 2i = read 1 of
// pair q0 + i).  iv/cum are device arrays (rg_iv_bytes per interval).
extern "C" int rg_generate(const uint8_t *d_text, const void *d_iv, const uint64_t *d_cum,
                           uint32_t n_iv, uint64_t total, uint64_t seed, uint64_t q0,
                           uint64_t n_pairs, uint32_t L, uint8_t *d_out, void *stream) {
  if (!n_pairs) return 0;
  const uint64_t n = 2 * n_pairs;
  k_gen<<<unsigned((n + 255) / 256), 256, 0, static_cast<hipStream_t>(stream)>>>(
      d_text, static_cast<const Iv *>(d_iv), d_cum, n_iv, total, seed, q0, n_pairs, L, d_out);
  return int(hipGetLastError());
}

extern "C" uint32_t rg_iv_bytes(void) { return sizeof(Iv); }

// Host side: pairs [0, n_pairs) of h_reads (prepared bytes, as rg_generate
// writes them) as two FASTQ files (read 1, read 2) with names r<q0 + i>
// zero-padded to 12 digits (already in samtools sort -n order), bases upper
// case with 'z' -> 'N' (what ingest's replaceN + lowercasing turns back into
// the same bytes), qualities 'I'.  gz: gzip level 1, else plain.  0 = ok.
// one mate's records of pairs [i0, i1) (names r%012llu/<mate>, fixed width:
// every record is 2L + 21 bytes) formatted into out
static void rg_format(const uint8_t *h_reads, uint64_t i0, uint64_t i1, uint32_t L, uint64_t q0,
                      int mate, char *out) {
  char *o = out;
  for (uint64_t i = i0; i < i1; ++i) {
    o += snprintf(o, 20, "@r%012llu/%d\n", (unsigned long long)(q0 + i), mate + 1);
    const uint8_t *r = h_reads + (2 * i + mate) * L;
    for (uint32_t j = 0; j < L; ++j) o[j] = r[j] == 'z' ? 'N' : char(r[j] - 32);
    o += L;
    *o++ = '\n';
    *o++ = '+';
    *o++ = '\n';
    memset(o, 'I', L);
    o += L;
    *o++ = '\n';
  }
}

// pairs [0, n) split into `lanes` consecutive lane files per mate
// (path1[k] / path2[k]), gzip (level 1) or plain; every file on its own
// thread, plain files formatted in parallel slices
extern "C" int rg_write_fastq_lanes(const uint8_t *h_reads, uint64_t n_pairs, uint32_t L,
                                    uint64_t q0, uint32_t lanes, const char *const *path1,
                                    const char *const *path2, int gz) {
  const uint64_t rec = 2ull * L + 21;
  std::vector<int> rc(2 * lanes, 0);
  std::vector<std::thread> th;
  for (uint32_t k = 0; k < lanes; ++k)
    for (int mate = 0; mate < 2; ++mate)
      th.emplace_back([&, k, mate] {
        const uint64_t i0 = n_pairs * k / lanes, i1 = n_pairs * (k + 1) / lanes;
        const char *path = mate ? path2[k] : path1[k];
        std::vector<char> out(size_t((i1 - i0) * rec) + 32);
        // format in 8 slices (plain files of one lane are large)
        std::vector<std::thread> fs;
        const uint32_t S = 8;
        for (uint32_t t = 0; t < S; ++t)
          fs.emplace_back([&, t] {
            const uint64_t a = i0 + (i1 - i0) * t / S, b = i0 + (i1 - i0) * (t + 1) / S;
            rg_format(h_reads, a, b, L, q0, mate, out.data() + (a - i0) * rec);
          });
        for (auto &x : fs) x.join();
        const size_t bytes = size_t((i1 - i0) * rec);
        int &r = rc[2 * k + mate];
        if (gz) {
          gzFile f = gzopen(path, "wb1");
          if (!f) { r = 1; return; }
          size_t o = 0;
          while (o < bytes) {
            const unsigned c = unsigned(std::min<size_t>(bytes - o, size_t(1) << 30));
            if (gzwrite(f, out.data() + o, c) != int(c)) { r = 2; break; }
            o += c;
          }
          if (gzclose(f) != Z_OK) r = 3;
        } else {
          FILE *f = fopen(path, "wb");
          if (!f) { r = 1; return; }
          const bool ok = fwrite(out.data(), 1, bytes, f) == bytes;
          if (fclose(f) != 0 || !ok) r = 2;
        }
      });
  for (auto &x : th) x.join();
  for (int r : rc)
    if (r) return r;
  return 0;
}

extern "C" int rg_write_fastq(const uint8_t *h_reads, uint64_t n_pairs, uint32_t L, uint64_t q0,
                              const char *path1, const char *path2, int gz) {
  return rg_write_fastq_lanes(h_reads, n_pairs, L, q0, 1, &path1, &path2, gz);
}
