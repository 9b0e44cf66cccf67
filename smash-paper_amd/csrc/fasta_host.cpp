// smash-paper_amd/csrc/fasta_host.cpp -- host-side reference text builder.
//
// Sequence::Sequence (fasta.cpp:133-285).  With -rcref: per contig the
// lowercased forward sequence, '`', its reverse complement (the IUPAC map of
// reverse_complement, fasta.cpp:26-61), '`' between contigs, one final '$'.
// Without it (fasta.cpp:165-168): c1 ` c2 ` ... cn $, one entry per contig.
// Line handling follows std::getline + trim (fasta.cpp:107-124,195-246),
// including the eof-without-newline behaviour.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/smash_gpu.h"

namespace smash { void set_error(const std::string &msg); }

namespace {
unsigned char comp(unsigned char c) {
  static unsigned char t[256];
  static bool init = false;
  if (!init) {
    for (int i = 0; i < 256; ++i) t[i] = (unsigned char)i;
    const char *a = "acgtrymkbdhvACGTRYMKBDHV", *b = "tgcayrkmvhdbTGCAYRKMVHDB";
    for (int i = 0; a[i]; ++i) t[(unsigned char)a[i]] = (unsigned char)b[i];
    init = true;
  }
  return t[c];
}
}  // namespace

extern "C" int smash_text_from_fasta_layout(const char *path, int rcref, uint8_t **text,
                                            uint64_t *N, uint32_t *n_seq, uint64_t **startpos,
                                            uint64_t **sizes, char ***names) {
  if (!path || !text || !N || !n_seq || !startpos || !sizes || !names) {
    smash::set_error("smash_text_from_fasta: bad arguments");
    return SMASH_ERR_ARG;
  }
  FILE *f = fopen(path, "rb");
  if (!f) {
    smash::set_error(std::string("cannot open ") + path);
    return SMASH_ERR_IO;
  }
  std::vector<char> buf;
  {
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    buf.resize(size_t(n));
    if (n && fread(buf.data(), 1, size_t(n), f) != size_t(n)) {
      fclose(f);
      smash::set_error("short read");
      return SMASH_ERR_IO;
    }
    fclose(f);
  }
  std::vector<uint8_t> seq;
  std::vector<uint64_t> sp{0}, sz;
  std::vector<std::string> descr;
  std::string meta;
  uint64_t length = 0;
  size_t pos = 0;
  const size_t fsz = buf.size();
  bool eof = false;
  while (!eof) {
    size_t a = pos, b;
    if (pos >= fsz) { b = pos; eof = true; }
    else {
      const char *nl = static_cast<const char *>(memchr(buf.data() + pos, '\n', fsz - pos));
      if (nl) { b = size_t(nl - buf.data()); pos = b + 1; }
      else { b = fsz; pos = fsz; eof = true; }
    }
    const char *line = buf.data() + a;
    const size_t lsz = b - a;
    if (!eof && lsz == 0) continue;
    size_t start = 0, end = lsz;
    const char c0 = lsz ? line[0] : 0;
    if (eof || c0 == '>') {
      if (length > 0) {
        const uint64_t this_start = sp.back();
        descr.push_back(meta);
        if (rcref || !eof) {
          seq.push_back('`');
          sp.push_back(seq.size());
        }
        sz.push_back(length);
        if (rcref) {
          descr.push_back(meta);
          sz.push_back(length);
          for (uint64_t k = 0; k < length; ++k)
            seq.push_back(comp(seq[this_start + length - 1 - k]));
          if (!eof) {
            seq.push_back('`');
            sp.push_back(seq.size());
          }
        }
        if (eof) break;
      }
      start = 1;
      meta.clear();
      length = 0;
    }
    for (size_t i = start; i < lsz; ++i)
      if (line[i] != ' ') { start = i; break; }
    for (size_t i = lsz; i != 1 && i != 0; --i)
      if (line[i - 1] != ' ') { end = i; break; }
    if (c0 == '>') {
      for (size_t i = start; i != end; ++i) {
        if (line[i] == ' ') break;
        meta += line[i];
      }
    } else {
      length += end - start;
      for (size_t i = start; i != end; ++i) {
        unsigned char ch = (unsigned char)line[i];
        seq.push_back((ch >= 'A' && ch <= 'Z') ? ch + 32 : ch);
      }
    }
  }
  seq.push_back('$');
  const uint32_t ns = uint32_t(sz.size());
  *N = seq.size();
  *text = static_cast<uint8_t *>(malloc(seq.size()));
  memcpy(*text, seq.data(), seq.size());
  *n_seq = ns;
  *startpos = static_cast<uint64_t *>(malloc(8 * (ns ? ns : 1)));
  *sizes = static_cast<uint64_t *>(malloc(8 * (ns ? ns : 1)));
  *names = static_cast<char **>(malloc(sizeof(char *) * (ns ? ns : 1)));
  for (uint32_t i = 0; i < ns; ++i) {
    (*startpos)[i] = sp[i];
    (*sizes)[i] = sz[i];
    (*names)[i] = strdup(descr[i].c_str());
  }
  return SMASH_OK;
}

extern "C" int smash_text_from_fasta(const char *path, uint8_t **text, uint64_t *N,
                                     uint32_t *n_seq, uint64_t **startpos,
                                     uint64_t **sizes, char ***names) {
  return smash_text_from_fasta_layout(path, 1, text, N, n_seq, startpos, sizes, names);
}

extern "C" void smash_text_free(uint8_t *text, uint32_t n_seq, uint64_t *startpos,
                                uint64_t *sizes, char **names) {
  free(text);
  free(startpos);
  free(sizes);
  if (names)
    for (uint32_t i = 0; i < n_seq; ++i) free(names[i]);
  free(names);
}
