// smash-paper_amd/cli/fastqs_to_sam.cpp -- `fastqs_to_sam fq1 fq2 [replaceN]`,
// the ingest CLI of the SMASH chain (smash_mapping.sh:19), byte-compatible
// with the reference's (fastqs_to_sam.cpp:29-111): both FASTQs are read in
// lock step, one unmapped SAM line per non-empty record, flag 77 for read 1
// and 141 for read 2, the second header token as XO:Z:, N -> Z in the bases
// when a third argument is given.  '>' records (FASTA) reuse the bases as
// qualities.  Host-only (it feeds `smash_cli.py map --sam` or the reference's
// mummer -samin).
#include <cstdio>
#include <cstring>
#include <string>

namespace {

struct In {
  FILE *f;
  int peek_skip_ws() {   // operator>>(char&): skip whitespace, read one char
    int c;
    do c = std::fgetc(f); while (c != EOF && (c == ' ' || c == '\t' || c == '\n' || c == '\r' ||
                                              c == '\v' || c == '\f'));
    return c;
  }
  bool getline(std::string &s) {
    s.clear();
    int c;
    bool any = false;
    while ((c = std::fgetc(f)) != EOF) {
      any = true;
      if (c == '\n') return true;
      s.push_back(char(c));
    }
    return any;
  }
};

bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }

// first and second whitespace-separated tokens (istringstream >> string)
void tokens(const std::string &line, std::string &a, std::string &b) {
  size_t i = 0, n = line.size();
  auto next = [&](std::string &t) {
    t.clear();
    while (i < n && is_ws(line[i])) ++i;
    while (i < n && !is_ws(line[i])) t.push_back(line[i++]);
  };
  next(a);
  next(b);
}

int fail(const char *msg, const char *arg = nullptr) {
  std::fprintf(stderr, "paa::Error:\n%s%s%s\n", msg, arg ? " " : "", arg ? arg : "");
  return 1;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc != 3 && argc != 4) return fail("usage: fastqs_to_sam fq1 fq2 [replaceN]");
  FILE *f1 = std::fopen(argv[1], "rb");
  if (!f1) return fail("Could not open fastq file", argv[1]);
  FILE *f2 = std::fopen(argv[2], "rb");
  if (!f2) return fail("Could not open fastq file", argv[2]);
  In in[2] = {{f1}, {f2}};
  bool ok[2] = {true, true};
  std::string line, name, optional, bases, errors;
  char plus = '+';
  while (ok[0] && ok[1]) {
    for (int i = 0; i < 2; ++i) {
      const int amp = in[i].peek_skip_ws();
      if (amp == EOF) { ok[i] = false; break; }
      in[i].getline(line);
      tokens(line, name, optional);
      if (name.empty()) return fail("Problem reading read name");
      in[i].getline(bases);
      if (amp == '@') {
        const int p = in[i].peek_skip_ws();
        plus = p == EOF ? plus : char(p);
        in[i].getline(errors);
        if (!in[i].getline(errors)) errors.clear();
      } else {
        errors = bases;
      }
      if (argc == 4)
        for (char &c : bases)
          if (c == 'N') c = 'Z';
      if (plus != '+') return fail("Fastq + parse error");
      if (amp != '@' && amp != '>') return fail("Fastq @ parse error");
      if (!bases.empty()) {
        std::printf("%s\t%d\t*\t0\t0\t*\t*\t0\t0\t%s\t%s", name.c_str(), i ? 141 : 77,
                    bases.c_str(), errors.c_str());
        if (!optional.empty()) std::printf("\tXO:Z:%s", optional.c_str());
        std::putchar('\n');
      }
    }
  }
  return 0;
}
