// oracle/ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (dev container).
//
// A small driver written for this repo that links against the UPSTREAM
// reference objects (built by oracle/Makefile from /root/reference, never
// copied here) and prints the raw match triples that longSA::MAM / MEM / MUM
// (longSA.cpp:503, 587, 549) push through Aligner::process_match
// (query.cpp:436).  These triples are the per-read golden vectors for the
// device search kernel (SURVEY.md §4 "recommended per-read golden-vector
// generator").
//
// usage: mam_harness <ref.fa> <reads.txt> [MAM|MEM|MUM] [min_len]
//   reads.txt: one read per line (raw bases; lowercased exactly like
//   NewQuery::extend, query.cpp:125-144, i.e. spaces skipped).
// output, one line per read:  <read_idx> <n> ref,qoff,len ref,qoff,len ...
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "longSA.h"
#include "query.h"

// longSA.h:104 declares `friend class Args` on SAArgs; this is our own Args.
class Args {
 public:
  static void configure(SAArgs &a, const char *fasta) {
    a.ref_args.ref_fasta = fasta;
    a.ref_args.rcref = true;
  }
};

int main(int argc, char **argv) {
  if (argc < 3) {
    std::cerr << "usage: mam_harness ref.fa reads.txt [MAM|MEM|MUM] [min_len]\n";
    return 2;
  }
  SAArgs sargs;
  Args::configure(sargs, argv[1]);
  const longSA sa(sargs);
  AlignerArgs aargs;
  if (argc > 3) {
    if (!strcmp(argv[3], "MEM")) aargs.type = MEM;
    else if (!strcmp(argv[3], "MUM")) aargs.type = MUM;
    else aargs.type = MAM;
  }
  if (argc > 4) aargs.min_len = atoi(argv[4]);
  Aligner al(aargs, sa);
  std::ifstream in(argv[2]);
  std::string line;
  uint64_t idx = 0;
  std::vector<match_t> m;
  while (std::getline(in, line)) {
    std::string q;
    uint64_t end = line.size();
    while (end && line[end - 1] == ' ') --end;
    for (uint64_t i = 0; i != end; ++i) {
      if (line[i] == ' ') continue;
      q.push_back(static_cast<char>(tolower(line[i])));
    }
    al.query = q;
    if (aargs.type == MAM) sa.MAM(al);
    else if (aargs.type == MUM) sa.MUM(al);
    else sa.MEM(al);
    m.clear();
    al.forget(m);
    std::printf("%llu %zu", (unsigned long long)idx, m.size());
    for (const auto &x : m)
      std::printf(" %llu,%llu,%llu", (unsigned long long)x.ref,
                  (unsigned long long)x.query, (unsigned long long)x.len);
    std::printf("\n");
    ++idx;
  }
  return 0;
}
