// smash-paper_amd/cli/mappability_tag.cpp -- the reference's
// `mappability_tag REF.fa in.sam` (mappability_tag.cpp:53-127), host code:
// SAM lines through to stdout, each mapped line followed by L<i>/R<i> tags
// (i < 10) of its '=' CIGAR blocks from REF.fa.bin/map.bin, with the
// contig offsets of REF.fa.bin/sam_header.txt (ChromosomeInfo,
// chromosomes.h:23-59; u32 arithmetic as the reference's unsigned int).
// Errors as the reference: the message on stderr, exit status 1, the output
// up to the offending line already written.
//
// The same tags are produced on the device for the count path (k_post_fast /
// k_post, smash_sam_records); this is the stream tool the scripts call.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

struct Fail : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// map.bin, memory-mapped (util.h:131-149 Mappability over MappedFile)
class Map {
 public:
  explicit Map(const std::string &path) {
    fd_ = open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw Fail("could not open " + path);
    struct stat st;
    fstat(fd_, &st);
    size_ = uint64_t(st.st_size);
    if (size_) {
      data_ = static_cast<const uint8_t *>(mmap(nullptr, size_, PROT_READ, MAP_SHARED, fd_, 0));
      if (data_ == MAP_FAILED) throw Fail("could not map " + path);
    }
  }
  ~Map() {
    if (data_ && data_ != MAP_FAILED) munmap(const_cast<uint8_t *>(data_), size_);
    if (fd_ >= 0) close(fd_);
  }
  // bytes past the end of the file read 0 (the rest of the last mmap page)
  unsigned at(uint64_t k) const { return k < size_ ? data_[k] : 0u; }
  unsigned left(unsigned n) const { return at(2 + uint64_t(n) * 2); }
  unsigned right(unsigned n) const { return at(2 + uint64_t(n) * 2 + 1); }

 private:
  int fd_ = -1;
  const uint8_t *data_ = nullptr;
  uint64_t size_ = 0;
};

// ChromosomeInfo(sam_header.txt): @SQ SN/LN lines, cumulative u32 offsets
std::map<std::string, unsigned> read_offsets(const std::string &path) {
  std::ifstream in(path);
  if (!in) throw Fail("Problem opening sam file " + path);
  if (in.peek() != '@') throw Fail("Is the sam header missing? " + path);
  std::map<std::string, unsigned> off;
  unsigned o = 0;
  unsigned n = 0;
  std::string line;
  while (in.peek() == '@' && std::getline(in, line)) {
    if (line.compare(0, 7, "@SQ\tSN:") != 0) continue;
    const size_t t = line.find('\t', 7);
    if (t == std::string::npos || line.compare(t, 4, "\tLN:") != 0)
      throw Fail("Parse Problem read_this LN:");
    const std::string name = line.substr(7, t - 7);
    const unsigned len = unsigned(std::stoul(line.substr(t + 4)));
    off[name] = o;
    o += len;
    ++n;
  }
  off["*"] = o;   // lookup["*"] = names.size(): never read for a '*' CIGAR
  return off;
}

int run(int argc, char **argv) {
  if (argc - 1 != 2) throw Fail("usage: mappability_tag fasta_file in.sam");
  const std::string ref = argv[1];
  const Map map(ref + ".bin/map.bin");
  const auto offsets = read_offsets(ref + ".bin/sam_header.txt");
  std::ifstream input(argv[2]);
  if (!input) throw Fail(std::string("Could not open smash sam file") + argv[2]);
  std::ios::sync_with_stdio(false);
  std::string line;
  while (std::getline(input, line)) {
    if (!line.empty() && line[0] == '@') {
      std::cout << line << '\n';
      continue;
    }
    std::istringstream ls(line);
    std::string name, chr, cigar;
    int flag = 0, qual = 0;
    uint32_t pos = 0;
    ls >> name >> flag >> chr >> pos >> qual >> cigar;
    const bool small_chr =
        chr.find("_gl000") != std::string::npos || chr.find("chrM") != std::string::npos;
    std::cout << line;
    if (!ls) std::cerr << "parse error";
    std::string optional;
    const auto c = offsets.find(chr);   // all_chr.abspos before the CIGAR test
    if (c == offsets.end()) {
      std::cout.flush();
      throw Fail("Unknown chromosome" + chr);
    }
    const unsigned abspos = c->second + pos;
    if (cigar != "*") {
      std::istringstream cs(cigar);
      uint32_t count = 0;
      char code = 0;
      int offset = 0, uindex = 0;
      while (cs >> count >> code) {
        if (code == '=') {
          const unsigned left_m = map.left(abspos + unsigned(offset) + count - 1);
          const unsigned left = left_m ? left_m - 1 : 255;
          const unsigned right_m = map.right(abspos + unsigned(offset) - 1);
          const unsigned right = right_m ? right_m : 255;
          if (uindex < 10)
            optional += "\tL" + std::to_string(uindex) + ":i:" + std::to_string(left) + "\tR" +
                        std::to_string(uindex) + ":i:" + std::to_string(right);
          if (left > count && !small_chr) {
            std::cout.flush();
            std::cerr << left_m << " " << right_m << " " << line << '\t' << optional << std::endl;
            throw Fail("left mappability too big" + std::to_string(left));
          }
          if (right > count && !small_chr) {
            std::cout.flush();
            throw Fail("right mappability too big" + std::to_string(right));
          }
          ++uindex;
        } else if (code != 'S' && code != 'M') {
          std::cout.flush();
          throw Fail(std::string("unexpected cigar") + code);
        }
        offset += int(count);
      }
    }
    std::cout << optional << '\n';
  }
  std::cout.flush();
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  try {
    return run(argc, argv);
  } catch (std::exception &e) {
    std::cerr << e.what() << std::endl;
    return 1;
  }
}
