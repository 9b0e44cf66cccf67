#!/bin/bash
# tools/make_golden_r02.sh -- round-2 fixtures from the UPSTREAM reference
# (dev container only: needs oracle/_ref built by `make -C oracle ref`).
# Inputs are the committed round-1 fixtures (tiny.fa.gz, s{100,150} reads),
# so nothing already committed changes.  Everything written is DATA.
#
#   1. rc1.i8 index files of the tiny genome: `mummer-long -rcref tiny.fa
#      dummy` (the 64-bit flavour mummer.cpp:156-183 re-execs for big
#      references) -> tests/golden/tiny_index_i8.sha256
#   2. the FULL mapout lines (SEQ, QUAL, XO:Z kept) of smash_mapping.sh:19-23
#      as written: `mummer -verbose -rcref -qthreads 12 -nomap -samin
#      -samout` on fastqs_to_sam output, then mappability_tag on the header
#      (head -n 100) + the perl-munged body -> {s}_mapout_full.txt.gz (sorted)
#      and {s}_mapout_tagged_full.txt.gz (sorted)
set -eu   # (no pipefail: `head` closes its pipe early by design)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
R=$ROOT/oracle/_ref
OUT=$ROOT/tests/golden
W=$(mktemp -d /tmp/golden2.XXXXXX)
trap 'rm -rf "$W"' EXIT
make -s -C "$ROOT/oracle" ref
cd "$W"
gzip -dc "$OUT/tiny.fa.gz" > tiny.fa

# 1. rc1.i8
mkdir i8 && cp tiny.fa i8/
(cd i8 && "$R/mummer-long" -rcref tiny.fa dummy > /dev/null 2>&1 || true)
{
  for f in rc1.i8.index.bin rc1.i8.index.sa.bin rc1.i8.index.isa.bin \
           rc1.i8.index.lcp.vec.bin rc1.i8.index.lcp.m.bin; do
    echo "$f $(sha256sum i8/tiny.fa.bin/$f | cut -d' ' -f1) $(stat -c %s i8/tiny.fa.bin/$f)"
  done
} > "$OUT/tiny_index_i8.sha256"

# 2. smash_mapping.sh:19-23 lines as written (minus samtools, absent here)
"$R/mummer" -rcref tiny.fa dummy > /dev/null 2>&1 || true
"$R/mummer" -rcref -mappability tiny.fa tiny.fa.bin/map.bin > /dev/null 2>&1
cp "$OUT/tiny_sam_header.txt" tiny.fa.bin/sam_header.txt     # index_setup.sh:31
cp "$OUT/tiny_chrom_sizes.txt" tiny.fa.bin/chrom_sizes.txt   # index_setup.sh:28
for s in s100 s150; do
  gzip -dc "$OUT/${s}_fastqs_to_sam.sam.gz" > $s.sam
  rm -rf mapout
  "$R/mummer" -verbose -rcref -qthreads 12 -nomap -samin -samout tiny.fa $s.sam 2> /dev/null
  cat mapout/*.txt | grep -v '^@' | LC_ALL=C sort > ${s}_mapout_full.txt
  "$R/mappability_tag" tiny.fa <(cat mapout/*.txt | head -n 100 | grep ^@ ;
                                 cat mapout/*.txt | grep -v ^@ | perl -pe 's/^(\S+?)\/\S+\/\d+/\1/') \
    | grep -v '^@' | LC_ALL=C sort > ${s}_mapout_tagged_full.txt
  gzip -9 -n -c ${s}_mapout_full.txt > "$OUT/${s}_mapout_full.txt.gz"
  gzip -9 -n -c ${s}_mapout_tagged_full.txt > "$OUT/${s}_mapout_tagged_full.txt.gz"
done
# the mapout header (fasta.cpp:243-252) of one output file
cat mapout/*.txt | grep '^@' | LC_ALL=C sort -u > "$OUT/tiny_mapout_header.txt"

# 3. the other query formats and search modes through -samout (the drop-in
#    CLI's other paths): FASTQ (-fastq) and FASTA input of s150, and -maxmatch
#    / -mum on the first 60 / 300 records of s100 (sorted full lines)
Q="python3 $ROOT/tools/golden_queries.py"
$Q "$OUT/s150_fastqs_to_sam.sam.gz" fastq q.fq
$Q "$OUT/s150_fastqs_to_sam.sam.gz" fasta q.fa
$Q "$OUT/s100_fastqs_to_sam.sam.gz" sam q300.sam 300
$Q "$OUT/s100_fastqs_to_sam.sam.gz" sam q60.sam 60
run() {   # $1 = output tag, rest = mummer arguments
  local tag=$1; shift
  rm -rf mapout
  "$R/mummer" "$@" 2> /dev/null
  cat mapout/*.txt | grep -v '^@' | LC_ALL=C sort > $tag.txt
  gzip -9 -n -c $tag.txt > "$OUT/$tag.txt.gz"
}
run s150_mapout_fastq_full -rcref -qthreads 2 -fastq -nomap -samout tiny.fa q.fq
run s150_mapout_fasta_full -rcref -qthreads 2 -nomap -samout tiny.fa q.fa
run s100_60_mapout_MEM_full -rcref -qthreads 2 -maxmatch -nomap -samin -samout tiny.fa q60.sam
run s100_300_mapout_MUM_full -rcref -qthreads 2 -mum -samin -samout tiny.fa q300.sam
# (mummer without -samout writes only the header: print_matches' non-SAM
# branch, query.cpp:404-412, never calls OutputSorter::end_line, so its
# lines are dropped; nothing to record)
echo "round-2 golden written to $OUT"
