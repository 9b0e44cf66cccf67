#!/bin/bash
# tools/make_golden_r03.sh -- round-3 fixtures from the UPSTREAM reference for
# `mummer` WITHOUT -rcref (the forward-only text layout, fasta.cpp:160-169)
# (dev container only: needs oracle/_ref built by `make -C oracle ref`).
# Inputs are committed fixtures (tiny.fa.gz, s100/s150 fastqs_to_sam output);
# everything written is DATA.
#
#   1. rc0 cache files of the tiny genome: `mummer tiny.fa dummy`
#      -> tests/golden/tiny_index_rc0.sha256
#   2. chr1 alone (tiny.fa up to its second '>' line, one contig: the
#      reference's MemSam map steps over the contigs by 2 even without -rcref,
#      query.cpp:547-551, so a samout run on more contigs ends in "map::at"):
#      -samout lines of s150 (MAM), the first 60 of s100 (-maxmatch) and the
#      first 300 of s100 (-mum), sorted full lines
#      -> {tag}_fwd_full.txt.gz, and the header -> tiny_chr1_fwd_mapout_header.txt
#   3. the same s150 run on all of tiny.fa: exit status and stderr
#      -> tiny_fwd_samout_error.txt
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
R=$ROOT/oracle/_ref
OUT=$ROOT/tests/golden
W=$(mktemp -d /tmp/golden3.XXXXXX)
trap 'rm -rf "$W"' EXIT
make -s -C "$ROOT/oracle" ref
cd "$W"
gzip -dc "$OUT/tiny.fa.gz" > tiny.fa
awk '/^>/{n++} n<2' tiny.fa > chr1.fa

# 1.
"$R/mummer" tiny.fa dummy > /dev/null 2>&1 || true
{
  for f in rc0.ref.bin rc0.ref.seq.bin rc0.i4.index.bin rc0.i4.index.sa.bin \
           rc0.i4.index.isa.bin rc0.i4.index.lcp.vec.bin rc0.i4.index.lcp.m.bin; do
    echo "$f $(sha256sum tiny.fa.bin/$f | cut -d' ' -f1) $(stat -c %s tiny.fa.bin/$f)"
  done
  # item_t{size_t idx; ANINT val} (longSA.h:19-28): the 4 i4 padding bytes
  # are uninitialised upstream, so the pin is on the masked words
  python3 -c "import hashlib,numpy as n,sys; m=n.fromfile(sys.argv[1],n.uint64).reshape(-1,2).copy(); m[:,1]&=0xFFFFFFFF; print('rc0.i4.index.lcp.m.bin:masked', hashlib.sha256(m.tobytes()).hexdigest(), m.nbytes)" tiny.fa.bin/rc0.i4.index.lcp.m.bin
} > "$OUT/tiny_index_rc0.sha256"

# 2.
Q="python3 $ROOT/tools/golden_queries.py"
gzip -dc "$OUT/s150_fastqs_to_sam.sam.gz" > s150.sam
$Q "$OUT/s100_fastqs_to_sam.sam.gz" sam q300.sam 300
$Q "$OUT/s100_fastqs_to_sam.sam.gz" sam q60.sam 60
run() {   # $1 = output tag, rest = mummer arguments
  local tag=$1; shift
  rm -rf mapout
  "$R/mummer" "$@" 2> /dev/null
  cat mapout/*.txt | grep -v '^@' | LC_ALL=C sort > $tag.txt
  gzip -9 -n -c $tag.txt > "$OUT/$tag.txt.gz"
}
run s150_chr1_mapout_fwd_full -qthreads 2 -nomap -samin -samout chr1.fa s150.sam
cat mapout/*.txt | grep '^@' | LC_ALL=C sort -u > "$OUT/tiny_chr1_fwd_mapout_header.txt"
run s100_60_chr1_mapout_MEM_fwd_full -qthreads 2 -maxmatch -nomap -samin -samout chr1.fa q60.sam
run s100_300_chr1_mapout_MUM_fwd_full -qthreads 2 -mum -samin -samout chr1.fa q300.sam

# 3.
rm -rf mapout
set +e
"$R/mummer" -qthreads 2 -nomap -samin -samout tiny.fa s150.sam > /dev/null 2> err.txt
rc=$?
set -e
{ echo "exit $rc"; cat err.txt; } > "$OUT/tiny_fwd_samout_error.txt"
echo "round-3 golden written to $OUT"
