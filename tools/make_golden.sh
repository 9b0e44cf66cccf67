#!/bin/bash
# tools/make_golden.sh -- regenerate tests/golden/ from the UPSTREAM reference.
#
# Dev container only (needs /root/reference and oracle/_ref built by
# `make -C oracle ref`).  Everything written to tests/golden/ is DATA (inputs
# and the reference's outputs); no reference source is copied.
#
#   1. tiny synthetic genome + SMASH reads          (tools/synth.py)
#   2. index: mummer -rcref ref dummy                (index_setup.sh:19)
#   3. map.bin: mummer -rcref -mappability           (index_setup.sh:22)
#   4. fastqs_to_sam r1 r2 1                         (smash_mapping.sh:19)
#   5. mummer -rcref -qthreads 2 -nomap -samin -samout  -> mapout/*.txt
#   6. mappability_tag                               (smash_mapping.sh:23)
#   7. raw MAM/MEM/MUM triples                       (oracle/_ref/mam_harness)
#   8. varbin.py (python3) on positions from the oracle's smashMEM
#      restatement and on a hand-made edge-case positions file.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REF=${REF:-/root/reference}
R=$ROOT/oracle/_ref
OUT=$ROOT/tests/golden
W=$(mktemp -d /tmp/golden.XXXXXX)
trap 'rm -rf "$W"' EXIT
make -s -C "$ROOT/oracle" ref oracle
mkdir -p "$OUT"
cd "$W"

python3 - <<EOF
import sys; sys.path.insert(0, "$ROOT/tools")
import synth
g = synth.make_genome("tiny")
synth.write_fasta("tiny.fa", g)
for tag, n, L, seed in (("s100", 2000, 100, 11), ("s150", 600, 150, 12)):
    r1, r2 = synth.make_reads(g, n, L, seed=seed)
    synth.write_fastq(tag + "_r1.fq", r1, 1)
    synth.write_fastq(tag + "_r2.fq", r2, 2)
synth.write_index_side_files("tiny.fa.bin", g)
synth.make_bins(g, 8, "bins.txt")
EOF

"$R/mummer" -rcref tiny.fa dummy >/dev/null 2>&1 || true
"$R/mummer" -rcref -mappability tiny.fa tiny.fa.bin/map.bin >/dev/null 2>&1

{
  for f in rc1.ref.seq.bin rc1.ref.bin rc1.i4.index.bin rc1.i4.index.sa.bin \
           rc1.i4.index.isa.bin rc1.i4.index.lcp.vec.bin rc1.i4.index.lcp.m.bin; do
    echo "$f $(sha256sum tiny.fa.bin/$f | cut -d' ' -f1) $(stat -c %s tiny.fa.bin/$f)"
  done
  # item_t{size_t idx; uint32 val} has 4 uninitialised padding bytes
  # (longSA.h:19-28): hash the (idx,val) content with the padding masked.
  python3 -c "
import hashlib, numpy as np
m = np.fromfile('tiny.fa.bin/rc1.i4.index.lcp.m.bin', np.uint64).reshape(-1, 2).copy()
m[:, 1] &= 0xFFFFFFFF
print('rc1.i4.index.lcp.m.bin:masked', hashlib.sha256(m.tobytes()).hexdigest(), m.size * 8)"
  echo "map.bin[2:] $(tail -c +3 tiny.fa.bin/map.bin | sha256sum | cut -d' ' -f1) $(stat -c %s tiny.fa.bin/map.bin)"
} > "$OUT/tiny_index.sha256"

for s in s100 s150; do
  "$R/fastqs_to_sam" ${s}_r1.fq ${s}_r2.fq 1 > $s.sam
  rm -rf mapout
  "$R/mummer" -rcref -qthreads 2 -nomap -samin -samout tiny.fa $s.sam 2>/dev/null
  cat mapout/*.txt | grep '^@' | sort -u > hdr.txt
  # mapped lines only need name..HI; SEQ/QUAL/XO are the inputs themselves
  cat mapout/*.txt | grep -v '^@' > body.sam
  "$R/mappability_tag" tiny.fa <(head -100 hdr.txt; cat body.sam) > tagged.sam
  grep -v '^@' tagged.sam \
    | awk -F'\t' 'BEGIN{OFS="\t"} {t=""; for(i=12;i<=NF;i++){ if($i ~ /^(XM|XU|XE|XS|NH|HI|L0|R0|cc|cp|xo|xc|CC|CP|XO|XC):/) t=t"\t"$i } print $1,$2,$3,$4,$5,$6,$7,$8,$9 t}' \
    | LC_ALL=C sort > ${s}_mapout_tagged.txt
  awk -F'\t' '{print tolower($10)}' $s.sam > ${s}_reads.txt
  head -300 ${s}_reads.txt > ${s}_reads300.txt
  for mode in MAM MUM; do
    "$R/mam_harness" tiny.fa ${s}_reads.txt $mode > ${s}_${mode}.txt
  done
  # -maxmatch output is large (repeats): first 300 reads only
  "$R/mam_harness" tiny.fa ${s}_reads300.txt MEM > ${s}_MEM.txt
  gzip -9 -n -c ${s}_mapout_tagged.txt > "$OUT/${s}_mapout_tagged.txt.gz"
  for mode in MAM MEM MUM; do gzip -9 -n -c ${s}_${mode}.txt > "$OUT/${s}_${mode}.txt.gz"; done
  gzip -9 -n -c ${s}_r1.fq > "$OUT/${s}_r1.fq.gz"
  gzip -9 -n -c ${s}_r2.fq > "$OUT/${s}_r2.fq.gz"
  gzip -9 -n -c $s.sam > "$OUT/${s}_fastqs_to_sam.sam.gz"
done
gzip -9 -n -c tiny.fa > "$OUT/tiny.fa.gz"
cp tiny.fa.bin/chrom_sizes.txt "$OUT/tiny_chrom_sizes.txt"
cp tiny.fa.bin/sam_header.txt "$OUT/tiny_sam_header.txt"
cp bins.txt "$OUT/tiny_bins.txt"

# positions through the oracle's smashMEM restatement (pysam is absent, so
# smashMEM.py itself cannot run: this link is parity-unpinned), then the
# REAL varbin.py on them.  varbin.py crashes at its median line under python3
# (varbin.py:113) after writing every bin row; its exit code is ignored.
for s in s100 s150; do
  python3 "$ROOT/tools/oracle_positions.py" tiny.fa ${s}_mapout_tagged.txt \
      tiny.fa.bin/chrom_sizes.txt > ${s}_positions.txt
  python3 "$REF/varbin.py" ${s}_positions.txt bins.txt ${s}_varbin.txt \
      ${s}_stats.txt tiny.fa.bin/chrom_sizes.txt > /dev/null 2>&1 || true
  cp ${s}_positions.txt "$OUT/${s}_positions.txt"
  cp ${s}_varbin.txt "$OUT/${s}_varbin.txt"
  cp ${s}_stats.txt "$OUT/${s}_varbin_stats_partial.txt"
done

# varbin quirk fixture: hg19 bins, hand-made positions (adjacent dups across
# chromosomes, chrM/_ skips, a position before the first bin start).
python3 - <<'EOF' > edge_positions.txt
rows = [("chr1", 5), ("chr1", 5), ("chr2", 5), ("chrM", 7), ("chr1_gl000191_random", 9),
        ("chr1", 100), ("chr3", 100), ("chr1", 100), ("chrX", 155270559), ("chrY", 0),
        ("chr22", 51304565), ("chr9", 46757576), ("chr9", 46757575), ("chrUn", 4),
        ("chr1", 0), ("chr1", 0), ("chr21", 9849871), ("chr21", 9849872), ("", 3)]
for c, p in rows:
    print(c, p)
EOF
python3 - <<EOF > chrom_sizes_hg19.txt
import sys; sys.path.insert(0, "$ROOT/tools")
import synth
n = 0
for name, L in synth.hg19_lengths() + [("chrM", 16571)]:
    print("%s\t%d\t%d" % (name, L, n)); n += L
EOF
# shift chr1 so that position 0 lands before the first bin start
python3 "$REF/varbin.py" edge_positions.txt "$ROOT/data/bins/50000/bins.txt" edge_varbin.txt \
    edge_stats.txt chrom_sizes_hg19.txt > /dev/null 2>&1 || true
cp edge_positions.txt chrom_sizes_hg19.txt "$OUT/"
gzip -9 -n -c edge_varbin.txt > "$OUT/edge_varbin.txt.gz"
cp edge_stats.txt "$OUT/edge_varbin_stats_partial.txt"
echo "golden written to $OUT"

# fastqs_to_sam parser quirks (blank lines, '+name' lines, an empty record,
# FASTA records whose qualities keep the N): tests/golden/edge_r{1,2}.fq are
# hand-written; the outputs are the reference binary's, with and without
# the replaceN argument.
"$R/fastqs_to_sam" "$OUT/edge_r1.fq" "$OUT/edge_r2.fq" > "$OUT/edge_fastqs_to_sam.sam"
"$R/fastqs_to_sam" "$OUT/edge_r1.fq" "$OUT/edge_r2.fq" 1 > "$OUT/edge_fastqs_to_sam_replaceN.sam"
