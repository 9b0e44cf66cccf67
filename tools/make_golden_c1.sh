#!/bin/bash
# tools/make_golden_c1.sh -- BASELINE config C1 from the UPSTREAM reference
# (dev container only: oracle/_ref built by `make -C oracle ref`):
# "chr21-only reference, 10k synthetic 100 bp reads, CPU memsam + varbin.py
# at sample_bins/500000".  SURVEY.md §8d: the chr21-sized synthetic genome
# (tools/synth.py "chr21", seed 21), 5 000 pairs x 100 bp (seed 1),
# sample_bins/500000 synthesized by splitting every 50 000 bin in 10,
# chrom_sizes with chr21 at its hg19 offset 2 781 598 825.
#
#   index      mummer -rcref (index_setup.sh:19) -> c1_index.sha256 (SA, ISA,
#              LCP, map.bin: the device build must match byte for byte)
#   mapping    fastqs_to_sam | mummer -verbose -rcref -qthreads 12 -nomap
#              -samin -samout | mappability_tag  (smash_mapping.sh:19-23)
#   smashMEM   the REFERENCE's smashMEM.py, unmodified, over tools/pysam_shim
#              (a SAM-text stand-in for its pysam 0.8 calls; round 3), on the
#              tagged SAM in samtools sort -n order, then the awk/perl
#              extraction of smash_mapping.sh:29
#   varbin     the REAL varbin.py (python3) -> c1_varbin_nonzero.txt
#              (bin index, count of every non-empty bin) + c1_varbin_stats.txt
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REF=${REF:-/root/reference}
R=$ROOT/oracle/_ref
OUT=$ROOT/tests/golden
W=$(mktemp -d /tmp/goldenc1.XXXXXX)
trap 'rm -rf "$W"' EXIT
make -s -C "$ROOT/oracle" ref oracle
cd "$W"
python3 - <<EOF
import sys; sys.path.insert(0, "$ROOT/tools")
import synth
g = synth.make_genome("chr21")
synth.write_fasta("chr21.fa", g)
r1, r2 = synth.make_reads(g, 5000, 100, seed=1)
synth.write_fastq("r1.fq", r1, 1)
synth.write_fastq("r2.fq", r2, 2)
synth.split_bins("$ROOT/data/bins/50000/bins.txt", 10, "bins500k.txt")
EOF
"$R/mummer" -rcref chr21.fa dummy > /dev/null 2>&1 || true
"$R/mummer" -rcref -mappability chr21.fa chr21.fa.bin/map.bin > /dev/null 2>&1
printf "@SQ\tSN:chr21\tLN:48129895\n" > chr21.fa.bin/sam_header.txt
printf "chr21\t48129895\t2781598825\n" > chrom_sizes.txt
{
  for f in rc1.ref.seq.bin rc1.i4.index.sa.bin rc1.i4.index.isa.bin rc1.i4.index.lcp.vec.bin; do
    echo "$f $(sha256sum chr21.fa.bin/$f | cut -d' ' -f1) $(stat -c %s chr21.fa.bin/$f)"
  done
  python3 -c "
import hashlib, numpy as np
m = np.fromfile('chr21.fa.bin/rc1.i4.index.lcp.m.bin', np.uint64).reshape(-1, 2).copy()
m[:, 1] &= 0xFFFFFFFF
print('rc1.i4.index.lcp.m.bin:masked', hashlib.sha256(m.tobytes()).hexdigest(), m.size * 8)"
  echo "map.bin[2:] $(tail -c +3 chr21.fa.bin/map.bin | sha256sum | cut -d' ' -f1) $(stat -c %s chr21.fa.bin/map.bin)"
} > "$OUT/c1_index.sha256"
"$R/fastqs_to_sam" r1.fq r2.fq 1 > c1.sam
rm -rf mapout
"$R/mummer" -verbose -rcref -qthreads 12 -nomap -samin -samout chr21.fa c1.sam 2> /dev/null
"$R/mappability_tag" chr21.fa <(cat mapout/*.txt | head -n 100 | grep ^@ ;
                                cat mapout/*.txt | grep -v ^@ | perl -pe 's/^(\S+?)\/\S+\/\d+/\1/') \
  | grep -v '^@' \
  | awk -F'\t' 'BEGIN{OFS="\t"} {t=""; for(i=12;i<=NF;i++){ if($i ~ /^(XM|XU|XE|XS|NH|HI|L0|R0|cc|cp|xo|xc|CC|CP|XO|XC):/) t=t"\t"$i } print $1,$2,$3,$4,$5,$6,$7,$8,$9 t}' \
  | LC_ALL=C sort > tagged.txt
"$R/mappability_tag" chr21.fa <(cat mapout/*.txt | head -n 100 | grep ^@ ;
                                cat mapout/*.txt | grep -v ^@ | perl -pe 's/^(\S+?)\/\S+\/\d+/\1/') \
  > tagged_full.sam
python3 - <<'PY'
lines = open("tagged_full.sam").read().splitlines()
head = [l for l in lines if l.startswith("@")]
body = [l for l in lines if l and not l.startswith("@")]
# samtools sort -n: fixed-width names r%09d (plain order), read 1 first
body.sort(key=lambda l: (l.split("\t", 1)[0], 0 if int(l.split("\t")[1]) & 64 else 1))
open("namesort.sam", "w").write("\n".join(head + body) + "\n")
PY
PYTHONPATH="$ROOT/tools/pysam_shim" python3 "$REF/smashMEM.py" namesort.sam 0 0 10000 4 > smash.txt
cat smash.txt | awk '{print $4, $5}' | perl -ne 'print if /^chr(\d+|[XY]) \d+$/' > positions.txt
python3 "$ROOT/tools/oracle_positions.py" chr21.fa tagged.txt chrom_sizes.txt > positions_oracle.txt
cmp positions.txt positions_oracle.txt   # the restatement agrees at C1 scale
python3 "$REF/varbin.py" positions.txt bins500k.txt varbin.txt stats.txt chrom_sizes.txt \
    > /dev/null 2>&1 || true
awk -F'\t' '$4 != 0 {print NR - 1 "\t" $4}' varbin.txt > "$OUT/c1_varbin_nonzero.txt"
echo "rows $(wc -l < varbin.txt)" >> "$OUT/c1_varbin_nonzero.txt"
cp stats.txt "$OUT/c1_varbin_stats_partial.txt"
echo "C1 golden: $(wc -l < positions.txt) positions, $(wc -l < "$OUT/c1_varbin_nonzero.txt") lines"
