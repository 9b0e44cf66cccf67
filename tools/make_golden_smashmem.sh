#!/bin/bash
# tools/make_golden_smashmem.sh -- goldens of the REFERENCE's smashMEM.py
# (dev container only: reads /root/reference; writes DATA to tests/golden).
#
# pysam is absent, so tools/pysam_shim (a SAM-text stand-in for the pysam 0.8
# calls the script makes) is put first on PYTHONPATH and smashMEM.py runs
# unmodified, as smash_mapping.sh:26 runs it (args 0 0 10000 4), on:
#   * {s100,s150}: the reference's own tagged mapout of the golden reads
#     (tests/golden/{s}_mapout_tagged_full.txt.gz, smash_mapping.sh:19-23)
#     with the mapout header, records in samtools sort -n order (fixed-width
#     names; read 1 before read 2; stable otherwise);
#   * edge: tools/smashmem_edge.py's hand-made tagged SAM (the filters, the
#     hit window, first-wins de-dup, key order, unmapped mates).
# Outputs: tests/golden/{s}_smashmem.txt.gz = the script's whole stdout, and
# the input SAM of the edge case (tests/golden/smashmem_edge.sam).
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REF=${REF:-/root/reference}
OUT=$ROOT/tests/golden
W=$(mktemp -d /tmp/smashmem.XXXXXX)
trap 'rm -rf "$W"' EXIT
export PYTHONPATH=$ROOT/tools/pysam_shim
for s in s100 s150; do
  python3 - "$OUT/tiny_mapout_header.txt" "$OUT/${s}_mapout_tagged_full.txt.gz" > "$W/$s.sam" <<'PY'
import gzip, sys
head = [l for l in open(sys.argv[1]) if l.startswith("@")]
body = gzip.open(sys.argv[2], "rt").read().splitlines()
# samtools sort -n: name (fixed-width r%09d: plain order), read 1 first
body.sort(key=lambda l: (l.split("\t", 1)[0], 0 if int(l.split("\t")[1]) & 64 else 1))
sys.stdout.write("".join(head) + "\n".join(body) + "\n")
PY
  python3 "$REF/smashMEM.py" "$W/$s.sam" 0 0 10000 4 > "$W/${s}_smashmem.txt"
  gzip -9 -n -c "$W/${s}_smashmem.txt" > "$OUT/${s}_smashmem.txt.gz"
done
python3 "$ROOT/tools/smashmem_edge.py" > "$OUT/smashmem_edge.sam"
python3 "$REF/smashMEM.py" "$OUT/smashmem_edge.sam" 0 0 10000 4 > "$W/edge_smashmem.txt"
gzip -9 -n -c "$W/edge_smashmem.txt" > "$OUT/edge_smashmem.txt.gz"
